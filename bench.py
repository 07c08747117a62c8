#!/usr/bin/env python3
"""Benchmark: batched pusher-slider NMPC solves/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the configuration the metric is quoted on):
  N = 20, batch = 65 536 lanes per GPU, 4 slider shapes mixed per lane
  (shape_id = lane mod 4: santal/balea/montana/pulirapid), K = 50 SQP-RTI
  (full Gauss-Newton) iterations, every lane a cold-start NMPC_controller.solve
  (acados_nmpc/NMPC_controller.m:329-423), x0 drawn from the config-2 law
  (ranges of main.m:53-56), x_ref = the config-1 straight line from index 1.
A step is one batched solve of all lanes; inputs are resident in HBM before the
timed region, which brackets exactly --steps kernel launches.

Multi-GPU (torchrun): one process per GPU, each rank solves its own shard of
65 536 lanes (weak scaling, no data-path collective); the timing is the max over
ranks.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NMPC solves/sec at N=20, batch=65 536; max |u0−u0_ref|"
SHAPES = ("santal", "balea", "montana", "pulirapid")

# Algorithmic FP64 flops of the kernel's arithmetic (hand count of
# uclv_qs_pushing_matlab_amd/csrc/qsp_math.hpp + qsp_solver.hip, FMA = 2,
# div/sqrt/sin/cos/fmod = 1):
FLOP_LIN_STAGE = 2267   # RK4 + forward sensitivities + defect/gradient + rollout/update, per stage per SQP iteration
FLOP_IPM_STAGE = 874    # one Mehrotra iteration (factor + 2 solves + barrier/step), per stage
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) peak, datasheet (MI355X_MICROARCH.md)


def config2_x0(nb, seed):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-0.0065, 0.0260, nb), rng.uniform(-0.0197, 0.0124, nb),
                     np.deg2rad(rng.uniform(-8.05, 9.30, nb)), rng.uniform(-0.0382, 0.0011, nb)], 1)


def straight_traj(T_end=10.0, Ts=0.05, v=0.01):
    t = np.arange(0.0, T_end + 1e-9, Ts)
    traj = np.zeros((len(t), 6))
    traj[:, 0] = v * t
    return traj


def make_inputs(B, N, seed, lo=0, hi=None):
    """Synthetic config-2/3 inputs for lanes [lo, hi) of a B-lane job (x0 drawn for all B lanes
    so that every shard sees the same values as a single-process run)."""
    hi = B if hi is None else hi
    x0 = config2_x0(B, seed)[lo:hi]
    traj = straight_traj()
    yref = np.broadcast_to(traj[None, :N], (hi - lo, N, 6)).copy()
    yref_e = yref[:, N - 1, :4].copy()
    shape_id = (np.arange(lo, hi) % len(SHAPES)).astype(np.int32)
    return x0, yref, yref_e, shape_id, traj


def shard_range(total, world, rank):
    """Contiguous, balanced shard of `total` units for `rank` (covers every unit once)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def flops_per_solve(N, K, qp_iter_total):
    return K * N * FLOP_LIN_STAGE + qp_iter_total * N * FLOP_IPM_STAGE


def cpu_baseline(x0, traj, shape_id, N, K, target_s, threads, nlp_mode=0):
    """Oracle (port) timed on a bounded sample of the same workload (cold-start controller solves)."""
    from oracle.oracle import Oracle, make_opts
    orc = Oracle(SHAPES)
    op = make_opts(N=N, sqp_iters=K, nlp_mode=nlp_mode)

    def run(sl, xx=None, K_run=K, **kw):
        xx = x0[sl] if xx is None else xx
        warm = orc.new_warm(len(xx), N)
        o = op if (K_run == K and not kw) else make_opts(N=N, sqp_iters=K_run, nlp_mode=nlp_mode, **kw)
        return orc.controller_solve(o, xx, traj, 1, warm, shape_id=shape_id[sl], nthreads=threads)

    probe = min(len(x0), max(2 * threads, 16))
    t0 = time.perf_counter()
    run(slice(0, probe))
    per = (time.perf_counter() - t0) / probe
    n = int(min(len(x0), max(probe, target_s / max(per, 1e-7))))
    n = min(len(x0), max(threads, (n // threads) * threads))
    t0 = time.perf_counter()
    r = run(slice(0, n))
    dt = time.perf_counter() - t0
    return n, dt, r, run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="lanes per GPU")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--sqp-iters", type=int, default=50)
    ap.add_argument("--qp-iters", type=int, default=50)
    ap.add_argument("--stages-per-lane", type=int, default=0)
    ap.add_argument("--stream-parts", type=int, default=0, choices=(0, 1, 2),
                    help="SQP loop in 1 or 2 lane parts on their own HIP streams (0 = the library's auto choice)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--nlp", choices=("SQP_RTI", "SQP"), default="SQP_RTI",
                    help="SQP_RTI: fixed-K full steps (the BASELINE metric); SQP: the reference's merit-backtracking "
                         "SQP with KKT tolerances (sqp_iters = max_iter)")
    ap.add_argument("--seed", type=int, default=20250303 + 3)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; QSP_DIST_BACKEND=gloo + several ranks per device is only for
    # rehearsing the multi-rank path on a one-GPU machine
    backend = os.environ.get("QSP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local_rank % ndev if backend == "gloo" and ndev else local_rank
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    red_dev = dev if backend == "nccl" else torch.device("cpu")   # device of the timing reductions

    from uclv_qs_pushing_matlab_amd._lib import DeviceIO
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver

    B, N, K = args.batch, args.N, args.sqp_iters
    # this rank's shard of the global lane set (weak scaling: B lanes per GPU)
    lo, hi = shard_range(B * world, world, rank)
    x0, yref, yref_e, sid, traj = make_inputs(B * world, N, args.seed, lo, hi)
    Bl = hi - lo

    solver = OcpSolver(N=N, batch=Bl, sqp_iters=K, qp_iters=args.qp_iters, stages_per_lane=args.stages_per_lane,
                       device=gpu, nlp_solver_type=args.nlp)
    solver.set_shapes([make_shape(n) for n in SHAPES])
    S_layout, L_layout = solver.layout()
    solver.set_stream_parts(args.stream_parts)
    parts = solver.stream_parts()

    t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
    d_x0, d_yref, d_yref_e = t(x0), t(yref), t(yref_e)
    d_sid = t(sid, torch.int32)
    d_Xin = torch.zeros((Bl, N + 1, 4), dtype=torch.float64, device=dev)
    d_Uin = torch.zeros((Bl, N, 2), dtype=torch.float64, device=dev)
    d_u0 = torch.empty((Bl, 2), dtype=torch.float64, device=dev)
    d_X = torch.empty((Bl, N + 1, 4), dtype=torch.float64, device=dev)
    d_U = torch.empty((Bl, N, 2), dtype=torch.float64, device=dev)
    d_PI = torch.empty((Bl, N, 4), dtype=torch.float64, device=dev)
    d_st = torch.empty((Bl,), dtype=torch.int32, device=dev)
    d_cost = torch.empty((Bl,), dtype=torch.float64, device=dev)
    io = DeviceIO()
    for name, ten in (("x0", d_x0), ("yref", d_yref), ("yref_e", d_yref_e), ("X_in", d_Xin), ("U_in", d_Uin),
                      ("shape_id", d_sid), ("u0", d_u0), ("X_out", d_X), ("U_out", d_U), ("PI_out", d_PI),
                      ("status", d_st), ("cost", d_cost)):
        setattr(io, name, ten.data_ptr())
    io.controller = 1          # NMPC_controller.solve semantics, cold start every step
    io.warm_valid = None
    # a dedicated stream: the kernels and the timing events are on the same queue
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream

    for _ in range(args.warmup):
        solver.solve_device(io, sh)
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # HIP events at every kernel boundary of the timed solves, recorded on the launch stream
    solver.set_kernel_timing(args.steps)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        solver.solve_device(io, sh)
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    ktimes = solver.kernel_times()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # per-lane IPM iteration counts of the (identical) timed solves -> algorithmic flops
    solver.synchronize()
    qp_iter = solver.get("qp_iter")
    status = d_st.cpu().numpy()
    u0 = d_u0.cpu().numpy()
    flops_solve = float(flops_per_solve(N, K, qp_iter.astype(np.float64)).sum())   # all lanes, one solve
    # dominant kernel: qp_step (one launch = one SQP iteration's QP for every lane of the shard).
    # With two stream parts the two half launches of an SQP iteration overlap each other and
    # the next iteration's, so the library times the whole loop (fork -> join on the launch
    # stream, packing sorts included) and reports K "launches": launch_ms_avg is then the loop
    # time per SQP iteration over the whole shard (rocprof: union of the qp_step intervals / K,
    # scripts/ktrace_union.py)
    qp_ms, qp_n = ktimes["qp_step"]
    qp_avg_s = qp_ms / max(qp_n, 1) * 1e-3
    qp_flops_launch = float(qp_iter.astype(np.float64).sum()) * N * FLOP_IPM_STAGE / K
    if args.nlp == "SQP_RTI":   # the SQP iteration's linearisation runs inside the qp_step launch
        qp_flops_launch += float(Bl) * N * FLOP_LIN_STAGE
    if dist:
        tt = torch.tensor([float(np.count_nonzero(status))], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        nbad = int(tt[0])
    else:
        nbad = int(np.count_nonzero(status))

    total_solves = B * world * args.steps
    value = total_solves / elapsed
    avg_kern_s = float(np.mean(kern_ms)) * 1e-3
    achieved = qp_flops_launch / qp_avg_s / 1e12

    result = {
        "metric": METRIC, "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"BASELINE configs[2]: batch={B} per GPU, N={N}, 4 shapes mixed per lane, "
                               + (f"K={K} SQP-RTI iterations" if args.nlp == "SQP_RTI" else
                                  f"merit-backtracking SQP, max_iter={K}, tol 1e-6")
                               + ", cold-start NMPC_controller.solve per lane",
                   "global_batch": B * world, "N": N, "sqp_iters": K, "qp_iters_max": args.qp_iters,
                   "nlp_solver_type": args.nlp,
                   "layout": {"stages_per_lane": S_layout, "lanes_per_instance": L_layout,
                              "stream_parts": parts},
                   "parallelism": f"dp{world} (independent lane shards, no collective in the solve)"},
        "kernel_ms_avg": avg_kern_s * 1e3,
        "qp_iters_mean_per_qp": float(qp_iter.mean() / K),
        "status_nonzero_lanes": nbad,
        "kernels_ms_avg": {k: (v[0] / v[1] if v[1] else None) for k, v in ktimes.items()},
        "roofline": {"bound": "mfma", "kernel": "qp_step_kernel",
                     "peak_kind": "FP64 vector (= FP64 matrix) dense peak; the kernel is FP64-VALU bound",
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": None,
                     "flops_per_launch": qp_flops_launch, "launch_ms_avg": qp_avg_s * 1e3,
                     "launch": (f"one SQP iteration over the shard: {parts} concurrent part launches on {parts} streams, "
                                "timed fork -> join" if parts > 1 else "one qp_step launch over the shard"),
                     "whole_solve_tflops": flops_solve / avg_kern_s / 1e12},
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("batch") == Bl and pm.get("N") == N and pm.get("sqp_iters") == K:
                result["roofline"]["traffic"] = pm.get("hbm_bytes_per_launch")
        except Exception:
            pass

    # host-boundary rate (not `value`): NMPC_controller.solve through the C ABI with x0 in
    # host memory and u0 copied back, y_ref staged on the device from the shared table
    if world == 1:
        solver.set_shape_ids(sid)
        solver.set_reference_trajectory(traj)
        solver.controller_solve(x0, 1)
        solver.controller_reset()
        th = time.perf_counter()
        nrep = max(1, min(args.steps, 3))
        for _ in range(nrep):
            solver.controller_reset()
            solver.controller_solve(x0, 1)
        result["host_boundary_solves_per_s"] = Bl * nrep / (time.perf_counter() - th)

    if rank == 0 and world == 1 and not args.no_cpu:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        threads = max(1, min(threads, 16))
        n, dt, r, run = cpu_baseline(x0, traj, sid, N, K, args.cpu_seconds, threads, 1 if args.nlp == "SQP" else 0)
        result["cpu_baseline"] = {"value": n / dt, "unit": "solves/s", "cores": threads, "kind": "port",
                                  "sample": f"{n} lanes of the same workload (oracle/qsp_oracle.c, OpenMP, "
                                            f"{dt:.1f} s)"}
        # parity on the sampled lanes: GPU u0 vs oracle u0 (same cold-start controller solve)
        u0_ref = r["u0"]
        d = np.abs(u0[:n] - u0_ref).max(1)
        m = min(n, 512)
        # a lane is 'stable' when the oracle itself stays put (< 1e-9) under three 1e-13 relative
        # perturbations of x0: the full-step SQP amplifies rounding on the other lanes
        stable = np.ones(m, bool)
        self_dev = np.zeros(m)   # how far the oracle itself moves under the perturbations
        for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
            rp = run(slice(0, m), x0[:m] * (1 + sgn * f * 1e-13))
            dev = np.abs(rp["u0"] - u0_ref[:m]).max(1)
            stable &= dev < 1e-9
            self_dev = np.maximum(self_dev, dev)
        # ... and converged (the K-1 and K iterates agree: not a limit cycle of the full-step SQP)
        if args.nlp == "SQP_RTI":
            stable &= np.abs(run(slice(0, m), K_run=K - 1)["u0"] - u0_ref[:m]).max(1) < 1e-9
            # ... and insensitive to where the IPM stop test (mu < mu_stop) fires
            stable &= np.abs(run(slice(0, m), mu_stop=1.5e-10)["u0"] - u0_ref[:m]).max(1) < 1e-9
        else:   # merit SQP: the lanes that met the KKT tolerances
            stable &= r["status"][:m] == 0
        result["parity"] = {"max_abs_u0_err": float(d.max()), "lanes": int(n),
                            "max_abs_u0_err_stable_lanes": float(d[:m][stable].max()) if stable.any() else None,
                            "stable_lanes": int(stable.sum()), "stable_checked": int(m),
                            "frac_lanes_err_le_1e-6": float(np.mean(d <= 1e-6)),
                            # the same statistic for the oracle against itself under 1e-13 relative
                            # perturbations of x0 (first `stable_checked` lanes): the GPU/oracle gap
                            # on the remaining lanes is the problem's own sensitivity
                            "frac_lanes_err_le_1e-6_first": float(np.mean(d[:m] <= 1e-6)),
                            "oracle_self_frac_le_1e-6_first": float(np.mean(self_dev <= 1e-6)),
                            "note": "u0_ref = CPU oracle (acados parity unpinned); 'stable' = oracle itself moves "
                                    "< 1e-9 under three 1e-13 relative perturbations of x0, between K-1 and K "
                                    "iterations and with mu_stop 1.5e-10 (converged, non-chaotic lane)"}
    if rank == 0:
        if nbad:
            print(f"bench: WARNING {nbad} of {B * world} lanes returned a non-zero status", file=sys.stderr)
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()
    solver.close()


if __name__ == "__main__":
    main()
