#!/usr/bin/env python3
"""Benchmark: batched pusher-slider NMPC solves/s on MI355X (BASELINE.json metric).

Workload at N = 1 GPU (BASELINE configs[2], the configuration the metric is quoted on):
  N = 20, batch = 65 536 lanes, 4 slider shapes mixed per lane (shape_id = lane mod 4:
  santal/balea/montana/pulirapid), K = 50 SQP-RTI (full Gauss-Newton) iterations, every lane a
  cold-start NMPC_controller.solve (acados_nmpc/NMPC_controller.m:329-423), x0 drawn from the
  config-2 law (ranges of main.m:53-56), x_ref = the config-1 straight line from index 1.
Workload at N > 1 GPUs (BASELINE configs[3]): the same law over a global batch of 262 144 lanes
  split into contiguous shards, one process per GPU (strong scaling: 131 072 lanes per GPU at
  N = 2, 32 768 at N = 8), no collective on the data path; after the timed region the u0/status
  of all shards are all-gathered over RCCL (xGMI), timed separately ("gather_ms").
A step is one batched solve of all lanes; inputs are resident in HBM before the timed region,
which brackets exactly --steps solves.  Rank 0 prints one JSON line.
`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts the N ranks itself, one
process per GPU through torch.distributed.run, before anything touches a GPU.
Parity: every lane's u0 (and status, iteration counts) against the oracle's kernel-order twin
(oracle/qsp_twin.c, bit for bit), and against the literal restatement (oracle/qsp_oracle.c) with
its own rounding sensitivity as the yardstick.
`python bench.py --closed-loop` measures SURVEY §8(f) row 1 instead: main.m's closed loop, batched
(closed_loop_bench).
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


from uclv_qs_pushing_matlab_amd.sharding import gather_lanes, shard_range  # noqa: E402,F401  (re-exported)

CONFIG2_BATCH = 65536          # BASELINE configs[2]: one GPU
CONFIG3_BATCH = 262144         # BASELINE configs[3]: sharded over the GPUs of one node
SEED = 20250303 + 3


def config4_inputs(B, N, seed, lo=0, hi=None):
    """BASELINE configs[4]: N = 50, the curved x_finals.mat reference (x, y, theta; s_ref = 0) with a
    random start index per lane in [1, 797 - N], x0 near the reference start (s inside its bounds),
    shapes mixed per lane; per-lane y_ref staged on the host (lanes [lo, hi) of a B-lane job)."""
    from uclv_qs_pushing_matlab_amd.objects import DATA_DIR
    hi = B if hi is None else hi
    xf = np.load(os.path.join(DATA_DIR, "x_finals.npz"))
    traj = np.zeros((len(xf["x"]), 6))
    traj[:, 0], traj[:, 1], traj[:, 2] = xf["x"], xf["y"], xf["theta"]
    rng = np.random.default_rng(seed)
    idx = rng.integers(1, len(traj) - N, B).astype(np.int32)
    x0 = traj[idx - 1, :4] + np.stack([rng.uniform(-0.005, 0.005, B), rng.uniform(-0.005, 0.005, B),
                                       rng.uniform(-0.05, 0.05, B), rng.uniform(-0.03, 0.005, B)], 1)
    idx, x0 = idx[lo:hi], x0[lo:hi]
    cols = np.minimum(idx[:, None] + np.arange(N)[None, :], len(traj)) - 1          # get_y_ref clamp
    yref = traj[cols]
    yref_e = yref[:, N - 1, :4].copy()
    shape_id = (np.arange(lo, hi) % len(SHAPES)).astype(np.int32)
    return x0, yref, yref_e, shape_id, traj, idx


def config1_inputs(N, B=4096, seed=20250303 + 1):
    """BASELINE configs[1]: B = 4 096 random x0 (config-2 law) around santal, straight x_ref."""
    x0 = config2_x0(B, seed)
    traj = straight_traj()
    return x0, traj, np.zeros(B, np.int32)


def host_cpu():
    """Host CPU facts for the cpu_baseline record: nproc, the CPUs this process may run on,
    the model name, and the worker threads used (OMP_NUM_THREADS when set: the GPU box sets it
    to this job's CPU share; otherwise every CPU of the affinity mask)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    quota = None   # the cgroup's CPU quota (cgroup v2 cpu.max "max 100000" = none), in CPUs
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    return dict(nproc=os.cpu_count(), affinity_cpus=aff, model=model, threads=max(1, env or aff), cgroup_cpus=quota)


def device_facts(dev):
    """The GPU the line was measured on: name, compute units, and the top of the shader clock table
    (sysfs pp_dpm_sclk of the card with this PCI bus id, when readable) -- boxes of the pool differ
    by up to ~13 % at the same build, and this is where the difference shows."""
    import glob
    import torch
    pr = torch.cuda.get_device_properties(dev)
    out = {"name": pr.name, "gcn_arch": getattr(pr, "gcnArchName", None), "cus": pr.multi_processor_count}
    try:
        bus = "%04x:%02x:%02x" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        for card in glob.glob("/sys/class/drm/card*/device"):
            if os.path.basename(os.path.realpath(card)).startswith(bus):
                with open(os.path.join(card, "pp_dpm_sclk")) as f:
                    mhz = [int(t.split(":")[1].strip().split("Mhz")[0].split("MHz")[0]) for t in f.read().splitlines() if ":" in t]
                out["sclk_max_mhz"] = max(mhz)
                for hw in glob.glob(os.path.join(card, "hwmon", "hwmon*")):
                    for nm, key in (("power1_cap", "power_cap_w"), ("power1_cap_max", "power_cap_max_w")):
                        pth = os.path.join(hw, nm)
                        if os.path.exists(pth):
                            with open(pth) as f:
                                out[key] = int(f.read().strip()) / 1e6
                for nm in ("product_name", "product_number"):
                    pth = os.path.join(card, nm)
                    if os.path.exists(pth):
                        with open(pth) as f:
                            out[nm] = f.read().strip()
                break
    except Exception:
        pass
    return out


def flops_per_solve(N, K, qp_iter_total):
    return K * N * FLOP_LIN_STAGE + qp_iter_total * N * FLOP_IPM_STAGE


def cpu_baseline(x0, traj, shape_id, N, K, target_s, threads, nlp_mode=0, twin=True, qp_iters=20, idx=1,
                 sample=None, lane_walk=0):
    """The CPU restatement (port) timed on a bounded sample of the same workload (cold-start
    controller solves): the kernel-order twin (twin=True: the library's formulation on the CPU,
    OpenMP over lanes) or the literal oracle.  idx: index_time (scalar, or per lane).  sample: a
    fixed lane count instead of the target_s time budget (no probe run).  lane_walk=1: the twin
    factorises in the lane walk's order (the fastest CPU formulation of the algorithm) instead of
    emulating the matrix cores' (the bit-exact checker's order)."""
    from oracle.oracle import Oracle, make_opts
    orc = Oracle(SHAPES, twin=twin)
    op = make_opts(N=N, sqp_iters=K, nlp_mode=nlp_mode, qp_iters=qp_iters, lane_walk=lane_walk)
    idx_all = np.broadcast_to(np.asarray(idx, np.int32), (len(x0),))

    def run(sl, xx=None, K_run=K, nthreads=None, precision=None, **kw):
        xx = x0[sl] if xx is None else xx
        warm = orc.new_warm(len(xx), N)
        o = op if (K_run == K and not kw) else make_opts(N=N, sqp_iters=K_run, nlp_mode=nlp_mode,
                                                         **dict(dict(qp_iters=qp_iters, lane_walk=lane_walk), **kw))
        nt = threads if nthreads is None else nthreads
        if precision is not None:   # the literal restatement in long double / __float128 (oracle OR_EXT)
            return orc.controller_solve_ext(o, xx, traj, idx_all[sl], warm, shape_id=shape_id[sl], nthreads=nt,
                                            precision=precision)
        return orc.controller_solve(o, xx, traj, idx_all[sl], warm, shape_id=shape_id[sl], nthreads=nt)

    if sample is not None:
        n = min(len(x0), int(sample))
    else:
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


def thread_scaling(run, rate_all, threads, aff, seconds=1.5):
    """The twin's solves/s on 1 and 4 threads (short samples) beside the job's `threads`: lanes are
    independent, so the rate scales with the cores given; `full_host_estimate` extrapolates the
    per-thread rate at `threads` to every CPU of the affinity mask (the GPU box allots this job
    `threads` of them: a run on all of them is not this job's to make)."""
    out = {"threads": [], "solves_per_s": []}
    for t in (1, 4):
        if t >= threads:
            continue
        t0 = time.perf_counter()
        run(slice(0, 2 * t), nthreads=t)
        per = (time.perf_counter() - t0) / (2 * t)
        n = max(t, int(seconds / max(per, 1e-7) * t) // t * t)
        t0 = time.perf_counter()
        run(slice(0, n), nthreads=t)
        out["threads"].append(t)
        out["solves_per_s"].append(n / (time.perf_counter() - t0))
    out["threads"].append(threads)
    out["solves_per_s"].append(rate_all)
    out["efficiency_vs_1_thread"] = (rate_all / threads) / out["solves_per_s"][0] if out["threads"][0] == 1 else None
    out["full_host_estimate"] = {"cpus": aff, "solves_per_s": rate_all / threads * aff,
                                 "note": f"per-thread rate at {threads} threads x {aff} CPUs (linear scaling: an "
                                         "upper bound for the CPU)"}
    return out


def extended_adjudication(u_gpu, u_lit, run, lanes_sets, max_lanes=64, control=None):
    """Where the GPU and the double literal restatement disagree by > 1e-6: the literal formulas in
    __float128 (and long double), the exact-arithmetic answer as far as the SQP's amplification
    allows (long double and quad agreeing to 1e-6 marks that), and which implementation it sides with
    (tests/tools/ext_adjudicate.py).  lanes_sets: (name, lane indices) in
    priority order, capped at max_lanes in total; control: lanes where both agree."""
    picked, names = [], []
    for name, ls in lanes_sets:
        for l in ls:
            if len(picked) < max_lanes and l not in picked:
                picked.append(int(l))
                names.append(name)
    lanes = np.array(picked + [int(c) for c in (control if control is not None else [])], dtype=np.int64)
    if len(lanes) == 0:
        return {"lanes": 0}
    t0 = time.perf_counter()
    uq = run(lanes, precision="quad")["u0"]
    ul = run(lanes, precision="long")["u0"]
    dt = np.abs(u_gpu[lanes] - uq).max(1)
    dl = np.abs(u_lit[lanes] - uq).max(1)
    ext_ok = np.abs(ul - uq).max(1) <= 1e-6
    n_sel = len(names)
    sel = np.arange(len(lanes)) < n_sel
    side = np.where((dt <= 1e-6) & (dl > 1e-6), "gpu", np.where((dl <= 1e-6) & (dt > 1e-6), "literal",
                    np.where((dt <= 1e-6) & (dl <= 1e-6), "both", "neither")))
    out = {"reference": "oracle/qsp_oracle.c in __float128 (libquadmath) and long double, the same formulas",
           "seconds": time.perf_counter() - t0}
    # the metric against exact arithmetic where it has an answer: every adjudicated lane (disagreeing
    # and control) on which long double and quad agree to 1e-6
    if ext_ok.any():
        out["extended_stable"] = {"lanes": int(ext_ok.sum()), "of_disagreeing": int(np.sum(ext_ok & sel)),
                                  "max_abs_u0_err_gpu_vs_quad": float(dt[ext_ok].max()),
                                  "max_abs_u0_err_literal_vs_quad": float(dl[ext_ok].max()),
                                  "gpu_within_1e-6_of_quad": int(np.sum(ext_ok & (dt <= 1e-6))),
                                  "literal_within_1e-6_of_quad": int(np.sum(ext_ok & (dl <= 1e-6)))}
    for name in dict.fromkeys(names):
        m = np.array([nm == name for nm in names] + [False] * (len(lanes) - len(names)))
        out[name] = {"lanes": int(m.sum()), "ext_stable": int(np.sum(m & ext_ok)),
                     **{f"sides_with_{k}": int(np.sum(m & (side == k))) for k in ("gpu", "literal", "both", "neither")}}
        if name == "stable_in_both":
            out[name]["per_lane"] = [{"lane": int(lanes[j]), "side": str(side[j]), "gpu_err": float(dt[j]),
                                      "literal_err": float(dl[j])} for j in np.flatnonzero(m)]
    if control is not None and len(control):
        m = np.arange(len(lanes)) >= len(names)
        out["control_agreeing_lanes"] = {"lanes": int(m.sum()), "gpu_within_1e-6_of_quad": int(np.sum(m & (dt <= 1e-6))),
                                         "literal_within_1e-6_of_quad": int(np.sum(m & (dl <= 1e-6)))}
    return out


def parity_leg(u0_gpu, x0, traj, sid, N, K, n, r, run, nlp, gpu_dev=None, qp_iters=20, extended=True, ext_lanes=48):
    """GPU u0 vs oracle u0 on the whole CPU sample (n lanes), with the oracle's own sensitivity
    as the yardstick: a lane is chaotic when the oracle's u0 moves by > 1e-9 under
    three 1e-13 relative perturbations of x0 or when mu_stop moves 1e-10 -> 1.5e-10; parity is
    asserted (informatively here, in tests/test_gpu_config2.py as a test) on the others."""
    u0_ref = r["u0"]
    d = np.abs(u0_gpu[:n] - u0_ref).max(1)
    self_dev = np.zeros(n)
    for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
        self_dev = np.maximum(self_dev, np.abs(run(slice(0, n), x0[:n] * (1 + sgn * f * 1e-13))["u0"] - u0_ref).max(1))
    mu_dev = np.abs(run(slice(0, n), mu_stop=1.5e-10)["u0"] - u0_ref).max(1)
    nonchaotic = (self_dev < 1e-9) & (mu_dev < 1e-9)
    # the model probe (oracle/or_opts.h): the linearisation's outputs moved by +-1e-14 of their scale,
    # the size by which the literal and the kernel-order formulations differ
    mod_dev = np.zeros(n)
    for seed in (1, 2):
        mod_dev = np.maximum(mod_dev, np.abs(run(slice(0, n), model_probe=1e-14, probe_seed=seed)["u0"] - u0_ref).max(1))
    out = {"lanes": int(n), "max_abs_u0_err": float(d.max()),
           "nonchaotic_lanes": int(nonchaotic.sum()),
           "max_abs_u0_err_nonchaotic": float(d[nonchaotic].max()) if nonchaotic.any() else None,
           "frac_nonchaotic_err_le_1e-6": float(np.mean(d[nonchaotic] <= 1e-6)) if nonchaotic.any() else None,
           "frac_lanes_err_le_1e-6": float(np.mean(d <= 1e-6)),
           "oracle_self_frac_le_1e-6": float(np.mean(self_dev <= 1e-6)),
           "lanes_err_gt_1e-6": int(np.sum(d > 1e-6)),
           "lanes_err_gt_1e-6_moving_under_x0_or_model_probes": int(np.sum((d > 1e-6) & ((self_dev > 1e-6) | (mod_dev > 1e-6)))),
           "lanes_stable_under_all_probes": int(np.sum(nonchaotic & (mod_dev < 1e-9))),
           "max_abs_u0_err_stable_under_all_probes": float(d[nonchaotic & (mod_dev < 1e-9)].max())
                                                     if np.any(nonchaotic & (mod_dev < 1e-9)) else None,
           "chaotic_frac": float(np.mean(self_dev > 1e-6)),
           "qp_rule": f"HPIPM-style: mu, bound, stationarity, equality residuals < 1e-10, cap {qp_iters}, stall exit, "
                      "stage-0 s bound"}
    if gpu_dev is not None:
        # the GPU's own response to the same probes: the same share of lanes moves, largely the same
        # lanes, and the two implementations disagree almost only where one of them moves
        gc, rc = gpu_dev[:n] > 1e-6, self_dev > 1e-6
        out["gpu_chaotic_frac"] = float(gc.mean())
        out["chaotic_overlap_jaccard"] = float((gc & rc).sum() / max(int((gc | rc).sum()), 1))
        out["frac_err_gt_1e-6_stable_in_both"] = float(np.mean((d > 1e-6) & ~gc & ~rc))
        # the metric max|u0 - u0_ref| on the lanes stable under every probe of both implementations
        # (x0 probes on the GPU; x0, mu_stop and model probes on the literal)
        sb = (gpu_dev[:n] <= 1e-6) & (self_dev <= 1e-6) & (mod_dev <= 1e-6)
        out["probe_stable_in_both"] = {"lanes": int(sb.sum()),
                                       "max_abs_u0_err": float(d[sb].max()) if sb.any() else None,
                                       "frac_err_le_1e-6": float(np.mean(d[sb] <= 1e-6)) if sb.any() else None}
    if extended:
        # the disagreements adjudicated in extended precision: first the lanes stable in both
        # implementations, then those the literal's probes call stable, then the others
        dis = d > 1e-6
        lit_stable = dis & (self_dev <= 1e-6) & (mod_dev <= 1e-6)
        both = lit_stable & (gpu_dev[:n] <= 1e-6) if gpu_dev is not None else np.zeros(n, bool)
        rng = np.random.default_rng(3)
        rest = np.flatnonzero(dis & ~lit_stable)
        agree = np.flatnonzero(~dis)
        out["extended_precision"] = extended_adjudication(
            u0_gpu[:n], u0_ref, run,
            [("stable_in_both", np.flatnonzero(both)), ("literal_stable", np.flatnonzero(lit_stable & ~both)),
             ("other_disagreeing", rng.permutation(rest))],
            max_lanes=ext_lanes, control=np.sort(rng.choice(agree, min(ext_lanes // 2, len(agree)), replace=False)))
    if nlp == "SQP_RTI":
        # the same statistics with round 1's QP stop rule (mu and bound residual < 1e-10, cap 20,
        # no stage-0 s bound), on the first lanes: the chaotic fraction does not depend on it
        m = min(n, 2048)
        r01 = dict(qp_iters=20, qp_tol_stat=float("inf"), qp_tol_eq=float("inf"), stage0_s_bound=0, qp_stall_iters=0)
        base = run(slice(0, m), **r01)["u0"]
        dev = np.zeros(m)
        for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
            dev = np.maximum(dev, np.abs(run(slice(0, m), x0[:m] * (1 + sgn * f * 1e-13), **r01)["u0"] - base).max(1))
        out["chaotic_frac_first"] = {"lanes": int(m), "this_rule": float(np.mean(self_dev[:m] > 1e-6)),
                                     "round1_rule": float(np.mean(dev > 1e-6))}
    out["note"] = ("u0_ref = CPU oracle (acados parity unpinned); nonchaotic = the oracle itself moves < 1e-9 under "
                   "three 1e-13 relative x0 perturbations and mu_stop 1.5e-10; model probes = the oracle with its "
                   "linearisation moved by +-1e-14 of scale (two sign patterns)")
    return out


def closed_loop_measure(B, seed, runs, cpu_seconds, no_cpu, device=0, qp_iters=50):
    """SURVEY §8(f) row 1, measured: helper.closed_loop_matlab as main.m runs it (helper.m:195-322;
    main.m:40-41, 105, 150-205): Hp = 10, the reference's SQP options (sqp + merit backtracking,
    max_iter 30, tol 1e-6; QP cap qp_iters = acados' default 50, as the MEX sets it), time_sim 10 s (201 steps of Ts = 0.05), the 2-waypoint straight line,
    no noise, no delays, the disturbance step t_dist = 15 / Ts (past the end of the run, as in main.m)
    -- batched over B lanes (x0 from the config-2 law, 4 shapes mixed per lane), the whole loop on
    the device in one host call (qsp_closed_loop_ex).  Returns lane-steps/s, the twin's closed loop
    on the host threads as the CPU baseline, and every sampled lane's trajectory (X, U, status)
    against the twin bit for bit."""
    import torch
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, K, Ts, T = 10, 30, 0.05, 201
    x0 = config2_x0(B, seed)
    sid = (np.arange(B) % len(SHAPES)).astype(np.int32)
    traj = straight_traj()
    t_dist = int(round(15 / Ts))
    s = OcpSolver(N=N, batch=B, sqp_iters=K, qp_iters=qp_iters, nlp_solver_type="SQP", device=device)
    s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
    s.set_reference_trajectory(traj)
    S_layout, L_layout = s.layout()
    s.closed_loop(x0, 3, disturbance=True, t_dist=t_dist)          # warm-up (kernels, allocations)
    s.synchronize()
    torch.cuda.synchronize()
    times = []
    for _ in range(max(1, runs)):
        t0 = time.perf_counter()
        r = s.closed_loop(x0, T, disturbance=True, t_dist=t_dist)
        times.append(time.perf_counter() - t0)
    s.close()
    el = float(np.median(times))
    out = {"workload": f"{B} closed loops of {T} steps (main.m: Hp=10, sqp + merit backtracking, max_iter 30, "
                       f"tol 1e-6, QP cap {qp_iters}, straight-line reference, no noise, no delay, t_dist past the end), 4 shapes mixed "
                       "per lane, x0 from the config-2 law, whole loop on the device (qsp_closed_loop_ex, one host "
                       "call; trajectories copied back inside the timed region)",
           "gpu_lane_steps_per_s": B * T / el, "ms_per_run": el * 1e3, "runs": len(times),
           "batch": B, "N": N, "sqp_max_iter": K, "closed_loop_steps": T,
           "layout": {"stages_per_lane": S_layout, "lanes_per_instance": L_layout},
           "status_lane_steps": {str(int(k)): int(v) for k, v in zip(*np.unique(r["status"], return_counts=True))},
           "status_note": "acados codes per controller step: 0 converged, 2 max_iter reached, 4 QP failure "
                          "(stage-0 s outside its bounds, or a diverged QP); helper.m applies u0 regardless"}
    if not no_cpu:
        from oracle.oracle import Oracle, make_opts
        hc = host_cpu()
        threads = hc["threads"]
        tw = Oracle(SHAPES, twin=True)
        op = make_opts(N=N, sqp_iters=K, nlp_mode=1, qp_iters=qp_iters)
        probe = min(B, max(threads, 16))
        tp = time.perf_counter()
        tw.closed_loop(op, x0[:probe], traj, 20, shape_id=sid[:probe], dist_step=t_dist, nthreads=threads)
        per = (time.perf_counter() - tp) / (probe * 20)
        n = int(min(B, max(probe, cpu_seconds / max(per * T, 1e-9))))
        n = min(B, max(threads, (n // threads) * threads))
        tp = time.perf_counter()
        rc = tw.closed_loop(op, x0[:n], traj, T, shape_id=sid[:n], dist_step=t_dist, nthreads=threads)
        dt = time.perf_counter() - tp
        out["cpu_baseline"] = {"value": n * T / dt, "unit": "lane-steps/s", "cores": threads, "kind": "port",
                               "cpu_model": hc["model"],
                               "sample": f"{n} of the {B} closed loops, all {T} steps (oracle/qsp_twin.c "
                                         f"tw_closed_loop, OpenMP over {threads} threads, {dt:.1f} s)"}
        same = (np.all(r["X"][:n] == rc["X"], axis=(1, 2)) & np.all(r["U"][:n] == rc["U"], axis=(1, 2))
                & np.all(r["status"][:n] == rc["status"], axis=1))
        out["parity"] = {"reference": "oracle/qsp_twin.c tw_closed_loop", "lanes": int(n),
                         "bit_identical_trajectory_lanes": int(same.sum()),
                         "max_abs_u_err": float(np.abs(r["U"][:n] - rc["U"]).max()),
                         "max_abs_x_err": float(np.abs(r["X"][:n] - rc["X"]).max())}
    return out


def side_rows_measure(gpu, no_cpu):
    """SURVEY §8(f) rows 2 and 3 measured beside the headline: the shape preprocessing (PLY contour ->
    B-spline control points and knots, PusherSliderModel.m:84-132, in the C ABI's qsp_shape_from_ply)
    against the oracle's numpy restatement, bit for bit; and the per-lane reference generation
    (TrajectoryGenerator.straight_line, TrajectoryGenerator.m:39-79, straight_lines_kernel) for 65 536
    lanes x 201 samples on the device against the host mirror on a sample of lanes."""
    import torch
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    from uclv_qs_pushing_matlab_amd.trajectory import TrajectoryGenerator
    out = {}
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        shapes = [make_shape(n) for n in SHAPES]
    dt = time.perf_counter() - t0
    sp = {"shapes_per_s": reps * len(SHAPES) / dt, "note": "qsp_shape_from_ply (C++ PLY reader, float32 greedy "
          "contour sort, knots), the four reference contours, 20 repeats"}
    if not no_cpu:
        from oracle.shapes_np import shape_table
        t0 = time.perf_counter()
        for _ in range(reps):
            tab = shape_table(SHAPES)
        dtn = time.perf_counter() - t0
        same = all(int(sh.n_ctrl) == int(tab["n_ctrl"][i])
                   and np.array_equal(np.ctypeslib.as_array(sh.ctrl)[:sh.n_ctrl], tab["ctrl"][i][:sh.n_ctrl])
                   and np.array_equal(np.ctypeslib.as_array(sh.knots)[:sh.n_ctrl + 4], tab["knots"][i][:sh.n_ctrl + 4])
                   for i, sh in enumerate(shapes))
        sp.update({"cpu_shapes_per_s": reps * len(SHAPES) / dtn, "cpu_kind": "oracle/shapes_np.py (numpy)",
                   "bit_identical_to_oracle": bool(same)})
    out["shape_preprocessing"] = sp
    B, T = CONFIG2_BATCH, 201
    rng = np.random.default_rng(SEED)
    x0 = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.05, 0.05, B), rng.uniform(-0.2, 0.2, B)], 1)
    xf = x0 + np.stack([rng.uniform(0.02, 0.3, B), rng.uniform(-0.05, 0.05, B), rng.uniform(-0.2, 0.2, B)], 1)
    s = OcpSolver(N=20, batch=B, device=gpu)
    s.set_shapes([shapes[0]])
    s.gen_straight_lines(x0, xf, 0.0, 10.0)
    s.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        Tg = s.gen_straight_lines(x0, xf, 0.0, 10.0)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 5
    tab = s.get_reference_trajectories()
    s.close()
    rg = {"lanes_per_s": B / dt, "samples": int(Tg), "lanes": B,
          "note": "straight_lines_kernel: one lane per thread, the quintic time law over 201 samples, host x0/xf in"}
    n = 256
    t0 = time.perf_counter()
    err = 0.0
    for i in range(n):
        tg = TrajectoryGenerator(0.05, 0.01)
        tg.set_target(x0[i], xf[i], 0.0, 10.0)
        _, ref = tg.straight_line(False)
        err = max(err, float(np.abs(tab[i, :, :3] - ref.T).max()))
    rg.update({"host_mirror_lanes_per_s": n / (time.perf_counter() - t0), "host_mirror_sample": n,
               "max_abs_err_vs_host_mirror": err})
    out["reference_generation"] = rg
    return out


def closed_loop_bench(args):
    """`bench.py --closed-loop`: the closed-loop measurement (closed_loop_measure) as its own line."""
    m = closed_loop_measure(args.global_batch or CONFIG2_BATCH, args.seed, args.steps, args.cpu_seconds, args.no_cpu)
    result = {"metric": "closed-loop controller steps/s (helper.closed_loop_matlab, main.m scenario)",
              "value": m.pop("gpu_lane_steps_per_s"), "unit": "lane-steps/s", "n_gpus": 1, "steps": m["runs"],
              "warmup": 1, "ms_per_step": m["ms_per_run"], "higher_is_better": True, "scaling": "strong",
              "vs_baseline": None, "dtype": "f64", "data": "synthetic",
              "config": {k: m.pop(k) for k in ("workload", "batch", "N", "sqp_max_iter", "closed_loop_steps", "layout")}}
    result.update(m)
    print(json.dumps(result), flush=True)


def launch_ranks(n):
    """--gpus N > 1 without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run on this node and return its exit code.  Runs before anything touches a
    GPU (only the device count is read, which initialises nothing).  The rank processes inherit
    stdout, so rank 0's JSON line is this command's output."""
    import socket
    import subprocess

    import torch
    rehearsal = os.environ.get("QSP_DIST_BACKEND", "nccl") == "gloo"   # ranks may share a device
    ndev = torch.cuda.device_count()
    if ndev < n and not (rehearsal and ndev >= 1):
        print(f"bench.py --gpus {n}: only {ndev} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--global-batch", type=int, default=0,
                    help="lanes over all GPUs (0: the configuration's batch: 65 536 = configs[2] on one GPU, "
                         "262 144 = configs[3] on several, 16 384 for configs[4])")
    ap.add_argument("--config", type=int, default=0, choices=(0, 2, 4),
                    help="BASELINE configuration: 0 = the metric's (configs[2] on one GPU, configs[3] on several); "
                         "4 = N = 50 over the curved x_finals reference")
    ap.add_argument("--N", type=int, default=0, help="horizon (0: the configuration's, 20 or 50)")
    ap.add_argument("--sqp-iters", type=int, default=50)
    ap.add_argument("--qp-iters", type=int, default=20,
                    help="QP iteration cap (the library default, 20; acados' qp_solver_iter_max default is 50: "
                         "-2.2 %% here, but 2.3x slower at B = 4 096 where every SQP iteration waits for its slowest "
                         "wave; DESIGN.md section 1)")
    ap.add_argument("--stages-per-lane", type=int, default=0)
    ap.add_argument("--factor-scan", action="store_true",
                    help="two stages per lane: the factorisation as an associative scan (qsp_options.factor_scan)")
    ap.add_argument("--stream-parts", type=int, default=0, choices=(0, 1, 2),
                    help="SQP loop in 1 or 2 lane parts on their own HIP streams (0 = the library's auto choice)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-configs1", action="store_true", help="skip the configs[1] (B = 4 096) side measurement")
    ap.add_argument("--no-configs4", action="store_true", help="skip the configs[4] (N = 50, B = 16 384) side measurement")
    ap.add_argument("--no-qp50", action="store_true",
                    help="skip the headline workload at acados' default QP cap (qp_solver_iter_max 50)")
    ap.add_argument("--no-closed-loop", action="store_true",
                    help="skip the closed-loop side measurement (main.m's loop over 16 384 lanes, SURVEY §8(f) row 1)")
    ap.add_argument("--nlp", choices=("SQP_RTI", "SQP"), default="SQP_RTI",
                    help="SQP_RTI: fixed-K full steps (the BASELINE metric); SQP: the reference's merit-backtracking "
                         "SQP with KKT tolerances (sqp_iters = max_iter)")
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--dump-u0", default=None, help="rank 0 writes the gathered u0/status (.npz) here")
    ap.add_argument("--closed-loop", action="store_true",
                    help="measure the batched closed loop of main.m instead (SURVEY §8(f) row 1; one GPU; "
                         "--global-batch lanes, --steps timed runs)")
    args = ap.parse_args()

    if args.closed_loop:
        if args.gpus != 1:
            raise SystemExit("bench.py --closed-loop runs on one GPU")
        return closed_loop_bench(args)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} under WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; QSP_DIST_BACKEND=gloo + several ranks per device is only for
    # rehearsing the multi-rank path on a one-GPU machine
    backend = os.environ.get("QSP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local_rank % ndev if backend == "gloo" and ndev else local_rank
    dist = None
    # QSP_DIST_FORCE=1 opens the process group at world size 1 too (under torch.distributed.run): the
    # one-GPU box can then run the RCCL branch (device tensors, barrier, MAX all_reduce, gather_lanes),
    # since RCCL refuses two ranks on one device (tests/test_gpu_multirank.py)
    if world > 1 or (os.environ.get("QSP_DIST_FORCE") == "1" and "WORLD_SIZE" in os.environ):
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    red_dev = dev if backend == "nccl" else torch.device("cpu")   # device of the reductions and the gather

    from uclv_qs_pushing_matlab_amd._lib import DeviceIO
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver

    cfg4 = args.config == 4
    N, K = args.N or (50 if cfg4 else 20), args.sqp_iters
    total = args.global_batch or (16384 if cfg4 else (CONFIG2_BATCH if world == 1 else CONFIG3_BATCH))
    lo, hi = shard_range(total, world, rank)        # this rank's shard of the global lane set
    if cfg4:
        x0, yref, yref_e, sid, traj, idx4 = config4_inputs(total, N, args.seed, lo, hi)
    else:
        x0, yref, yref_e, sid, traj = make_inputs(total, N, args.seed, lo, hi)
        idx4 = None
    Bl = hi - lo

    solver = OcpSolver(N=N, batch=Bl, sqp_iters=K, qp_iters=args.qp_iters, stages_per_lane=args.stages_per_lane,
                       device=gpu, nlp_solver_type=args.nlp, factor_scan=args.factor_scan)
    solver.set_shapes([make_shape(n) for n in SHAPES])
    S_layout, L_layout = solver.layout()
    factor_walk = solver.factor_walk()
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
    qp_capped = solver.get("qp_capped")

    # the trivial gather (north_star): u0 and status of every shard to every rank, one fixed-size
    # all_gather each over RCCL (device tensors; gloo: host tensors), timed on its own
    gather_ms = None
    if dist:
        g_u0, g_st = d_u0.to(red_dev), d_st.to(red_dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        u0_all = gather_lanes(g_u0, total, dist, world, rank)
        st_all = gather_lanes(g_st, total, dist, world, rank)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - tg) * 1e3
        tt = torch.tensor([gather_ms], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        gather_ms = float(tt.item())
        u0_all, status_all = u0_all.cpu().numpy(), st_all.cpu().numpy()
    else:
        u0_all, status_all = d_u0.cpu().numpy(), d_st.cpu().numpy()
    u0 = u0_all[lo:hi]
    nbad = int(np.count_nonzero(status_all))
    if rank == 0 and args.dump_u0:
        np.savez(args.dump_u0, u0=u0_all, status=status_all)

    flops_solve = float(flops_per_solve(N, K, qp_iter.astype(np.float64)).sum())   # this shard, one solve
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

    total_solves = total * args.steps
    value = total_solves / elapsed
    avg_kern_s = float(np.mean(kern_ms)) * 1e-3
    achieved = qp_flops_launch / qp_avg_s / 1e12
    if cfg4:
        workload = (f"BASELINE configs[4]: batch={total} over {world} GPU(s), curved x_finals reference, "
                    "random start index per lane")
    elif world == 1:
        workload = f"BASELINE configs[2]: batch={total} on 1 GPU"
    else:
        workload = (f"BASELINE configs[3]: global batch={total} sharded over {world} GPUs "
                    f"({Bl} lanes on rank {rank}), u0/status all-gathered over "
                    f"{'RCCL' if backend == 'nccl' else backend} after the timed region")

    result = {
        "metric": METRIC, "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": workload + f", N={N}, 4 shapes mixed per lane, "
                               + (f"K={K} SQP-RTI iterations" if args.nlp == "SQP_RTI" else
                                  f"merit-backtracking SQP, max_iter={K}, tol 1e-6")
                               + ", cold-start NMPC_controller.solve per lane",
                   "global_batch": total, "N": N, "sqp_iters": K, "qp_iters_max": args.qp_iters,
                   "nlp_solver_type": args.nlp,
                   "layout": {"stages_per_lane": S_layout, "lanes_per_instance": L_layout,
                              "stream_parts": parts, "factor_scan": bool(args.factor_scan and S_layout == 2),
                              # as the library reports it (qsp_get_factor_walk)
                              "factor_walk": factor_walk},
                   "parallelism": f"dp{world} (contiguous lane shards, no collective in the solve)"},
        "kernel_ms_avg": avg_kern_s * 1e3,
        "qp_iters_mean_per_qp": float(qp_iter.mean() / K),
        "qp_capped_frac": float(qp_capped.sum() / (Bl * K)),
        "status_nonzero_lanes": nbad,
        "gather_ms": gather_ms,
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
    result["device"] = device_facts(dev)
    # HBM traffic per launch from the PMC record of this workload (profiles/pmc_traffic*.json: the
    # headline's and configs[4]'s), only while the library is built from the kernel code it was
    # collected at
    import glob
    recs = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json")))
    if recs:
        result["roofline"]["traffic_source"] = ("not reported: no profiles/pmc_traffic*.json record of this "
                                                "kernel source and workload")
        try:
            from uclv_qs_pushing_matlab_amd.build import source_digest
            dig = source_digest()
            for path in recs:
                with open(path) as f:
                    pm = json.load(f)
                if (pm.get("kernel_digest") == dig and pm.get("batch") == Bl and pm.get("N") == N
                        and pm.get("sqp_iters") == K and pm.get("qp_iters", 20) == args.qp_iters):
                    result["roofline"]["traffic"] = pm.get("hbm_bytes_per_launch")
                    result["roofline"]["traffic_source"] = (f"profiles/{os.path.basename(path)}: rocprofv3 FETCH_SIZE x 2 "
                                                            "+ WRITE_SIZE of this kernel source (digest "
                                                            f"{pm.get('kernel_digest')})")
                    break
        except Exception:
            pass

    if world == 1:
        # host-boundary rate (not `value`): NMPC_controller.solve through the C ABI with x0 in
        # host memory and u0 copied back, y_ref staged on the device from the shared table
        solver.set_shape_ids(sid)
        solver.set_reference_trajectory(traj)
        idx_h = idx4 if cfg4 else 1
        solver.controller_solve(x0, idx_h)
        solver.controller_reset()
        th = time.perf_counter()
        nrep = max(1, min(args.steps, 3))
        for _ in range(nrep):
            solver.controller_reset()
            u_host = solver.controller_solve(x0, idx_h)
        result["host_boundary_solves_per_s"] = Bl * nrep / (time.perf_counter() - th)
        gpu_dev = None
        if rank == 0 and not args.no_cpu and not cfg4:
            # the GPU's own sensitivity to the parity leg's 1e-13 x0 probes (three solves, untimed)
            gpu_dev = np.zeros(Bl)
            for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
                solver.controller_reset()
                gpu_dev = np.maximum(gpu_dev, np.abs(solver.controller_solve(x0 * (1 + sgn * f * 1e-13), idx_h)
                                                     - u_host).max(1))
            result["host_boundary_u0_equals_device_u0"] = bool(np.array_equal(u_host, u0))
    solver.close()

    if (rank == 0 and world == 1 and not cfg4 and args.nlp == "SQP_RTI" and not args.no_qp50
            and args.qp_iters != 50):
        # the same workload at acados' default QP cap, qp_solver_iter_max = 50, which the reference leaves
        # in place (NMPC_controller.m:275): the same device-resident inputs and timing as the headline
        s50 = OcpSolver(N=N, batch=Bl, sqp_iters=K, qp_iters=50, stages_per_lane=args.stages_per_lane,
                        device=gpu, nlp_solver_type=args.nlp, factor_scan=args.factor_scan)
        s50.set_shapes([make_shape(n) for n in SHAPES])
        s50.set_stream_parts(args.stream_parts)
        s50.solve_device(io, sh)
        torch.cuda.synchronize(dev)
        n50 = max(1, min(args.steps, 5))
        t50 = time.perf_counter()
        for _ in range(n50):
            s50.solve_device(io, sh)
        torch.cuda.synchronize(dev)
        dt50 = time.perf_counter() - t50
        s50.synchronize()
        cap50 = s50.get("qp_capped")
        it50 = s50.get("qp_iter")
        u50 = d_u0.cpu().numpy()
        result["configs2_qp50"] = {
            "workload": "the headline workload with qp_iters_max = 50 (acados' qp_solver_iter_max default)",
            "solves_per_s": Bl * n50 / dt50, "ratio_to_headline": Bl * n50 / dt50 / value,
            "qp_capped_frac": float(cap50.sum() / (Bl * K)), "qp_iters_mean_per_qp": float(it50.mean() / K),
            "status_nonzero_lanes": int(np.count_nonzero(d_st.cpu().numpy())),
            "frac_u0_within_1e-6_of_cap20": float(np.mean(np.abs(u50 - u0).max(1) <= 1e-6)),
            "steps": n50, "factor_walk": s50.factor_walk()}
        s50.close()

    if rank == 0 and world == 1 and not args.no_configs1 and not cfg4:
        # BASELINE configs[1] beside the headline (its own GPU timing; CPU in full below)
        x1, traj1, sid1 = config1_inputs(N)
        s1 = OcpSolver(N=N, batch=len(x1), sqp_iters=K, qp_iters=args.qp_iters, device=gpu, nlp_solver_type=args.nlp)
        s1.set_shapes([make_shape("santal")], shape_id=sid1)
        s1.set_reference_trajectory(traj1)
        s1.controller_solve(x1, 1)
        s1.synchronize()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(10):
            s1.controller_reset()
            s1.controller_solve(x1, 1)
        result["configs1"] = {"workload": "BASELINE configs[1]: batch=4096 santal, N=20, K=50 SQP-RTI, cold start",
                              "gpu_solves_per_s": len(x1) * 10 / (time.perf_counter() - t1),
                              "note": "host-boundary controller solves (x0 in, u0 out), 10 repeats"}
        u1_gpu = s1.get_u0()
        s1.close()

    if rank == 0 and world == 1 and not args.no_configs4 and not cfg4 and args.nlp == "SQP_RTI":
        # BASELINE configs[4] beside the headline: N = 50, B = 16 384, curved x_finals reference with a
        # random start index per lane (bench.py --config 4 measures it as the main line)
        x4, _, _, sid4, traj4, idx4b = config4_inputs(16384, 50, args.seed)
        s4 = OcpSolver(N=50, batch=len(x4), sqp_iters=K, qp_iters=args.qp_iters, device=gpu)
        s4.set_shapes([make_shape(n) for n in SHAPES])
        s4.set_shape_ids(sid4)
        s4.set_reference_trajectory(traj4)
        s4.controller_solve(x4, idx4b)
        s4.synchronize()
        t4 = time.perf_counter()
        for _ in range(3):
            s4.controller_reset()
            s4.controller_solve(x4, idx4b)
        s4.synchronize()
        S4, L4 = s4.layout()
        result["configs4"] = {"workload": "BASELINE configs[4]: batch=16384, N=50, curved x_finals reference, random "
                                          "start index per lane, 4 shapes mixed per lane, K=50 SQP-RTI, cold start",
                              "gpu_solves_per_s": len(x4) * 3 / (time.perf_counter() - t4),
                              "layout": {"stages_per_lane": S4, "lanes_per_instance": L4,
                                         "factor_walk": s4.factor_walk()},
                              "note": "host-boundary controller solves (x0 in, u0 out), 3 repeats"}
        u4_gpu = s4.get_u0()
        # the factorisation-scan option (qsp_options.factor_scan) on the same workload: its rate, and its
        # u0 against the default's (it rounds differently: two digits less accurate)
        s4s = OcpSolver(N=50, batch=len(x4), sqp_iters=K, qp_iters=args.qp_iters, device=gpu, factor_scan=True)
        s4s.set_shapes([make_shape(n) for n in SHAPES])
        s4s.set_shape_ids(sid4)
        s4s.set_reference_trajectory(traj4)
        s4s.controller_solve(x4, idx4b)
        s4s.synchronize()
        t4s = time.perf_counter()
        for _ in range(3):
            s4s.controller_reset()
            u4_scan = s4s.controller_solve(x4, idx4b)
        s4s.synchronize()
        dsc = np.abs(u4_scan - u4_gpu).max(1)
        result["configs4"]["factor_scan"] = {"gpu_solves_per_s": len(x4) * 3 / (time.perf_counter() - t4s),
                                             "frac_u0_within_1e-6_of_default": float(np.mean(dsc <= 1e-6)),
                                             "status_equal_lanes": int(np.sum(s4s.get("status") == s4.get("status"))),
                                             "factor_walk": s4s.factor_walk()}
        s4s.close()
        # the GPU's own response to the literal parity leg's 1e-13 x0 probes (untimed)
        gpu_dev4 = np.zeros(len(x4))
        for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
            s4.controller_reset()
            gpu_dev4 = np.maximum(gpu_dev4, np.abs(s4.controller_solve(x4 * (1 + sgn * f * 1e-13), idx4b) - u4_gpu).max(1))
        s4.close()

    if rank == 0 and world == 1 and not args.no_closed_loop and not cfg4 and args.nlp == "SQP_RTI":
        result["side_rows"] = side_rows_measure(gpu, args.no_cpu)
        # SURVEY §8(f) row 1 beside the headline: main.m's closed loop, batched (bench.py --closed-loop
        # measures it alone, over 65 536 lanes by default)
        result["closed_loop"] = closed_loop_measure(16384, args.seed, 1, max(3.0, args.cpu_seconds / 3), args.no_cpu,
                                                    device=gpu)

    if rank == 0 and world == 1 and not args.no_cpu and not cfg4:
        hc = host_cpu()
        threads = hc["threads"]
        nlp_mode = 1 if args.nlp == "SQP" else 0
        # CPU baseline: the twin in its fastest CPU order (the same algorithm and formulation, the
        # factorisation as the lane walk's 4x4 algebra, OpenMP over lanes); the matrix-core order, which
        # the CPU can only emulate, is timed beside it (it is the bit-exact checker below)
        n, dt, rt, run_t = cpu_baseline(x0, traj, sid, N, K, args.cpu_seconds, threads, nlp_mode, twin=True,
                                        qp_iters=args.qp_iters, lane_walk=1)
        result["cpu_baseline"] = {"value": n / dt, "unit": "solves/s", "cores": threads, "kind": "port",
                                  "host_nproc": hc["nproc"], "host_affinity_cpus": hc["affinity_cpus"],
                                  "host_cgroup_cpu_quota": hc["cgroup_cpus"], "cpu_model": hc["model"],
                                  "sample": f"{n} lanes of the same workload (oracle/qsp_twin.c: the library's "
                                            f"formulation on the CPU, factorisation in the lane walk's order, OpenMP "
                                            f"over {threads} threads, {dt:.1f} s)"}
        nm, dtm, _, _ = cpu_baseline(x0, traj, sid, N, K, max(3.0, args.cpu_seconds / 3), threads, nlp_mode,
                                     twin=True, qp_iters=args.qp_iters)
        result["cpu_baseline"]["mfma_order_twin"] = {
            "value": nm / dtm, "unit": "solves/s", "cores": threads,
            "sample": f"{nm} lanes: the twin emulating the matrix cores' rounding order (the bit-exact checker; "
                      "not the CPU's best formulation)"}
        result["cpu_baseline"]["thread_scaling"] = thread_scaling(run_t, n / dt, threads, hc["affinity_cpus"])
        # bit-exact parity: every lane of the batch against the twin (the CPU sample above included)
        from oracle.oracle import Oracle, make_opts
        tw = Oracle(SHAPES, twin=True)
        tp = time.perf_counter()
        rt_all = tw.controller_solve(make_opts(N=N, sqp_iters=K, nlp_mode=nlp_mode, qp_iters=args.qp_iters), x0, traj, 1, tw.new_warm(Bl, N),
                                     shape_id=sid, nthreads=threads)
        tp = time.perf_counter() - tp
        same_u0 = np.all(u0 == rt_all["u0"], axis=1)
        result["parity"] = {"reference": "oracle/qsp_twin.c (kernel-order restatement, every FMA explicit)",
                            "lanes": int(Bl), "bit_identical_u0_lanes": int(same_u0.sum()),
                            "max_abs_u0_err": float(np.abs(u0 - rt_all["u0"]).max()),
                            "status_equal_lanes": int(np.sum(status_all[lo:hi] == rt_all["status"])),
                            "qp_iter_equal_lanes": int(np.sum(qp_iter == rt_all["qp_iter"])),
                            "cpu_seconds": tp}
        # the literal restatement on the first lanes, with its own sensitivity as the yardstick
        lit_s = max(3.0, args.cpu_seconds / 3)
        nl, dtl, rl, run_l = cpu_baseline(x0, traj, sid, N, K, lit_s, threads, nlp_mode, twin=False,
                                        qp_iters=args.qp_iters)
        result["cpu_literal_oracle"] = {"value": nl / dtl, "unit": "solves/s", "cores": threads,
                                        "sample": f"{nl} lanes (oracle/qsp_oracle.c: full basis sum, forward AD)"}
        pl = parity_leg(u0, x0, traj, sid, N, K, nl, rl, run_l, args.nlp, gpu_dev, qp_iters=args.qp_iters)
        # the GPU equals the twin, so its differences from the literal restatement are the two CPU
        # formulations' differences (span-based de Boor + hand-derived Jacobian vs basis sum + AD)
        pl["twin_vs_literal_max_abs_u0_err"] = float(np.abs(rt_all["u0"][:nl] - rl["u0"]).max())
        result["parity_literal"] = pl
        # the independent parity in one place beside the bit-exact one: agreement with the literal
        # restatement, and how the disagreements that survive every probe are adjudicated in __float128
        ep = pl.get("extended_precision", {})
        sb = ep.get("stable_in_both", {})
        ps = pl.get("probe_stable_in_both", {})
        es = ep.get("extended_stable", {})
        # the metric max|u0 - u0_ref| against the independent restatement, on three strata, at the top of
        # `parity` (max_abs_u0_err above is against the twin, a consistency check of the kernel's order)
        result["parity"]["max_abs_u0_err_vs_twin"] = result["parity"]["max_abs_u0_err"]
        result["parity"]["max_abs_u0_err_vs_literal"] = {
            "all_lanes": {"lanes": pl["lanes"], "max": pl["max_abs_u0_err"], "frac_le_1e-6": pl["frac_lanes_err_le_1e-6"]},
            "probe_stable_in_both": {"lanes": ps.get("lanes"), "max": ps.get("max_abs_u0_err"),
                                     "frac_le_1e-6": ps.get("frac_err_le_1e-6")},
            "extended_stable_vs_quad": {"lanes": es.get("lanes", 0), "max": es.get("max_abs_u0_err_gpu_vs_quad"),
                                        "literal_max": es.get("max_abs_u0_err_literal_vs_quad"),
                                        "note": "adjudicated sample only (disagreeing lanes first, then agreeing "
                                                "controls) where long double and __float128 agree to 1e-6: u0_ref = quad"}}
        result["parity"]["independent"] = {
            "reference": "oracle/qsp_oracle.c (literal restatement), adjudicated by its __float128 build",
            "lanes": pl["lanes"], "frac_within_1e-6": pl["frac_lanes_err_le_1e-6"],
            "literal_self_frac_within_1e-6": pl["oracle_self_frac_le_1e-6"],
            "disagreeing_stable_in_both": sb.get("lanes", 0),
            "of_those_quad_sides_with_gpu": sb.get("sides_with_gpu", 0),
            "of_those_quad_sides_with_literal": sb.get("sides_with_literal", 0)}
        if "configs1" in result:
            # configs[1] on the CPU in full (the twin: rate and bit-for-bit parity of every lane)
            x1, traj1, sid1 = config1_inputs(N)
            tc = time.perf_counter()
            r1 = tw.controller_solve(make_opts(N=N, sqp_iters=K, nlp_mode=nlp_mode, qp_iters=args.qp_iters), x1, traj1, 1,
                                     tw.new_warm(len(x1), N), shape_id=sid1, nthreads=threads)
            dtc = time.perf_counter() - tc
            result["configs1"].update({"cpu_solves_per_s": len(x1) / dtc, "cpu_seconds": dtc, "cpu_threads": threads,
                                       "cpu_kind": "port (oracle/qsp_twin.c, the full batch)",
                                       "bit_identical_u0_lanes": int(np.sum(np.all(u1_gpu == r1["u0"], axis=1))),
                                       "lanes": int(len(x1))})
        if "configs4" in result:
            # configs[4]: every lane against the twin (N = 50: the two-stages-per-lane layout's order)
            t4c = time.perf_counter()
            r4 = tw.controller_solve(make_opts(N=50, sqp_iters=K, qp_iters=args.qp_iters), x4, traj4, idx4b, tw.new_warm(len(x4), 50),
                                     shape_id=sid4, nthreads=threads)
            result["configs4"].update({"lanes": int(len(x4)), "cpu_seconds": time.perf_counter() - t4c,
                                       "bit_identical_u0_lanes": int(np.sum(np.all(u4_gpu == r4["u0"], axis=1))),
                                       "status_nonzero_lanes": int(np.count_nonzero(r4["status"]))})
            # and the literal restatement on the first 1 024 lanes, with its probes and the extended-
            # precision adjudication of the disagreements (as parity_literal above)
            n4 = min(1024, len(x4))
            _, _, r4l, run4 = cpu_baseline(x4[:n4], traj4, sid4[:n4], 50, K, 0.0, threads, 0, twin=False,
                                           qp_iters=args.qp_iters, idx=idx4b[:n4], sample=n4)
            pl4 = parity_leg(u4_gpu[:n4], x4[:n4], traj4, sid4[:n4], 50, K, n4, r4l, run4, "SQP_RTI_N50",
                             gpu_dev4[:n4], qp_iters=args.qp_iters, ext_lanes=16)
            result["configs4"]["parity_literal"] = pl4
    if rank == 0:
        if nbad:
            print(f"bench: WARNING {nbad} of {total} lanes returned a non-zero status", file=sys.stderr)
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
