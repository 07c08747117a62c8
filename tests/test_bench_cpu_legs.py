"""CPU: bench.py's CPU legs (no GPU): the host facts, the sampled CPU baseline with its thread
scaling, and the extended-precision adjudication of a disagreeing lane, with the twin standing in
for the device (the device equals it bit for bit, tests/test_gpu_twin.py)."""
import json
import os

import numpy as np

from conftest import GOLDEN


def test_host_facts_and_thread_scaling():
    import bench
    hc = bench.host_cpu()
    assert {"nproc", "affinity_cpus", "model", "threads", "cgroup_cpus"} <= set(hc)
    x0, _, _, sid, traj = bench.make_inputs(64, 20, bench.SEED)
    n, dt, r, run = bench.cpu_baseline(x0, traj, sid, 20, 5, 0.0, 2, sample=32)
    assert n == 32 and dt > 0 and r["u0"].shape == (32, 2)
    ts = bench.thread_scaling(run, n / dt, 2, 256, seconds=0.05)
    assert ts["threads"] == [1, 2] and all(v > 0 for v in ts["solves_per_s"])
    assert ts["full_host_estimate"]["cpus"] == 256
    np.testing.assert_allclose(ts["full_host_estimate"]["solves_per_s"], n / dt / 2 * 256)


def test_extended_adjudication_sides_with_the_gpu_on_the_stable_lane():
    """Lane 4 891 of the bench sample: stable under every probe in both implementations, 0.1 apart in
    u0; the __float128 literal restatement sides with the device's formulation."""
    import bench
    g = json.load(open(os.path.join(GOLDEN, "ext_adjudication_c2.json")))
    lane = next(l for l in g["lanes"] if l["stable_under_all_probes"])
    assert lane["lane"] == 4891
    x0, _, _, sid, traj = bench.make_inputs(65536, 20, bench.SEED)
    pick = np.array([lane["lane"]])
    _, _, r, run = bench.cpu_baseline(x0[pick], traj, sid[pick], 20, 50, 0.0, 1, twin=False, sample=1)
    u_gpu = np.array([lane["u0_twin"]])
    np.testing.assert_array_equal(r["u0"], [lane["u0_literal"]])
    out = bench.extended_adjudication(u_gpu, r["u0"], run, [("stable_in_both", [0])], max_lanes=1)
    sb = out["stable_in_both"]
    assert sb["lanes"] == 1 and sb["sides_with_gpu"] == 1 and sb["ext_stable"] == 1
    assert sb["per_lane"][0]["gpu_err"] < 1e-12 and sb["per_lane"][0]["literal_err"] > 0.09


def test_parity_leg_strata():
    """The bench line's independent parity: max|u0 - u0_ref| against the literal restatement on all
    lanes, on the lanes stable under every probe of both implementations, and against __float128 on the
    extended-stable adjudicated lanes (the twin standing in for the device)."""
    import bench
    n, K = 12, 6
    x0, _, _, sid, traj = bench.make_inputs(n, 20, bench.SEED)
    _, _, rt, run_t = bench.cpu_baseline(x0, traj, sid, 20, K, 0.0, 2, sample=n)
    _, _, rl, run_l = bench.cpu_baseline(x0, traj, sid, 20, K, 0.0, 2, twin=False, sample=n)
    gdev = np.zeros(n)
    for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
        gdev = np.maximum(gdev, np.abs(run_t(slice(0, n), x0 * (1 + sgn * f * 1e-13))["u0"] - rt["u0"]).max(1))
    pl = bench.parity_leg(rt["u0"], x0, traj, sid, 20, K, n, rl, run_l, "SQP_RTI", gdev, ext_lanes=4)
    d = np.abs(rt["u0"] - rl["u0"]).max(1)
    assert pl["max_abs_u0_err"] == d.max()
    ps = pl["probe_stable_in_both"]
    assert 0 < ps["lanes"] <= n and ps["max_abs_u0_err"] <= d.max()
    es = pl["extended_precision"].get("extended_stable")
    assert es is None or (es["lanes"] >= 1 and es["max_abs_u0_err_gpu_vs_quad"] >= 0.0)
