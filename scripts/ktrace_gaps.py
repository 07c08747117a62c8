"""Idle gaps between kernels in a rocprofv3 --kernel-trace CSV (developer tool).

Sorts every dispatch by start time, merges overlapping intervals, and reports the device-busy
union, the wall span, and the idle gaps before each kernel name (count, mean, total): the
launch-boundary overhead of a per-iteration SQP loop.

    python scripts/ktrace_gaps.py <dir-or-kernel_trace.csv> [--skip-gap-us 1000]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--skip-gap-us", type=float, default=1000.0, help="gaps above this are host-side pauses, not counted")
args = ap.parse_args()

files = [args.path] if os.path.isfile(args.path) else glob.glob(os.path.join(args.path, "**", "*kernel_trace.csv"),
                                                                 recursive=True)
assert files, f"no kernel_trace.csv under {args.path}"
ks = []
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
ks.sort()
gaps = defaultdict(list)
busy = 0
cs, ce, _ = ks[0]
for s, e, name in ks[1:]:
    if s > ce:
        g = (s - ce) / 1e3
        if g <= args.skip_gap_us:
            gaps[name].append(g)
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
span = (ks[-1][1] - ks[0][0]) / 1e6
print(f"dispatches {len(ks)}  busy {busy / 1e6:.3f} ms  span {span:.3f} ms")
for name, g in sorted(gaps.items(), key=lambda t: -sum(t[1])):
    print(f"  gap before {name[:60]:60s} n={len(g):6d} mean {sum(g) / len(g):7.2f} us  total {sum(g) / 1e3:8.3f} ms")
dur = defaultdict(list)
for s, e, name in ks:
    dur[name].append((e - s) / 1e3)
for name, d in sorted(dur.items(), key=lambda t: -sum(t[1])):
    print(f"  kernel {name[:60]:60s} n={len(d):6d} mean {sum(d) / len(d):9.2f} us  total {sum(d) / 1e3:8.3f} ms")
