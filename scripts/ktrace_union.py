"""qp_step time per SQP iteration from a rocprofv3 --kernel-trace CSV (developer tool).

With the SQP loop split over two HIP streams (qsp_set_stream_parts), the two half launches
of an SQP iteration run concurrently, so rocprof's per-kernel average is the duration of a
half launch that shares the chip with the other half.  The comparable figure to bench.py's
roofline.launch_ms_avg (fork -> join per SQP iteration) is the union of the qp_step busy
intervals divided by the number of SQP iterations (dispatches / parts).

    python scripts/ktrace_union.py <dir-or-kernel_trace.csv> [--parts 2] [--kernel qp_step_kernel]
"""
import argparse
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--parts", type=int, default=2)
ap.add_argument("--kernel", default="qp_step_kernel")
args = ap.parse_args()

files = [args.path] if os.path.isfile(args.path) else glob.glob(os.path.join(args.path, "**", "*kernel_trace.csv"),
                                                                 recursive=True)
assert files, f"no kernel_trace.csv under {args.path}"
iv = []
for f in files:
    for r in csv.DictReader(open(f)):
        if args.kernel in r["Kernel_Name"]:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
iv.sort()
assert iv, f"no {args.kernel} dispatches"
busy, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
n = len(iv)
iters = n / args.parts
mean = sum(e - s for s, e in iv) / n
print(f"{args.kernel}: {n} dispatches, mean dispatch {mean * 1e-6:.4f} ms; union of busy intervals "
      f"{busy * 1e-6:.3f} ms over {iters:.0f} SQP iterations = {busy / iters * 1e-6:.4f} ms per SQP iteration "
      f"({args.parts} parts)")
