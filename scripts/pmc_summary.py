"""Summarise rocprofv3 --pmc CSV passes per kernel (developer tool) and, with --json,
write the HBM traffic of the dominant kernel per launch (profiles/pmc_traffic.json,
read by bench.py's roofline.traffic).

Units/corrections (MI355X_MICROARCH.md, HBM section): rocprofv3's FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled; WRITE_SIZE is taken as is.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uclv_qs_pushing_matlab_amd.build import source_digest  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
ap.add_argument("--json", default=None)
ap.add_argument("--kernel", default="qp_step_kernel")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--N", type=int, default=20)
ap.add_argument("--sqp-iters", type=int, default=50)
ap.add_argument("--qp-iters", type=int, default=20, help="QP iteration cap of the profiled solves (bench.py default)")
ap.add_argument("--parts", type=int, default=2, help="stream parts of the profiled solves (bench.py layout)")
args = ap.parse_args()

tot = collections.defaultdict(lambda: collections.defaultdict(float))
ndisp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"{args.root}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ndisp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k, d in tot.items():
    if "qsp" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        n = len(ndisp[k][c])
        print(f"   {c:28s} total {v:.4e}   per launch {v / n:.4e}  ({n} launches)")

if args.json:
    ks = [k for k in tot if args.kernel in k]
    assert ks, f"no {args.kernel} dispatches"
    # per SQP iteration over the whole batch: with --parts 2 every iteration is two half
    # launches (one per stream), so the per-dispatch counters are summed over `parts` dispatches
    fetch = sum(tot[k]["FETCH_SIZE"] for k in ks) / (sum(len(ndisp[k]["FETCH_SIZE"]) for k in ks) / args.parts)
    write = sum(tot[k]["WRITE_SIZE"] for k in ks) / (sum(len(ndisp[k]["WRITE_SIZE"]) for k in ks) / args.parts)
    rd, wr = fetch * 1024 * 2, write * 1024
    out = {"kernel": args.kernel, "batch": args.batch, "N": args.N, "sqp_iters": args.sqp_iters,
           "qp_iters": args.qp_iters, "stream_parts": args.parts, "per": "SQP iteration over the whole batch (= bench roofline launch)",
           "hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
           "raw_FETCH_SIZE_KiB": fetch, "raw_WRITE_SIZE_KiB": write,
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count), WRITE_SIZE KiB x 1024",
           "kernel_digest": source_digest()}
    json.dump(out, open(args.json, "w"), indent=1)
    print(json.dumps(out))
