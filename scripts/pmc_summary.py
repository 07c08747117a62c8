"""Summarise rocprofv3 --pmc CSV passes per kernel (developer tool)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((f, r["Dispatch_Id"]))
for k, d in tot.items():
    if "qsp" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:.4e}")
