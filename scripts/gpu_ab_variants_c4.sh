#!/bin/bash
# Interleaved A/B of configs[4] (N = 50, B = 16 384, S = 2) over library variants in variants/*.so
# (developer tool): bench.py --config 4 per variant, twice in alternation, u0 compared with the first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=${R:-gpurun_out/ab_c4}
mkdir -p $R
VS=${VARIANTS:-$(ls variants/*.so)}
for rep in 1 2; do
  for v in $VS; do
    n=$(basename $v .so)
    QSP_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --config 4 --no-cpu --steps ${STEPS:-3} --warmup 1 \
      --dump-u0 $R/$n.npz > $R/$n.$rep.json 2> $R/$n.$rep.err || { tail -5 $R/$n.$rep.err; exit 1; }
    python - "$R" "$n" "$rep" $(basename $(echo $VS | cut -d' ' -f1) .so) <<'PY'
import json, sys
import numpy as np
R, n, rep, first = sys.argv[1:5]
d = json.load(open(f"{R}/{n}.{rep}.json"))
a, b = np.load(f"{R}/{first}.npz"), np.load(f"{R}/{n}.npz")
e = np.abs(a["u0"] - b["u0"]).max(1)
print(n, rep, round(d["value"]), "qp_step ms", round(d["kernels_ms_avg"]["qp_step"], 3),
      f"u0 vs {first}: identical {int((e == 0).sum())}, <=1e-9 {int((e <= 1e-9).sum())}, <=1e-6 {int((e <= 1e-6).sum())} of {len(e)}",
      "status equal", int((a["status"] == b["status"]).sum()), flush=True)
PY
  done
done
