#!/bin/bash
# A/B of two-stage-per-lane (S = 2) kernel variants in variants/*.so (developer tool):
# configs[4] (N = 50, B = 16 384) and the bench workload at S = 2 (N = 20), u0 dumped per variant
# and compared bit for bit against the first variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ab_s2
first=""
for v in ${VARIANTS:-variants/*.so}; do
  n=$(basename $v .so)
  QSP_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --config 4 --no-cpu --steps ${STEPS:-3} --warmup 1 \
    --dump-u0 gpurun_out/ab_s2/$n.c4.npz > gpurun_out/ab_s2/$n.c4.json 2> gpurun_out/ab_s2/$n.c4.err || { tail -5 gpurun_out/ab_s2/$n.c4.err; exit 1; }
  QSP_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --stages-per-lane 2 \
    --steps ${STEPS:-3} --warmup 1 --dump-u0 gpurun_out/ab_s2/$n.c2.npz > gpurun_out/ab_s2/$n.c2.json 2> gpurun_out/ab_s2/$n.c2.err || { tail -5 gpurun_out/ab_s2/$n.c2.err; exit 1; }
  python - "$n" "$first" <<'EOF'
import json, sys
import numpy as np
n, first = sys.argv[1], sys.argv[2]
out = [n]
for c in ("c4", "c2"):
    d = json.load(open(f"gpurun_out/ab_s2/{n}.{c}.json"))
    out += [c, round(d["value"]), round(d["kernels_ms_avg"]["qp_step"], 3)]
    if first:
        a = np.load(f"gpurun_out/ab_s2/{first}.{c}.npz")
        b = np.load(f"gpurun_out/ab_s2/{n}.{c}.npz")
        out += ["u0 bit-identical" if np.array_equal(a["u0"], b["u0"]) else "u0 DIFFERS"]
print(*out)
EOF
  [ -z "$first" ] && first=$n
done
