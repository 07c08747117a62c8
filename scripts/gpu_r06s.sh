#!/bin/bash
# Round 6, step s: the matrix-core closed-loop walk for some of the three walks only, to balance VALU issue
# (lane walks) against LDS traffic (matrix-core walks): aw1 = the predictor's forward walk, aw2 = also
# the corrector's difference walk; fwb = all three on the VALU.  Interleaved A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06s
mkdir -p $R
for round in 1 2; do
  for v in fwb aw1 aw2; do
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
