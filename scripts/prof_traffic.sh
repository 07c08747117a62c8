#!/bin/bash
# HBM traffic of the QP kernel on one workload: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; kernel
# trace only) and the per-launch record (scripts/pmc_summary.py --json).  Env: OUT, ARGS (bench.py),
# JSON (record path), BATCH, NN (horizon), PARTS.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/traffic}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || exit $?
  echo "traffic pass $i done"
done
python scripts/pmc_summary.py $OUT --json ${JSON:-$OUT/traffic.json} --batch ${BATCH:-65536} --N ${NN:-20} --parts ${PARTS:-2} > $OUT/summary.txt
