#!/bin/bash
# One PMC pass per library variant on the bench workload (developer tool): per-kernel counter
# totals of qp_step_kernel for A/B comparisons.  VARIANTS="variants/a.so variants/b.so"
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"}
for v in $VARIANTS; do
  n=$(basename $v .so)
  mkdir -p gpurun_out/abpmc/$n
  QSP_LIB_PATH=$PWD/$v timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/abpmc/$n/p1 -o p1 -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 1 --warmup 0 > gpurun_out/abpmc/$n/log 2>&1 || exit $?
  echo "== $n"
  python scripts/pmc_summary.py gpurun_out/abpmc/$n | grep -A12 "qp_step_kernel<1"
done
