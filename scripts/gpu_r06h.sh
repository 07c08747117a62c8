#!/bin/bash
# Round 6, step h: configs[1] with the fused SQP loop at one and at two waves per SIMD (QSP_MIN_WAVES=2
# build) against the per-iteration launches; then the PMC passes of the headline kernel (VALU, LDS, bank
# conflicts, traffic record at this digest).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06h
mkdir -p $R
export TMPDIR=/tmp
for round in 1 2; do
  timeout -k 10 200 python scripts/configs1_fused.py --tag per-iteration --u0 $R/u0_iter.npy | tee -a $R/configs1.txt || exit $?
  timeout -k 10 200 python scripts/configs1_fused.py --tag fused-1wave --fused 1 --u0 $R/u0_f1.npy | tee -a $R/configs1.txt || exit $?
  QSP_LIB_PATH=$PWD/variants/mw2.so timeout -k 10 200 python scripts/configs1_fused.py --tag fused-2waves --fused 1 --u0 $R/u0_f2.npy | tee -a $R/configs1.txt || exit $?
done
python -c "import numpy as np; a=np.load('$R/u0_iter.npy'); b=np.load('$R/u0_f1.npy'); c=np.load('$R/u0_f2.npy'); print('u0 fused-1wave == per-iteration:', np.array_equal(a,b), ' fused-2waves == per-iteration:', np.array_equal(a,c))" | tee -a $R/configs1.txt
OUT=$R/pmc bash scripts/prof_pmc.sh || exit $?
grep -A24 "qp_step_kernel" $R/pmc/summary.txt | head -26
