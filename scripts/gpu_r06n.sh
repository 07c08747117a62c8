#!/bin/bash
# Round 6, step n: where the QP kernel's IPM time goes besides the factorisation, each group of segments
# stamped alone (the stamps distort less when few): kernel head / IPM / tail (segH), the factorisation
# (segF), the three closed-loop lane walks (segW: predictor forward, corrector difference, corrector
# forward), the stage-parallel segments (segP: iteration head, barrier terms, affine and corrector
# directions and steps).  In-tree library = the unstamped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06n
mkdir -p $R
for v in tree segH segF segW segP; do
  echo "== $v" | tee -a $R/seg.txt
  L=""; [ $v = tree ] || L=$PWD/variants/$v.so
  QSP_LIB_PATH=$L timeout -k 10 300 python scripts/segstamps.py --json $R/seg_$v.json >> $R/seg.txt 2>&1 || { cat $R/seg.txt; exit 1; }
done
cat $R/seg.txt
