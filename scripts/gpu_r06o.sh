#!/bin/bash
# Round 6, step o: what the three closed-loop lane walks cost per IPM iteration: head / IPM / tail stamps
# with the walks (segH) and with the walk loops compiled out (segHnw, -DQSP_NOWALK: wrong results, timing
# only), plus the unstamped pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06o
mkdir -p $R
for v in fwb nowalk segH segHnw; do
  echo "== $v" | tee -a $R/seg.txt
  QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python scripts/segstamps.py --json $R/seg_$v.json >> $R/seg.txt 2>&1 || { cat $R/seg.txt; exit 1; }
done
cat $R/seg.txt
