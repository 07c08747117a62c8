#!/bin/bash
# Round 6, step d: the segment stamps' own distortion (all segments / factor walk only / kernel head,
# IPM, tail only) against the unstamped library's wall time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06d
mkdir -p $R
for v in base segH segF seg; do
  echo "== $v" | tee -a $R/seg.txt
  QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python scripts/segstamps.py --json $R/seg_$v.json >> $R/seg.txt 2>&1 || { cat $R/seg.txt; exit 1; }
done
cat $R/seg.txt
