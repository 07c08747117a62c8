#!/bin/bash
# Fused SQP loop (sqp_loop_kernel, QSP_FUSED_LOOP=1) vs per-iteration launches at small batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/fused
for B in ${BATCHES:-1024 2048 3072 4096}; do
  for F in 0 1; do
    QSP_FUSED_LOOP=$F timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 --batch $B --stream-parts 1 > gpurun_out/fused/B${B}_F$F.json 2> gpurun_out/fused/B${B}_F$F.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/fused/B${B}_F$F.json'));print('B $B fused $F', round(d['value']), 'solves/s', round(d['ms_per_step'],2), 'ms/solve')"
  done
done
for F in 0 1; do
  QSP_FUSED_LOOP=$F timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 --batch 4096 --stages-per-lane 2 --stream-parts 1 > gpurun_out/fused/S2_B4096_F$F.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/fused/S2_B4096_F$F.json'));print('S2 B 4096 fused $F', round(d['value']), 'solves/s')"
done
