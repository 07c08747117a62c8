#!/bin/bash
# Round 5: matrix-core factor walk (default) against the lane walk (QSP_MFMA_WALK=0), interleaved:
# the bench workload, configs[1] (B = 4 096, per-iteration launches) and a fused small batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for rep in 1 2; do
  for mw in 0 1; do
    QSP_MFMA_WALK=$mw timeout -k 10 200 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps ${STEPS:-5} --warmup 1 > gpurun_out/mfw_$mw.json 2> gpurun_out/mfw_$mw.err || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/mfw_$mw.json'))
print('bench mfw=$mw', round(d['value']), round(d['kernels_ms_avg']['qp_step'],3), 'status_nonzero', d['status_nonzero_lanes'])
" | tee -a gpurun_out/mfw_ab.txt
  done
done
for gb in 4096 2048; do
  for mw in 0 1; do
    QSP_MFMA_WALK=$mw timeout -k 10 200 python bench.py --global-batch $gb --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 5 --warmup 1 > gpurun_out/mfw_b${gb}_${mw}.json 2> gpurun_out/mfw_b${gb}_$mw.err || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/mfw_b${gb}_${mw}.json'))
print('B=$gb mfw=$mw', round(d['value']), 'status_nonzero', d['status_nonzero_lanes'])
" | tee -a gpurun_out/mfw_ab.txt
  done
done
