#!/bin/bash
# Round 5: matrix-core factor walk (QSP_MFMA_WALK=1) against the lane walk, interleaved, plus the
# v_mfma_f64_4x4x4 rounding probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 60 scripts/ubench/mfma_f64_round 30000 > gpurun_out/mfma_round.txt 2>&1 || exit 1
cat gpurun_out/mfma_round.txt
for rep in 1 2; do
  for mw in 0 1; do
    QSP_MFMA_WALK=$mw timeout -k 10 200 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps ${STEPS:-5} --warmup 1 > gpurun_out/mfw_$mw.json 2> gpurun_out/mfw_$mw.err || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/mfw_$mw.json'))
pa=d.get('parity',{})
print('mfw=$mw', round(d['value']), round(d['kernels_ms_avg']['qp_step'],3), 'status_nonzero', d['status_nonzero_lanes'], 'vs twin', pa.get('max_abs_u0_err'), pa.get('frac_lanes_err_le_1e-6'), 'literal', pa.get('max_abs_u0_err_vs_literal'))
" | tee -a gpurun_out/mfw_ab.txt
  done
done
