#!/bin/bash
# Round 6, step q: the matrix-core factorisation from N = 12 (four instances per wave) instead of N = 15:
# twin bit-identity across the horizons (11 lane walk, 12 and 14 matrix cores), the reported walk, then
# N = 12 and 14 with the lane walk (QSP_MFMA_WALK=0) against the matrix cores, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06q
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_twin.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "horizons_and_layouts or reports_its_factor_walk or lane_walk_switch" > $R/gpu_tests.txt 2>&1
rc=$?
tail -3 $R/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $R/gpu_tests.txt | head -20; exit $rc; }
for round in 1 2; do
  for N in 12 14; do
    for mw in 0 1; do
      QSP_MFMA_WALK=$mw timeout -k 10 300 python bench.py --N $N --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_${N}_$mw.json 2> $R/ab_${N}_$mw.err || exit $?
      python -c "import json;d=json.load(open('$R/ab_${N}_$mw.json'));print('N=$N mfma_walk=$mw', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['config']['layout']['factor_walk'])" | tee -a $R/ab.txt
    done
  done
done
