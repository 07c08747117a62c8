#!/bin/bash
# Round 5: the matrix-core factorisation at two stages per lane (configs[4]) — twin tests, then the
# interleaved A/B against the lane walk (QSP_MFMA_WALK=0), then the headline (one stage per lane).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05m
mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_twin.py -m gpu -v -x -k "configs4 or horizons or qp_bit_identical or lane_walk_switch" --timeout 240 --timeout-method thread -p no:cacheprovider > $R/tests.log 2>&1
rc=$?
grep -E "passed|failed" $R/tests.log | tail -2
grep -E "^FAILED|^E  " $R/tests.log | head -20 || true
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mw in 0 1; do
    QSP_MFMA_WALK=$mw timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 5 --warmup 1 > $R/cfg4_$mw.json 2> $R/cfg4_$mw.err || { tail -5 $R/cfg4_$mw.err; exit 1; }
    python -c "import json; d=json.load(open('$R/cfg4_$mw.json')); print('cfg4 mfw=$mw', round(d['value']), round(d['kernels_ms_avg']['qp_step'],3), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 5 --warmup 1 > $R/bench.json 2> $R/bench.err || exit 1
python -c "import json; d=json.load(open('$R/bench.json')); print('bench', round(d['value']), round(d['kernels_ms_avg']['qp_step'],3))" | tee -a $R/ab.txt
