#!/bin/bash
# Round 5: the S = 2 factorisation scan in the leading IPM iterations only -- twin bit-identity and the
# configs[4] parity tests, then configs[4] throughput per factor_scan setting (interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05d
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_twin.py -k "factor_scan or qp_bit or configs4" > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 1; }
tail -2 $R/tests.log
for rep in 1 2; do
  for fs in 0 4 255 3 5; do
    timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 5 --warmup 1 --factor-scan $fs --dump-u0 $R/u0_$fs.npz > $R/cfg4_$fs.$rep.json 2> $R/cfg4_$fs.$rep.err || { tail -20 $R/cfg4_$fs.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$R/cfg4_$fs.$rep.json')); print('factor_scan $fs', round(d['value']), round(d['kernels_ms_avg']['qp_step'], 4), d['qp_iters_mean_per_qp'])"
  done
done
