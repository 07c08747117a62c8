#!/bin/bash
# Round 5: the S = 2 factorisation-scan option -- GPU tests (all), then configs[4] with and without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05b
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 1; }
tail -3 $R/tests.log
for v in walk scan walk scan; do
  f=""; [ $v = scan ] && f="--factor-scan"
  timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 5 --warmup 1 $f > $R/cfg4_$v.json 2> $R/cfg4_$v.err || { tail -20 $R/cfg4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$R/cfg4_$v.json')); print('$v', round(d['value']), d['kernels_ms_avg']['qp_step'], d['config']['layout'])"
done
