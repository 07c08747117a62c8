#!/bin/bash
# quick GPU cycle: parity tests + layout sweep of the bench (no CPU leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?; tail -15 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
for S in ${LAYOUTS:-1 2}; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --stages-per-lane $S > gpurun_out/bench_S$S.json 2> gpurun_out/bench_S$S.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_S$S.json'));print('S=$S', round(d['value']), 'solves/s', round(d['kernel_ms_avg'],1), 'ms', 'frac', round(d['roofline']['frac'],4))"
done
