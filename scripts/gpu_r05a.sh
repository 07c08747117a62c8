#!/bin/bash
# Round 5, first session: the changed GPU test, configs[3]'s per-GPU shard (32 768 lanes, the 8-GPU
# split), and the default bench line with the stratified independent parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05a
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_errors.py tests/test_gpu_merit.py > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 1; }
tail -3 $R/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --global-batch 32768 --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 20 --warmup 3 > $R/bench_shard32k_$i.json 2> $R/bench_shard32k_$i.err || { tail -20 $R/bench_shard32k_$i.err; exit 1; }
  cat $R/bench_shard32k_$i.json
done
timeout -k 10 900 python bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 1; }
cat $R/bench.json
