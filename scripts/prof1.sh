#!/bin/bash
# profiling pass 1: layout sweep, kernel trace, counter list
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
for S in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --stages-per-lane $S > gpurun_out/prof1/bench_S$S.json 2>gpurun_out/prof1/bench_S$S.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/kt -o kt -- python3 bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/prof1/kt.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof1/counters.txt 2>&1 || true
echo done
