#!/bin/bash
# kernel trace + stats of the default bench config (one rocprofv3 pass, no counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/kt}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 bench.py --no-cpu --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS} > $OUT/bench.log 2>&1 || exit $?
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
