#!/bin/bash
# One GPU session: smoke, GPU tests, kernel-trace stats, PMC passes, configs[4], full bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=${R:-gpurun_out/round}
mkdir -p $R
export TMPDIR=/tmp
echo "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { cat $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
if [ -z "$SKIP_TESTS" ]; then
  echo "gpu tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 1; }
  tail -2 $R/tests.log
fi
if [ -z "$SKIP_PROF" ]; then
  echo "kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 3 --warmup 1 > $R/kt_bench.json 2> $R/kt_bench.err || exit $?
  python scripts/ktrace_union.py $R/kt --parts 2 > $R/kt_union.txt || exit $?
  cat $R/kt_union.txt
  echo "pmc"
  OUT=$R/pmc bash scripts/prof_pmc.sh || exit $?
  cp $R/pmc/pmc_traffic.json profiles/pmc_traffic.json
fi
echo "configs[4]"
timeout -k 10 600 python bench.py --config 4 --no-cpu --steps 5 --warmup 1 > $R/bench_cfg4.json 2> $R/bench_cfg4.err || { tail -20 $R/bench_cfg4.err; exit 1; }
cat $R/bench_cfg4.json
echo "bench"
timeout -k 10 900 python bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 1; }
cat $R/bench.json
