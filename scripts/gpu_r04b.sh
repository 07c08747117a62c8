#!/bin/bash
# r04 session b: the MEX gateway test, kernel-trace + PMC profiles of the bench, configs[4] at one and
# two stages per lane.  Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=${R:-gpurun_out/r04b}
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mex.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $R/mex.log 2>&1 || { tail -30 $R/mex.log; exit 1; }
tail -1 $R/mex.log
for S in 1 2; do
  timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 3 --warmup 1 --stages-per-lane $S > $R/cfg4_S$S.json 2> $R/cfg4_S$S.err || { tail -20 $R/cfg4_S$S.err; exit 1; }
  python -c "import json; d=json.load(open('$R/cfg4_S$S.json')); print('S=$S', d['value'], d['roofline']['frac'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 3 --warmup 1 > $R/kt_bench.json 2> $R/kt_bench.err || exit $?
python scripts/ktrace_union.py $R/kt --parts 2 > $R/kt_union.txt || exit $?
cat $R/kt_union.txt
OUT=$R/pmc bash scripts/prof_pmc.sh || exit $?
cp $R/pmc/pmc_traffic.json profiles/pmc_traffic.json
cat $R/pmc/summary.txt | head -40
