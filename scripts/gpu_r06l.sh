#!/bin/bash
# Round 6 final rehearsal: smoke, every GPU test, the default bench line,
# configs[3]'s per-GPU shard (B = 32 768), configs[4] (walk and the factorisation-scan option).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06l
mkdir -p $R
export TMPDIR=/tmp
echo "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { cat $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
echo "gpu tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 1; }
tail -2 $R/tests.log
echo "bench"
timeout -k 10 900 python bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 1; }
python -c "import json; d=json.load(open('$R/bench.json')); print('bench', round(d['value']), d['roofline']['frac'], d['roofline']['traffic'], d['configs1']['gpu_solves_per_s'], d['configs4']['gpu_solves_per_s'], d['parity']['bit_identical_u0_lanes'])"
timeout -k 10 300 python bench.py --global-batch 32768 --no-cpu --steps 10 --warmup 2 > $R/cfg3_shard.json 2> $R/cfg3_shard.err || { tail -20 $R/cfg3_shard.err; exit 1; }
python -c "import json; d=json.load(open('$R/cfg3_shard.json')); print('cfg3 shard', round(d['value']))"
for v in walk scan; do
  f=""; [ $v = scan ] && f="--factor-scan"
  timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 5 --warmup 1 $f > $R/cfg4_$v.json 2> $R/cfg4_$v.err || { tail -20 $R/cfg4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$R/cfg4_$v.json')); print('cfg4 $v', round(d['value']), d['roofline']['frac'], d['roofline']['traffic'])"
done
