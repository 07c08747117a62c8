#!/bin/bash
# Round 5 profiles at the final kernel digest: kernel trace of the bench, the PMC passes (headline traffic
# record), configs[4]'s traffic record, and the wave-packing traffic/time A/B (QSP_PACKING=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05c
mkdir -p $R profiles/r05
export TMPDIR=/tmp
echo "kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 3 --warmup 1 > $R/kt_bench.json 2> $R/kt_bench.err || exit $?
python scripts/ktrace_union.py $R/kt --parts 2 > $R/kt_union.txt || exit $?
cat $R/kt_union.txt
echo "pmc (headline)"
OUT=$R/pmc bash scripts/prof_pmc.sh || exit $?
cp $R/pmc/pmc_traffic.json profiles/pmc_traffic.json
echo "traffic (configs[4])"
OUT=$R/tr_cfg4 ARGS="--config 4 --no-cpu --steps 1 --warmup 0" JSON=profiles/pmc_traffic_cfg4.json BATCH=16384 NN=50 PARTS=2 bash scripts/prof_traffic.sh || exit $?
echo "traffic (headline, packing off)"
QSP_PACKING=0 OUT=$R/tr_nopack ARGS="--no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 1 --warmup 0" JSON=profiles/r05/pmc_traffic_nopack.json bash scripts/prof_traffic.sh || exit $?
echo "time A/B packing on/off"
for v in on off on off; do
  if [ $v = off ]; then export QSP_PACKING=0; else unset QSP_PACKING; fi
  timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 10 --warmup 2 > $R/pack_$v.json 2> $R/pack_$v.err || { tail -5 $R/pack_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$R/pack_$v.json')); print('packing $v', round(d['value']), d['kernels_ms_avg']['qp_step'], d['roofline']['traffic'])"
done
