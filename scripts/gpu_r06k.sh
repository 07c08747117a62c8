#!/bin/bash
# Round 6 final digest, profiles: kernel trace of the headline, the headline PMC passes (traffic record),
# configs[4]'s traffic record; the records are installed under profiles/ so a later bench on this box
# reports traffic.  The rehearsal is scripts/gpu_r06l.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06k
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 3 --warmup 1 > $R/kt_bench.json 2> $R/kt_bench.err || exit $?
python scripts/ktrace_union.py $R/kt --parts 2 > $R/kt_union.txt || exit $?
cat $R/kt_union.txt
OUT=$R/pmc ARGS="--no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 1 --warmup 0" bash scripts/prof_pmc.sh || exit $?
OUT=$R/tr_cfg4 ARGS="--config 4 --no-cpu --steps 1 --warmup 0" JSON=$R/pmc_traffic_cfg4.json BATCH=16384 NN=50 PARTS=2 bash scripts/prof_traffic.sh || exit $?
cat $R/pmc/summary.txt $R/tr_cfg4/summary.txt
