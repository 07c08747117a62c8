#!/bin/bash
# Round 5 profiles at the matrix-core-walk digest: kernel trace of the bench, the PMC passes (headline
# traffic record), configs[4]'s traffic record, and the same PMC passes with the lane walk
# (QSP_MFMA_WALK=0) for the A/B of the counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05j
mkdir -p $R
export TMPDIR=/tmp
echo "kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 3 --warmup 1 > $R/kt_bench.json 2> $R/kt_bench.err || exit $?
python scripts/ktrace_union.py $R/kt --parts 2 > $R/kt_union.txt || exit $?
cat $R/kt_union.txt
echo "pmc (headline)"
OUT=$R/pmc bash scripts/prof_pmc.sh || exit $?
echo "traffic (configs[4])"
OUT=$R/tr_cfg4 ARGS="--config 4 --no-cpu --steps 1 --warmup 0" JSON=$R/pmc_traffic_cfg4.json BATCH=16384 NN=50 PARTS=2 bash scripts/prof_traffic.sh || exit $?
echo "pmc (headline, lane walk)"
QSP_MFMA_WALK=0 OUT=$R/pmc_lane bash scripts/prof_pmc.sh || exit $?
echo "matrix-core busy"
mkdir -p $R/mfma
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/mfma/p1 -o p1 -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 1 --warmup 0 > $R/mfma/p1.log 2>&1 || exit $?
python scripts/pmc_summary.py $R/mfma > $R/mfma/summary.txt || exit $?
