#!/bin/bash
# Round 6, step p: the closed-loop walks on the matrix cores again (aff_walk_mfma, conflict-free
# layout: odd record stride, one writer lane per row), in-tree: every GPU test (the walks must stay
# bit-identical to the lane walk and so to the twin), an interleaved A/B against fwb (the lane walks),
# one PMC pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06p
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $R/gpu_tests.txt 2>&1
rc=$?
tail -3 $R/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $R/gpu_tests.txt | head -20; exit $rc; }
for round in 1 2; do
  for v in fwb tree; do
    L=""; [ $v = tree ] || L=$PWD/variants/$v.so
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
A="--no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 1 --warmup 0"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/pmc/p1 -o p1 -- python3 bench.py $A > $R/pmc_p1.log 2>&1 || exit $?
python scripts/pmc_summary.py $R/pmc > $R/pmc_summary.txt 2>&1 || exit $?
grep -A9 "qp_step_kernel" $R/pmc_summary.txt | head -10
