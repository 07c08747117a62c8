#!/bin/bash
# Round 6, step u: the instances' record regions at a bank-disjoint stride (mfw_stride; configs[4]'s two
# instances were 30 doubles apart mod 32, so their operand reads shared banks), in-tree: twin tests at
# two stages per lane, then an interleaved A/B against fwb on configs[4] and the headline, and a PMC pass
# on configs[4].
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06u
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_twin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $R/gpu_tests.txt 2>&1
rc=$?
tail -2 $R/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $R/gpu_tests.txt | head -20; exit $rc; }
for round in 1 2; do
  for v in fwb tree; do
    L=""; [ $v = tree ] || L=$PWD/variants/$v.so
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 3 --warmup 1 > $R/ab4_$v.json 2> $R/ab4_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab4_$v.json'));print('$v cfg4', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
A="--config 4 --no-cpu --steps 1 --warmup 0"
for v in fwb tree; do
  L=""; [ $v = tree ] || L=$PWD/variants/$v.so
  QSP_LIB_PATH=$L timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/pmc_$v/p1 -o p1 -- python3 bench.py $A > $R/pmc_$v.log 2>&1 || exit $?
  python scripts/pmc_summary.py $R/pmc_$v > $R/pmc_summary_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -A9 "qp_step_kernel" $R/pmc_summary_$v.txt | grep -E "VALU |INSTS_LDS|BANK|WAVE_CYCLES"
done
