#!/bin/bash
# Round 6, step v: the group sums' partner values by DPP and row permutes instead of LDS shuffles (the
# same additions in the same order), in-tree: every GPU test (bit-identical to the twin), then an
# interleaved A/B against fin (the kept kernel) on the headline and configs[4].
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06v
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $R/gpu_tests.txt 2>&1
rc=$?
tail -2 $R/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $R/gpu_tests.txt | head -20; exit $rc; }
for round in 1 2; do
  for v in fin tree; do
    L=""; [ $v = tree ] || L=$PWD/variants/$v.so
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 3 --warmup 1 > $R/ab4_$v.json 2> $R/ab4_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab4_$v.json'));print('$v cfg4', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
