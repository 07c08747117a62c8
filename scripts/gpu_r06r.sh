#!/bin/bash
# Round 6, step r: the kernel head.  Stamps inside it (segK: iterate loads / RK4 + sensitivities / the
# rest) before and after reading the spline's span-search knots as one window (segK2), the twin and
# parity tests on the in-tree build (the window changes reads only), and an interleaved A/B against
# fwb, and the linearisation run twice (head2, -DQSP_HEAD2: what a head costs in throughput).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06r
mkdir -p $R
export TMPDIR=/tmp
for v in segH segK segK2; do
  echo "== $v" | tee -a $R/seg.txt
  QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 200 python scripts/segstamps.py 2>&1 | grep -v amdgpu.ids >> $R/seg.txt || exit 1
done
cat $R/seg.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $R/gpu_tests.txt 2>&1
rc=$?
tail -2 $R/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $R/gpu_tests.txt | head -20; exit $rc; }
for round in 1 2; do
  for v in fwb tree head2; do
    L=""; [ $v = tree ] || L=$PWD/variants/$v.so
    QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
