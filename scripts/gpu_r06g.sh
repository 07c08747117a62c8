#!/bin/bash
# Round 6, step g: the nine-product factor step (fw3, in-tree): twin bit-identity and parity tests,
# then an interleaved A/B against the eleven-product step (fw2) and the round-5 walk (base).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06g
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_twin.py tests/test_gpu_parity.py tests/test_gpu_config4.py -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpu_tests.txt 2>&1
rc=$?
tail -3 $R/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in base fw2 fw3; do
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 2 --warmup 1 > $R/ab4_$v.json 2> $R/ab4_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab4_$v.json'));print('$v cfg4', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
