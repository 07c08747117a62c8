#!/bin/bash
# Round 6, step a: the closed-loop walks on the matrix cores.  GPU tests on the in-tree library (every
# twin/parity check of the matrix-core kernel), then an interleaved A/B against the round-5 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06a
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpu_tests.txt 2>&1
rc=$?
tail -3 $R/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in base aw; do
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'], d['u0_checksum'] if 'u0_checksum' in d else '')" | tee -a $R/ab.txt
  done
done
