#!/bin/bash
# A/B two compiled libraries in merit-SQP mode (developer tool): bench.py --nlp SQP --sqp-iters 30
# twice each, then bit identity of the gathered u0/status (A=name B=name of variants/<name>.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
A=${A:-base}; Bv=${Bv:-new}
mkdir -p gpurun_out/abls
for r in 1 2; do
  for v in $A $Bv; do
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 200 python bench.py --nlp SQP --sqp-iters 30 --no-cpu --no-configs1 \
      --no-configs4 --steps 5 --warmup 1 ${EXTRA} --dump-u0 gpurun_out/abls/$v.npz > gpurun_out/abls/$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abls/$v.json'));print('$v', round(d['value']))"
  done
done
python -c "
import numpy as np
a=np.load('gpurun_out/abls/$A.npz'); b=np.load('gpurun_out/abls/$Bv.npz')
print('merit u0 bit-identical:', np.array_equal(a['u0'], b['u0']), 'status:', np.array_equal(a['status'], b['status']))"
