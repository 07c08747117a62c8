#!/bin/bash
# A/B two compiled libraries (developer tool): bit identity of one K = 50 controller solve on 8 192
# bench lanes, fused = per-iteration launches, then bench throughput (VARIANTS="a b", default base/new).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
A=${A:-base}; Bv=${Bv:-new}
mkdir -p gpurun_out/ab
for v in $A $Bv; do
  QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 120 python scripts/ab_solve.py gpurun_out/ab/$v.npz 8192 50 > /dev/null 2>&1 || exit 1
done
python -c "
import numpy as np
a=np.load('gpurun_out/ab/$A.npz'); b=np.load('gpurun_out/ab/$Bv.npz')
print('$A vs $Bv: u0 bit-identical:', np.array_equal(a['u0'], b['u0']), 'x:', np.array_equal(a['x'], b['x']), 'qp_iter:', np.array_equal(a['qp_iter'], b['qp_iter']))"
QSP_LIB_PATH=$PWD/variants/$Bv.so timeout -k 10 120 python scripts/fused_check.py 3072 2>&1 | grep -v amdgpu.ids || exit 1
for r in 1 2; do VARIANTS="variants/$A.so variants/$Bv.so" STEPS=10 bash scripts/ab_variants.sh || exit 1; done
