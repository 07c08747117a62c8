#!/bin/bash
# A/B of configs[4] (N = 50, two stages per lane): the current library vs the previous build kept
# as uclv_qs_pushing_matlab_amd/libqsp_nmpc_prev.so (QSP_LIB selects it).  No CPU legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=${R:-gpurun_out/ab_cfg4}
mkdir -p $R
for v in new prev new prev; do
  if [ $v = prev ]; then export QSP_LIB_PATH=$PWD/uclv_qs_pushing_matlab_amd/libqsp_nmpc_prev.so; else unset QSP_LIB_PATH; fi
  timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 3 --warmup 1 --dump-u0 $R/u0_$v.npz > $R/cfg4_$v.json 2> $R/cfg4_$v.err || { tail -20 $R/cfg4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$R/cfg4_$v.json')); print('$v', d['value'], d['kernels_ms_avg']['qp_step'])"
done
python -c "
import numpy as np
a=np.load('$R/u0_new.npz'); b=np.load('$R/u0_prev.npz')
d=np.abs(a['u0']-b['u0']).max(1)
print('u0 new vs prev: bit-identical', int(np.sum(d==0)), 'of', len(d), 'within 1e-9', int(np.sum(d<=1e-9)), 'within 1e-6', int(np.sum(d<=1e-6)), 'status equal', int(np.sum(a['status']==b['status'])))
"
