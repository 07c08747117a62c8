#!/bin/bash
# Round 6, step m: one stream part against two, with the in-tree build (249 VGPRs: the packing sort
# cannot co-reside with two QP waves) and the round-5 walk (variants/base.so, 247 VGPRs: it can).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06m
mkdir -p $R
export TMPDIR=/tmp
for round in 1 2; do
  for v in tree base; do
    L=""; [ $v = base ] && L=$PWD/variants/base.so
    for P in 1 2; do
      QSP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 --stream-parts $P > $R/ab_${v}_$P.json 2> $R/ab_${v}_$P.err || exit $?
      python -c "import json;d=json.load(open('$R/ab_${v}_$P.json'));print('$v parts=$P', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4))" | tee -a $R/ab.txt
    done
  done
done
