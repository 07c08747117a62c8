#!/bin/bash
# Throughput of both lane layouts (stages per lane S = 1, 2) at several horizons (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/sweep
for cfg in "10 65536" "20 65536" "50 16384"; do
  set -- $cfg
  for S in 1 2; do
    timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --N $1 --batch $2 --stages-per-lane $S \
      > gpurun_out/sweep/N$1_S$S.json 2> gpurun_out/sweep/N$1_S$S.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/sweep/N$1_S$S.json'));print('N=$1 B=$2 S=$S', round(d['value']), 'solves/s', round(d['kernels_ms_avg']['qp_step'],3), 'ms/qp_step')"
  done
done
