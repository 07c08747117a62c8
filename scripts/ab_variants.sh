#!/bin/bash
# A/B the compiled variants in variants/*.so on the bench workload (developer tool).
# ARGS: extra bench.py arguments (e.g. "--stream-parts 1"); STEPS: timed solves per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for v in ${VARIANTS:-variants/*.so}; do
  QSP_LIB_PATH=$PWD/$v timeout -k 10 200 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps ${STEPS:-5} --warmup 1 ${ARGS} > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', '${ARGS}', round(d['value']), round(d['kernels_ms_avg']['qp_step'],3), d['status_nonzero_lanes'])"
done
