#!/bin/bash
# S=2 closed-loop composite walks: configs[4] A/B against the scan build, then the twin/config4 GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r04h
R=gpurun_out/r04h bash scripts/gpu_ab_cfg4.sh > gpurun_out/r04h/ab.txt 2>&1 || { cat gpurun_out/r04h/ab.txt; exit 1; }
cat gpurun_out/r04h/ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_twin.py tests/test_gpu_config4.py tests/test_gpu_fullsize.py > gpurun_out/r04h/tests.log 2>&1; rc=$?
tail -25 gpurun_out/r04h/tests.log
exit $rc
