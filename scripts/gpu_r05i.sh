#!/bin/bash
# Round 5: the matrix-core walk with the symmetric P — parity and twin tests, then the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_twin.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_i.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_i.log | tail -2
grep -E "^FAILED|^E  " gpurun_out/gpu_tests_i.log | head -20 || true
if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
bash scripts/gpu_r05h.sh
