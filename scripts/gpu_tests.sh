# GPU test suite + a short bench, one gpurun call (each step under its own time limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
grep -E "^FAILED" gpurun_out/gpu_tests.log || true
if [ "${BENCH:-1}" = "1" ] && [ $rc -ne 124 ] && [ $rc -ne 137 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
  echo "bench rc=$?"
  cat gpurun_out/bench_quick.json
fi
