# GPU test suite + a bench run, one gpurun call (each step under its own time limit).
# BENCH=0: tests only; BENCH=1: quick bench (no CPU leg); BENCH=full: the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
grep -E "^FAILED" gpurun_out/gpu_tests.log || true
if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
case "${BENCH:-1}" in
  1) timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
     echo "bench rc=$?"; cat gpurun_out/bench_quick.json ;;
  full) timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
     echo "bench rc=$?"; cat gpurun_out/bench_full.json ;;
esac
