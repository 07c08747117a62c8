# GPU tests + quick bench + short kernel trace (developer loop)
set -o pipefail
mkdir -p gpurun_out/ktq
export TMPDIR=/tmp
BENCH=1 bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktq -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 3 --warmup 1 > gpurun_out/ktq/b.json 2> gpurun_out/ktq/b.err || exit $?
python scripts/ktrace_union.py gpurun_out/ktq --parts 2
head -4 gpurun_out/ktq/kt_kernel_stats.csv
