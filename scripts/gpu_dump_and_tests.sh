set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tests/tools/dump_config2.py && BENCH=1 bash scripts/gpu_tests.sh
