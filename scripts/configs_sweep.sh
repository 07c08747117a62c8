#!/bin/bash
# Throughput at the BASELINE configurations (no CPU leg): configs[1] B = 4 096, configs[2]
# B = 65 536 (the bench), configs[3] per-GPU share B = 32 768 of 262 144 over 8 GPUs,
# configs[4] N = 50, B = 16 384; plus main.m's own controller (N = 10, merit SQP, max_iter 30).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/configs
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/configs/$name.json'));print('$name', round(d['value']), 'solves/s', round(d['ms_per_step'],2), 'ms/solve', 'frac', round(d['roofline']['frac'],4))"
}
run cfg1_B4096 --global-batch 4096
run cfg2_B65536 --global-batch 65536
run cfg3_B32768 --global-batch 32768
run cfg4_N50_B16384 --N 50 --global-batch 16384
run mainm_N10_SQP --N 10 --global-batch 65536 --nlp SQP --sqp-iters 30
