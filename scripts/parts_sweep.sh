#!/bin/bash
# Stream parts of the SQP loop across batch sizes and NLP modes (no CPU leg); the data behind
# sqp_parts_auto.  PARTS / BATCHES override the sweep.  (3 and 4 parts, measured slower than one
# part at every size before the library was capped at two -- DESIGN.md section 4.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/parts
PARTS=${PARTS:-"1 2"}
BATCHES=${BATCHES:-"4096 8192 16384 32768 65536"}
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 "$@" > gpurun_out/parts/$name.json 2> gpurun_out/parts/$name.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/parts/$name.json'));print('$name', round(d['value']), 'solves/s', round(d['ms_per_step'],2), 'ms/solve')"
}
for B in $BATCHES; do
  for P in $PARTS; do run B${B}_P$P --batch $B --stream-parts $P; done
done
for P in $PARTS; do run N50_B16384_P$P --N 50 --batch 16384 --stream-parts $P; done
for P in $PARTS; do run SQP_B65536_P$P --nlp SQP --sqp-iters 30 --stream-parts $P; done
for P in $PARTS; do run mainm_N10_SQP_P$P --N 10 --batch 65536 --nlp SQP --sqp-iters 30 --stream-parts $P; done
