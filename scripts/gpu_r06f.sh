#!/bin/bash
# Round 6, step f: interleaved A/B of the select-free factor walk (fw) against its software-pipelined
# form (fw2, the in-tree library), then the full GPU suite and the default bench line on fw2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06f
mkdir -p $R
export TMPDIR=/tmp
for round in 1 2; do
  for v in fw fw2; do
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 5 --warmup 1 > $R/ab_$v.json 2> $R/ab_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab_$v.json'));print('$v', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 300 python bench.py --config 4 --no-cpu --steps 2 --warmup 1 > $R/ab4_$v.json 2> $R/ab4_$v.err || exit $?
    python -c "import json;d=json.load(open('$R/ab4_$v.json'));print('$v cfg4', round(d['value']), round(d['kernels_ms_avg']['qp_step'],4), d['status_nonzero_lanes'])" | tee -a $R/ab.txt
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpu_tests.txt 2>&1
rc=$?
tail -3 $R/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $R/bench.json 2> $R/bench.err || exit $?
python -c "import json;d=json.load(open('$R/bench.json'));print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['mfma_order_twin']['value'], d.get('configs2_qp50'), d['config']['layout'])"
