#!/bin/bash
# r04 session c: PMC passes of the configs[4] kernel (qp_step_kernel<2, ...>), the closed-loop line and
# the merit-SQP line.  Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=${R:-gpurun_out/r04c}
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench/riccati_scan_s2 50 16384 10 36 > $R/riccati_scan_s2.txt 2>&1 || { cat $R/riccati_scan_s2.txt; exit 1; }
timeout -k 10 120 ./scripts/ubench/riccati_scan_s2 50 16384 10 0 >> $R/riccati_scan_s2.txt 2>&1 || { cat $R/riccati_scan_s2.txt; exit 1; }
cat $R/riccati_scan_s2.txt
OUT=$R/pmc_cfg4 ARGS="--config 4 --no-cpu --steps 1 --warmup 0" bash scripts/prof_pmc.sh || exit $?
head -60 $R/pmc_cfg4/summary.txt
timeout -k 10 600 python bench.py --closed-loop --steps 2 > $R/closed_loop.json 2> $R/closed_loop.err || { tail -20 $R/closed_loop.err; exit 1; }
python -c "import json; d=json.load(open('$R/closed_loop.json')); print('closed loop', d['value'], d.get('cpu_baseline', {}).get('value'))"
timeout -k 10 600 python bench.py --nlp SQP --sqp-iters 30 --qp-iters 50 --no-configs1 --no-closed-loop --steps 10 --cpu-seconds 6 > $R/merit.json 2> $R/merit.err || { tail -20 $R/merit.err; exit 1; }
python -c "import json; d=json.load(open('$R/merit.json')); print('merit', d['value'], d['status_nonzero_lanes'], d['parity']['bit_identical_u0_lanes'])"
