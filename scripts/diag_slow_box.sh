#!/bin/bash
# Developer tool: quick bench; on a box below 490k solves/s also the one-part rate and a kernel trace
# (the pool has boxes 9-13 % slower at the same build)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 5 --warmup 1 > gpurun_out/dq.json 2>/dev/null || exit 1
V=$(python -c "import json;print(int(json.load(open('gpurun_out/dq.json'))['value']))")
echo value=$V
if [ $V -lt 490000 ]; then
  timeout -k 10 200 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 5 --warmup 1 --stream-parts 1 > gpurun_out/dq1.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/dq1.json'));print('1 part', int(d['value']), d['kernels_ms_avg']['qp_step'])"
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dqkt -o kt -- python3 bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --steps 2 --warmup 1 > /dev/null 2>&1
  find gpurun_out/dqkt -name "*kernel_stats.csv" -exec head -4 {} \;
  python scripts/ktrace_union.py gpurun_out/dqkt --parts 2
fi
