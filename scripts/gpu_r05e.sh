#!/bin/bash
# Round 5: the factorisation scan at N = 20 (two stages per lane, opt-in) against the default layout, at the
# headline batch and at configs[1]'s B = 4 096 (fused small-batch loop), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r05e
mkdir -p $R
for rep in 1 2; do
  for v in s1 s2 s2scan; do
    a=""; [ $v = s2 ] && a="--stages-per-lane 2"; [ $v = s2scan ] && a="--stages-per-lane 2 --factor-scan"
    for b in 65536 4096; do
      timeout -k 10 300 python bench.py --no-cpu --no-configs1 --no-configs4 --no-closed-loop --global-batch $b --steps 5 --warmup 1 $a > $R/${v}_$b.$rep.json 2> $R/${v}_$b.$rep.err || { tail -5 $R/${v}_$b.$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$R/${v}_$b.$rep.json')); print('$v B=$b', round(d['value']), round(d['kernels_ms_avg']['qp_step'] or 0, 4), d['config']['layout'])"
    done
  done
done
