#!/bin/bash
# Round 6, step c: where a wave's time goes in the headline QP kernel (s_memtime segments, diagnostic
# build), and PMC of the round-5 kernel against the matrix-core closed-loop walks (aw1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06c
mkdir -p $R
export TMPDIR=/tmp
QSP_LIB_PATH=$PWD/variants/seg.so timeout -k 10 300 python scripts/segstamps.py --json $R/seg.json > $R/seg.txt 2>&1 || { cat $R/seg.txt; exit 1; }
cat $R/seg.txt
A="--no-cpu --no-configs1 --no-configs4 --no-closed-loop --no-qp50 --steps 1 --warmup 0"
for v in base aw1; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    QSP_LIB_PATH=$PWD/variants/$v.so timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/pmc_$v/p$i -o p$i -- python3 bench.py $A > $R/pmc_${v}_p$i.log 2>&1 || exit $?
    echo "$v pass $i done"
  done
  python scripts/pmc_summary.py $R/pmc_$v > $R/pmc_summary_$v.txt 2>&1 || exit $?
done
grep -A20 "qp_step_kernel" $R/pmc_summary_base.txt | head -22
grep -A20 "qp_step_kernel" $R/pmc_summary_aw1.txt | head -22
