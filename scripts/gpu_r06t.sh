#!/bin/bash
# Round 6, step t: PMC of configs[4] (N = 50, B = 16 384, two stages per lane) at the final digest:
# VALU, LDS, bank conflicts, wave and busy cycles of the QP kernel (one pass, kernel trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=gpurun_out/r06t
mkdir -p $R
export TMPDIR=/tmp
A="--config 4 --no-cpu --steps 1 --warmup 0"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/pmc/p1 -o p1 -- python3 bench.py $A > $R/pmc_p1.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d $R/pmc/p2 -o p2 -- python3 bench.py $A > $R/pmc_p2.log 2>&1 || exit $?
python scripts/pmc_summary.py $R/pmc > $R/pmc_summary.txt 2>&1 || exit $?
grep -A20 "qp_step_kernel" $R/pmc_summary.txt | head -22
