#!/bin/bash
# PMC counters for one gemm_micro case (run via gpurun from the repo root): tools/pmc_gemm.sh <case> [outdir]
set -e
C=${1:-qkv_fwd}; O=${2:-gpurun_out/pmc}
R=$(pwd); mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/$O -o p$N -- python3 $R/tools/gemm_micro.py $C --no-torch --reps 5 > $R/$O/log$N.txt 2>&1; N=$((N+1)); }
N=0
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
run FETCH_SIZE
run WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
