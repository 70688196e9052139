#!/bin/bash
# PMC passes over tools/fused_micro.py (B from $MB, default 4): one rocprofv3 run per counter set.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B=${MB:-4}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d $R/gpurun_out/pmcA -o run --output-format csv -- python3 $R/tools/fused_micro.py $B 5 > $R/gpurun_out/pmcA.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM -d $R/gpurun_out/pmcB -o run --output-format csv -- python3 $R/tools/fused_micro.py $B 5 > $R/gpurun_out/pmcB.log 2>&1 || exit 1
echo ok
