#!/bin/bash
# SQ-block counters over the training step (B = 32): where each kernel's waves spend their cycles
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4p; rm -rf $O; mkdir -p $O
timeout -k 10 200 python -u tools/roles.py 4 > $O/roles4.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o sq -- python3 $R/tools/prof_step.py 32 3 > $O/sq_log.txt 2>&1 || { echo "sq pass failed"; tail -5 $O/sq_log.txt; exit 1; }
echo pmc done
