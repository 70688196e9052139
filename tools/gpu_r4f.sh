#!/bin/bash
# halo conv micro: timings, then SQ / GRBM and FETCH PMC passes (separate runs)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4f; rm -rf $O; mkdir -p $O
timeout -k 10 120 python -u tools/conv_micro.py 20 > $O/conv_micro.txt 2>&1 || { tail -20 $O/conv_micro.txt; exit 1; }
cat $O/conv_micro.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o sq -- python3 $R/tools/conv_micro.py 3 > $O/sq_log.txt 2>&1 || { echo "sq pass failed"; tail -5 $O/sq_log.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/f -o f -- python3 $R/tools/conv_micro.py 3 > $O/f_log.txt 2>&1 || { echo "fetch pass failed"; tail -5 $O/f_log.txt; exit 1; }
find $O -name "*counter_collection*"
echo done
