#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_wr_gpu.py > gpurun_out/r4g_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r4g_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/conv_micro.py 20 > gpurun_out/r4g_micro.txt 2>&1; cat gpurun_out/r4g_micro.txt
cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4g; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o sq -- python3 $R/tools/conv_micro.py 3 > $O/sq_log.txt 2>&1 || { echo "sq pass failed"; tail -5 $O/sq_log.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/tc -o tc -- python3 $R/tools/conv_micro.py 3 > $O/tc_log.txt 2>&1 || { echo "tc pass failed"; tail -5 $O/tc_log.txt; exit 1; }
echo pmc done
