#!/bin/bash
set -o pipefail
bash tools/gpu_tests.sh || exit 1
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4q_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4q_bench.log | cut -c1-200
timeout -k 10 300 $B --per-gpu-batch 4 > gpurun_out/r4q_bench4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4q_bench4.log | cut -c1-200
R=$(pwd); O=$R/gpurun_out/r4q; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o sq -- python3 $R/tools/prof_step.py 32 3 > $O/sq_log.txt 2>&1 || { echo "sq pass failed"; exit 1; }
echo done
