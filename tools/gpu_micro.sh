set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/fused_micro.py 32 50 > $R/gpurun_out/m32.log 2>&1 || exit 1
timeout -k 10 120 python tools/fused_micro.py 4 100 > $R/gpurun_out/m4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/mpmc -o run --output-format csv -- python3 $R/tools/fused_micro.py 32 5 > $R/gpurun_out/mpmc.log 2>&1 || exit 1
echo ok
