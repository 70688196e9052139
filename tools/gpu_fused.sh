# fused-kernel check on the GPU box: parity of the fused block kernels, micro timings, parity probe
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/f_test.log 2>&1 || exit 1
KAIR_SPLIT=1 timeout -k 10 120 python tools/fused_micro.py 32 50 > $R/gpurun_out/m32s.log 2>&1 || exit 1
KAIR_SPLIT=0 timeout -k 10 120 python tools/fused_micro.py 32 50 > $R/gpurun_out/m32.log 2>&1 || exit 1
KAIR_SPLIT=1 timeout -k 10 120 python tools/fused_micro.py 4 100 > $R/gpurun_out/m4s.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/parity_probe.py 25 > $R/gpurun_out/probe4.log 2>&1 || exit 1
echo ok
