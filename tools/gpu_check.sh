# quick GPU check: the block / network parity tests + fused tests + backward micro
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_swinir_gpu.py tests/test_kernels_gpu.py tests/test_ops_gpu.py -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_chk.log 2>&1 || { tail -40 $R/gpurun_out/t_chk.log; exit 1; }
tail -2 $R/gpurun_out/t_chk.log
timeout -k 10 120 python tools/bwd_micro.py 32 30 2>/dev/null | tail -1
