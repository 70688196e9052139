set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py tests/test_swinir_gpu.py -x -q --timeout 240 --timeout-method thread -k "attention or window or swinir_classical_full or droppath or golden" > $R/gpurun_out/t_attn.log 2>&1 || { tail -30 $R/gpurun_out/t_attn.log; exit 1; }
tail -2 $R/gpurun_out/t_attn.log
timeout -k 10 120 python tools/attn_stamps.py 32 2>/dev/null | tail -1
timeout -k 10 120 python tools/bwd_micro.py 32 30 2>/dev/null | tail -1
