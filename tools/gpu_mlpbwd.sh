set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_swinir_gpu.py -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_mb.log 2>&1 || { tail -40 $R/gpurun_out/t_mb.log; exit 1; }
tail -1 $R/gpurun_out/t_mb.log
for f in 1 0; do
  KAIR_FUSED_MLP_BWD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/q32_$f.log 2>&1 || { echo "b32 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$R/gpurun_out/q32_$f.log').read().strip().split(chr(10))[-1]); print('fused_mlp_bwd=$f', d['value'], d['ms_per_step'], d['psnr']['bf16_delta_db'], d['psnr']['uint8_bf16_delta_db'])"
done
