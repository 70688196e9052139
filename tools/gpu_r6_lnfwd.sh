#!/bin/bash
# round 6: LayerNorm forward / narrow backward with two rows in flight per 16-lane group -- parity, C2 and the headline
set -o pipefail
R=$(pwd); O=$R/gpurun_out/lnbwd; mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_x3_gpu.py tests/test_full_configs_gpu.py tests/test_swinir_gpu.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 > $O/c2_$i.txt 2>&1 || { tail -5 $O/c2_$i.txt; exit 1; }
  echo "c2 $(grep -o '"patches_per_s": [0-9.]*' $O/c2_$i.txt)"
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles > $O/h_$i.txt 2>&1 || { tail -3 $O/h_$i.txt; exit 1; }
  echo "headline $(grep -o '"value": [0-9.]*' $O/h_$i.txt | head -1)"
done
echo done
