#!/bin/bash
# round 6: the 16-wide head layout (C2, head dim 10) -- kernel + engine parity, then C2 throughput A/B (pad 16 vs 32)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/hp16; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "window_attention" > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -3 $O/kern.txt
timeout -k 10 400 $T tests/test_full_configs_gpu.py -k "c2" -s > $O/c2.txt 2>&1 || { tail -30 $O/c2.txt; exit 1; }
grep "C2 bf16" $O/c2.txt; tail -2 $O/c2.txt
for hp in 16 32 16 32; do
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 --head-pad $hp > $O/b_$hp.txt 2>&1 || { tail -5 $O/b_$hp.txt; exit 1; }
  echo "head_pad $hp $(grep -o '"patches_per_s": [0-9.]*' $O/b_$hp.txt)"
done
echo done
