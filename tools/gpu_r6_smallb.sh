#!/bin/bash
# round 6 closing: per-GPU batch 16 / 8 / 4 lines (the 2 / 4 / 8-GPU strong-scaling shapes) after the C2 / LayerNorm work
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6smallb; mkdir -p $O
for b in 16 8 4; do
  timeout -k 10 300 python3 bench.py --per-gpu-batch $b --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs \
    --no-fp32-line --no-psnr > $O/bench_b$b.txt 2>&1 || { tail -3 $O/bench_b$b.txt; exit 1; }
  echo "b$b $(grep -o '"value": [0-9.]*' $O/bench_b$b.txt | head -1)"
done
echo done
