#!/bin/bash
# round 6: side-stream workgroup cap at the small per-GPU batches (grouped fp32x3 weight gradients): 48 / 64 / 96 / 128
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6t; mkdir -p $O
B="python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for c in 96 64 48 128; do
  for b in 4 8; do
    timeout -k 10 300 $B --per-gpu-batch $b --side-ctas $c > $O/b${b}_$c.txt 2>&1 || { echo "failed"; tail -3 $O/b${b}_$c.txt; exit 1; }
    echo "b$b side-ctas $c $(grep -o '"value": [0-9.]*' $O/b${b}_$c.txt)"
  done
done
echo done
