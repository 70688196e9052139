#!/bin/bash
# round 6: side-stream workgroup cap A/B with the grouped fp32x3 weight gradients, B = 32 and B = 4
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6l; mkdir -p $O
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for c in 192 0 144 96 -2 -4; do
  timeout -k 10 300 $B --side-ctas $c > $O/b32_$c.txt 2>&1 || exit 1
  echo "B32 side-ctas $c $(grep -o '"value": [0-9.]*' $O/b32_$c.txt)"
  timeout -k 10 300 $B --side-ctas $c --per-gpu-batch 4 > $O/b4_$c.txt 2>&1 || exit 1
  echo "B4 side-ctas $c $(grep -o '"value": [0-9.]*' $O/b4_$c.txt)"
done
echo done
