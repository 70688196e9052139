#!/bin/bash
# round 6: grouped fp32x3 weight gradients in place (--no-side-stream) vs on the side stream; side-ctas 96 vs 192
# at B = 4 / 8 / 16
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6n; mkdir -p $O
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
run() {   # label, args
  local l=$1; shift
  timeout -k 10 300 $B "$@" > $O/$l.txt 2>&1 || { echo "$l failed"; tail -3 $O/$l.txt; exit 1; }
  echo "$l $(grep -o '"value": [0-9.]*' $O/$l.txt)"
}
run b32_side
run b32_inplace --no-side-stream
run b4_side --per-gpu-batch 4
run b4_inplace --per-gpu-batch 4 --no-side-stream
run b4_c96 --per-gpu-batch 4 --side-ctas 96
run b8_side --per-gpu-batch 8
run b8_c96 --per-gpu-batch 8 --side-ctas 96
run b16_side --per-gpu-batch 16
run b16_c96 --per-gpu-batch 16 --side-ctas 96
echo done
