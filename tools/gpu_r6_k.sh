#!/bin/bash
# round 6: grouped fp32x3 block weight gradients (one TN-ring launch per RSTB): kernel + engine parity tests, then
# bench lines grouped vs per-linear (KAIR_X3_GROUPED=0) at B = 32 and B = 4
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x3_gpu.py tests/test_x3_range_gpu.py tests/test_swinir_variants_gpu.py tests/test_dist_gpu.py tests/test_measure_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B5 "Error\|assert" $O/t.log | head -40; exit $rc; fi
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for gr in 1 0; do
  KAIR_X3_GROUPED=$gr timeout -k 10 300 $B > $O/b32_$gr.txt 2>&1 || exit 1
  echo "B32 grouped=$gr $(grep -o '"value": [0-9.]*' $O/b32_$gr.txt)"
  KAIR_X3_GROUPED=$gr timeout -k 10 300 $B --per-gpu-batch 4 > $O/b4_$gr.txt 2>&1 || exit 1
  echo "B4 grouped=$gr $(grep -o '"value": [0-9.]*' $O/b4_$gr.txt)"
done
echo done
