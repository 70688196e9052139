#!/bin/bash
# round 6: 9-stage A ring for 64-row NT tiles: x3 tests, then B = 4 / 8 bench lines against the previous library
# (KAIR_LIB=base: the same sources before the change)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x3_gpu.py tests/test_swinir_variants_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A12 "Error\|assert" $O/t.log | head -50; exit $rc; fi
B="python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for lib in new base new base; do
  for b in 4 8; do
    if [ $lib = base ]; then export KAIR_LIB=base; else unset KAIR_LIB; fi
    timeout -k 10 300 $B --per-gpu-batch $b > $O/b${b}_$lib.txt 2>&1 || { echo "b$b $lib failed"; tail -3 $O/b${b}_$lib.txt; exit 1; }
    echo "b$b $lib $(grep -o '"value": [0-9.]*' $O/b${b}_$lib.txt)"
  done
done
unset KAIR_LIB
echo done
