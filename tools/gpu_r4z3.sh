#!/bin/bash
# 64-wide narrow weight-gradient tiles: tests, then base vs new on C5 / C2 / B = 32 (same box)
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_convnets_gpu.py tests/test_full_configs_gpu.py tests/test_usrnet_gpu.py tests/test_swinir_gpu.py tests/test_swinir_variants_gpu.py > gpurun_out/r4z3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4z3_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4z3_tests.log | head; exit 1; }
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for lib in base new; do
  KAIR_LIB=$lib timeout -k 10 300 python -u tools/bench_models.py rrdbnet swinir_light --steps 8 --warmup 3 > gpurun_out/r4z3_${lib}_m.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/r4z3_${lib}_m.log | cut -c1-80 | sed "s/^/$lib /"
  KAIR_LIB=$lib timeout -k 10 200 $B > gpurun_out/r4z3_${lib}_b32.log 2>&1 || exit 1
  echo "$lib B 32: $(grep -h '^{' gpurun_out/r4z3_${lib}_b32.log | cut -c80-115)"
done
