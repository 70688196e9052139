#!/bin/bash
# 32 x 160 narrow weight-gradient tile (K <= 160): tests, then base vs new on C3 USRNet (same box)
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_convnets_gpu.py tests/test_usrnet_gpu.py > gpurun_out/r4z4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4z4_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4z4_tests.log | head; exit 1; }
for lib in base new; do
  KAIR_LIB=$lib timeout -k 10 300 python -u tools/bench_models.py usrnet --steps 5 --warmup 3 > gpurun_out/r4z4_${lib}.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/r4z4_${lib}.log | cut -c1-90 | sed "s/^/$lib /"
done
