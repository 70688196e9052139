#!/bin/bash
# narrow weight-gradient tiles with >= 512-row splits: tests, then C5 RRDBNet base vs new (same box)
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_convnets_gpu.py tests/test_full_configs_gpu.py tests/test_usrnet_gpu.py > gpurun_out/r4z2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4z2_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4z2_tests.log | head; exit 1; }
for rep in 1 2; do for lib in base new; do
  KAIR_LIB=$lib timeout -k 10 200 python -u tools/bench_models.py rrdbnet --steps 8 --warmup 3 > gpurun_out/r4z2_${lib}_c5.log 2>&1 || exit 1
  echo "$lib C5: $(grep -h '^{' gpurun_out/r4z2_${lib}_c5.log | cut -c1-90)"
done; done
