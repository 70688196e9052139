#!/bin/bash
# finalize / split-sum with every partial-batch load in flight: tests, B = 32 / B = 4 lines, B = 32 roles
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_swinir_gpu.py tests/test_swinir_variants_gpu.py tests/test_conv_wr_gpu.py tests/test_convnets_gpu.py tests/test_full_configs_gpu.py -rA > gpurun_out/r4y_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4y_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4y_tests.log | head; exit 1; }
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for b in 32 4; do
  timeout -k 10 200 $B --global-batch $b > gpurun_out/r4y_b$b.log 2>&1 || exit 1
  echo "B $b: $(grep -h '^{' gpurun_out/r4y_b$b.log | cut -c80-125)"
done
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4y_roles32.txt 2>&1; grep -E "finalize|dtable|ln_param" gpurun_out/r4y_roles32.txt
timeout -k 10 300 python -u tools/bench_models.py rrdbnet swinir_light --steps 5 --warmup 3 > gpurun_out/r4y_models.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4y_models.log | cut -c1-160
