#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_swinir_variants_gpu.py tests/test_swinir_gpu.py > gpurun_out/r4t_tests.log 2>&1; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r4t_tests.log | head -10
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4t_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4t_bench.log | cut -c1-200
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4t_roles32.txt 2>&1; grep -E "l1_loss|conv3x3_wr" gpurun_out/r4t_roles32.txt
