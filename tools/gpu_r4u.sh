#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_tail_gpu.py tests/test_conv_wr_gpu.py tests/test_split_gpu.py > gpurun_out/r4u_tests.log 2>&1; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r4u_tests.log | head -10
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4u_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4u_bench.log | cut -c1-200
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4u_roles32.txt 2>&1; grep -E "narrow|l1_loss|936|933" gpurun_out/r4u_roles32.txt
