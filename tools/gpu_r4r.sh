#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_conv_wr_gpu.py tests/test_swinir_gpu.py > gpurun_out/r4r_tests.log 2>&1; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r4r_tests.log | head -10
timeout -k 10 120 python -u tools/conv_micro.py 20 > gpurun_out/r4r_micro.txt 2>&1; grep -v amdgpu gpurun_out/r4r_micro.txt | grep wr
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4r_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4r_bench.log | cut -c1-200
timeout -k 10 300 $B --per-gpu-batch 4 > gpurun_out/r4r_bench4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4r_bench4.log | cut -c1-200
