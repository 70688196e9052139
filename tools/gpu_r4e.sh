#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_fused_gpu.py tests/test_swinir_gpu.py tests/test_swinir_variants_gpu.py tests/test_tail_gpu.py tests/test_split_gpu.py > gpurun_out/r4e_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r4e_tests.log | head -30; tail -5 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4e_roles32.txt 2>&1
timeout -k 10 200 python -u tools/roles.py 4 > gpurun_out/r4e_roles4.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line > gpurun_out/r4e_bench.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --per-gpu-batch 4 > gpurun_out/r4e_bench4.log 2>&1
echo OK; grep -h "^{" gpurun_out/r4e_bench.log gpurun_out/r4e_bench4.log | cut -c1-300
timeout -k 10 200 python -u tools/b4_micro.py > gpurun_out/r4e_b4micro.txt 2>&1
echo MICRO
