#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 350 --timeout-method thread tests/test_swinir_gpu.py tests/test_conv_wr_gpu.py > gpurun_out/r4k_tests.log 2>&1; grep -E "PASS|FAIL|Error|assert|^step" gpurun_out/r4k_tests.log | head -40
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line"
timeout -k 10 300 $B > gpurun_out/r4k_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4k_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('psnr'))"
timeout -k 10 300 $B --per-gpu-batch 4 --no-psnr > gpurun_out/r4k_bench4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4k_bench4.log | cut -c1-200
timeout -k 10 300 $B --no-psnr --split-linear > gpurun_out/r4k_bench_sl.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4k_bench_sl.log | cut -c1-200
