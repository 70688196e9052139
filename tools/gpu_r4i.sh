#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_swinir_gpu.py -k "psnr_along or segmented or golden" > gpurun_out/r4i_tests.log 2>&1; grep -E "PASS|FAIL|Error|assert" gpurun_out/r4i_tests.log | head -20
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4i_bench.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4i_bench.log | cut -c1-200
timeout -k 10 300 $B --conv-wr-min-tiles -1 > gpurun_out/r4i_bench_nowr.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4i_bench_nowr.log | cut -c1-200
timeout -k 10 300 $B --per-gpu-batch 4 > gpurun_out/r4i_bench4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4i_bench4.log | cut -c1-200
timeout -k 10 300 $B --per-gpu-batch 4 --conv-wr-min-tiles 0 > gpurun_out/r4i_bench4_wr.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4i_bench4_wr.log | cut -c1-200
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4i_roles32.txt 2>&1; head -16 gpurun_out/r4i_roles32.txt
