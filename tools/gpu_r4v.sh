#!/bin/bash
# binned bias-table gradient: attention tests, engine tests, B = 32 / B = 4 bench lines, B = 4 roles
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_swinir_gpu.py tests/test_swinir_variants_gpu.py > gpurun_out/r4v_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4v_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4v_tests.log | head; exit 1; }
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
timeout -k 10 300 $B > gpurun_out/r4v_b32.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4v_b32.log | cut -c1-200
timeout -k 10 300 $B --global-batch 4 > gpurun_out/r4v_b4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/r4v_b4.log | cut -c1-200
timeout -k 10 200 python -u tools/roles.py 4 > gpurun_out/r4v_roles4.txt 2>&1; grep -E "attn|dtable" gpurun_out/r4v_roles4.txt
