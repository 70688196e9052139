#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_tail_gpu.py tests/test_split_gpu.py > gpurun_out/r4d_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" gpurun_out/r4d_tests.log | head -30; tail -5 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4d_roles32.txt 2>&1
echo OK
