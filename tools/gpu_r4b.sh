#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r4b_dist.log 2>&1 || { tail -30 gpurun_out/r4b_dist.log; exit 1; }
grep -E "params|PASS|FAIL" gpurun_out/r4b_dist.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4b_bench.log 2>&1 || { tail -20 gpurun_out/r4b_bench.log; exit 1; }
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/r4b_roles32.txt 2>&1 && timeout -k 10 200 python -u tools/roles.py 4 > gpurun_out/r4b_roles4.txt 2>&1
echo OK
