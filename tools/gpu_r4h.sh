#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_wr_gpu.py > gpurun_out/r4h_tests.log 2>&1; grep -E "PASS|FAIL|Error|assert" gpurun_out/r4h_tests.log | head -30
