#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 350 --timeout-method thread tests/test_swinir_gpu.py -k "psnr_along or eval" > gpurun_out/r4l_tests.log 2>&1; grep -E "PASS|FAIL|Error|assert|^step" gpurun_out/r4l_tests.log | head -40
