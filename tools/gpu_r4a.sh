#!/bin/bash
# round 4: split-activation engine -- kernel tests, the 160-step PSNR test, drift ablation, a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_split_gpu.py \
  tests/test_swinir_gpu.py > gpurun_out/r4a_tests.log 2>&1 || { tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line \
  > gpurun_out/r4a_bench.log 2>&1 || { tail -20 gpurun_out/r4a_bench.log; exit 1; }
timeout -k 10 300 python -u tools/drift_ablation.py 160 40 > gpurun_out/r4a_drift.log 2>&1 || { tail -20 gpurun_out/r4a_drift.log; exit 1; }
echo OK
