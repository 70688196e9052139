#!/bin/bash
# full GPU suite, then bench at B=32 (fused MLP on / off) and B=4, then a rocprofv3 kernel-trace summary.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_full.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/t_full.log; exit 1; }
tail -3 $R/gpurun_out/t_full.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/q32.log 2>&1 || { echo "b32 failed"; exit 1; }
KAIR_FUSED_MLP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/q32u.log 2>&1 || { echo "b32u failed"; exit 1; }
timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/q4.log 2>&1 || { echo "b4 failed"; exit 1; }
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qprof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/qp.log 2>&1 || { echo "profile failed"; exit 1; }
fi
echo done
