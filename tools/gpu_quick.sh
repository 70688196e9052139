#!/bin/bash
# bench at B=32 and B=4 (no CPU baseline) + a rocprofv3 kernel-trace summary of a short B=32 run.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/q32.log 2>&1 || { echo "b32 failed"; exit 1; }
timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/q4.log 2>&1 || { echo "b4 failed"; exit 1; }
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qprof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/qp.log 2>&1 || { echo "profile failed"; exit 1; }
fi
echo done
