#!/bin/bash
# rocprofv3 kernel-trace stats of short bench runs at B=32 (the N=1 config) and B=4 (the per-GPU
# shape of the N=8 strong-scaling run).
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof32 -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/p32.log 2>&1 || { echo "profile32 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o run -- \
  python3 $R/bench.py --global-batch 4 --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/p4.log 2>&1 || { echo "profile4 failed"; exit 1; }
echo done
