#!/bin/bash
# Perf iteration on the GPU box: gpu tests, bench at the N=1 config (B=32) and at the per-GPU shape
# of the N=8 config (B=4), with extra args from $BENCH_EXTRA; GEMM micro-benchmark.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b32.log 2>&1 || { echo "bench32 failed"; exit 1; }
timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b4.log 2>&1 || { echo "bench4 failed"; exit 1; }
KAIR_RING_MIN_TILES=0 timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b4ring.log 2>&1 || { echo "bench4ring failed"; exit 1; }
timeout -k 10 120 python tools/gemm_micro.py --no-torch > gpurun_out/gm.log 2>&1 || { echo "micro failed"; exit 1; }
if [ -n "$PROFILE" ]; then
  R=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof32 -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/p32.log 2>&1 || { echo "profile32 failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o run -- \
    python3 $R/bench.py --global-batch 4 --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/p4.log 2>&1 || { echo "profile4 failed"; exit 1; }
  cd $R
fi
echo done
