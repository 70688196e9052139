#!/bin/bash
# Standard GPU-box check (run through gpurun from the repo root):
#   tests -m gpu, smoke, bench (N=1), rocprofv3 kernel-trace stats of a short bench.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 30 --warmup 10} > gpurun_out/b.log 2>&1 || { echo "bench failed"; exit 1; }
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/p.log 2>&1 || { echo "profile failed"; exit 1; }
fi
echo done
