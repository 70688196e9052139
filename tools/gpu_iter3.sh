#!/bin/bash
# Iteration record: -m gpu tests, short bench lines at B=32 and B=4, rocprofv3 per-step breakdowns.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; echo "tests failed"; exit 1; }
tail -1 gpurun_out/t.log
Q="--no-cpu-baseline --no-fp32-line --no-other-configs"
timeout -k 10 300 python bench.py --steps 30 --warmup 10 $Q > gpurun_out/b32.log 2>&1 || { tail -20 gpurun_out/b32.log; echo "bench failed"; exit 1; }
tail -1 gpurun_out/b32.log | cut -c1-400
timeout -k 10 300 python bench.py --global-batch 4 --steps 50 --warmup 10 $Q > gpurun_out/b4.log 2>&1 || { tail -20 gpurun_out/b4.log; echo "bench4 failed"; exit 1; }
tail -1 gpurun_out/b4.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr32 -o run -- \
  python3 $R/bench.py --steps 8 --warmup 3 $Q > $R/gpurun_out/tr32.log 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr4 -o run -- \
  python3 $R/bench.py --global-batch 4 --steps 8 --warmup 3 $Q > $R/gpurun_out/tr4.log 2>&1 || { echo "profile4 failed"; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/tr32/run_kernel_trace.csv 6 > gpurun_out/b32_breakdown.txt
python3 tools/step_breakdown.py gpurun_out/tr4/run_kernel_trace.csv 6 > gpurun_out/b4_breakdown.txt
rm -f gpurun_out/tr4/run_kernel_trace.csv gpurun_out/tr32/run_kernel_trace.csv
head -16 gpurun_out/b32_breakdown.txt; head -16 gpurun_out/b4_breakdown.txt
echo done
