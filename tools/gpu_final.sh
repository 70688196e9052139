#!/bin/bash
# End-of-round GPU record: -m gpu tests, smoke, the default bench line, rocprofv3 kernel-trace stats
# at B=32 and a per-step breakdown at B=4, and the two PMC passes (HBM traffic) -> gpurun_out/
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; echo "tests failed"; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s.log 2>&1 || { tail gpurun_out/s.log; echo "smoke failed"; exit 1; }
tail -1 gpurun_out/s.log
timeout -k 10 600 python bench.py > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; echo "bench failed"; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --no-other-configs > $R/gpurun_out/p.log 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr4 -o run -- \
  python3 $R/bench.py --global-batch 4 --steps 8 --warmup 3 --no-cpu-baseline --no-fp32-line --no-other-configs > $R/gpurun_out/tr4.log 2>&1 || { echo "profile4 failed"; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv 5 > gpurun_out/b32_breakdown.txt
python3 tools/step_breakdown.py gpurun_out/tr4/run_kernel_trace.csv 6 > gpurun_out/tr4_breakdown.txt
rm -f gpurun_out/tr4/run_kernel_trace.csv gpurun_out/prof/run_kernel_trace.csv
head -3 gpurun_out/b32_breakdown.txt; head -3 gpurun_out/tr4_breakdown.txt
timeout -k 10 600 bash tools/gpu_pmc.sh || { echo "pmc failed"; exit 1; }
echo done
