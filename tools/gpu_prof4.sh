#!/bin/bash
# rocprofv3 kernel trace of a short B=4 bench run (the per-GPU shape of the N=8 strong-scaling
# run) + per-step breakdown.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr4 -o run -- \
  python3 $R/bench.py --global-batch 4 --steps 8 --warmup 3 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/tr4.log 2>&1 || { echo "profile4 failed"; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/tr4/run_kernel_trace.csv 6 > gpurun_out/tr4_breakdown.txt
rm -f gpurun_out/tr4/run_kernel_trace.csv
echo done
