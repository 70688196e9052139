#!/bin/bash
# Idle gaps between kernels in graph-replayed steps at per-GPU batch $B (default 4)
set -o pipefail
B=${B:-4}
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gp$B -o run -- \
  python3 $R/bench.py --global-batch $B --steps 8 --warmup 3 --no-cpu-baseline --no-fp32-line --no-other-configs --no-roles > $R/gpurun_out/gp$B.log 2>&1 || { echo "profile failed"; exit 1; }
cd $R
python3 tools/step_gaps.py gpurun_out/gp$B/run_kernel_trace.csv
rm -f gpurun_out/gp$B/run_kernel_trace.csv
