#!/bin/bash
# rocprofv3 kernel trace of a short bench run at per-GPU batch $B (default 4: the per-GPU shape of
# the N=8 strong-scaling run) + per-step breakdown -> gpurun_out/tr$B_breakdown.txt
set -o pipefail
B=${B:-4}
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr$B -o run -- \
  python3 $R/bench.py --global-batch $B --steps 8 --warmup 3 --no-cpu-baseline --no-fp32-line --no-other-configs --no-roles > $R/gpurun_out/tr$B.log 2>&1 || { echo "profile failed"; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/tr$B/run_kernel_trace.csv 6 > gpurun_out/tr${B}_breakdown.txt
rm -f gpurun_out/tr$B/run_kernel_trace.csv
echo done
