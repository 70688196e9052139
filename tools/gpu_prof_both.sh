#!/bin/bash
# rocprofv3 kernel traces of short bench runs at B=32 and B=4 -> per-step breakdowns
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for B in 32 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pr$B -o run -- \
    python3 $R/bench.py --global-batch $B --steps 8 --warmup 3 --no-cpu-baseline --no-fp32-line --no-other-configs > $R/gpurun_out/pr$B.log 2>&1 || { echo "profile $B failed"; exit 1; }
  (cd $R && python3 tools/step_breakdown.py gpurun_out/pr$B/run_kernel_trace.csv 5 > gpurun_out/pr${B}_breakdown.txt && rm -f gpurun_out/pr$B/run_kernel_trace.csv)
done
cd $R; head -22 gpurun_out/pr32_breakdown.txt; head -16 gpurun_out/pr4_breakdown.txt
