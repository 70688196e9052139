#!/bin/bash
# round 6: B = 4 kernel trace of the current engine (step breakdown + timeline)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $O -o b4 -- \
  python3 $R/tools/prof_step.py 4 12 > $O/log.txt 2>&1 || { echo "trace failed"; tail -3 $O/log.txt; exit 1; }
cd $R
python3 tools/step_breakdown.py $O/b4_kernel_trace.csv 40 > $O/step_breakdown_b4.txt
head -3 $O/step_breakdown_b4.txt
echo done
