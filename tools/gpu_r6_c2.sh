#!/bin/bash
# round 6: where C2 (SwinIR-lightweight x2, head dim 10) spends its step -- kernel trace of tools/bench_models.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c2; mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 10 --warmup 4 > $O/line.txt 2>&1 || { tail -5 $O/line.txt; exit 1; }
grep config $O/line.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c2 -- python3 tools/bench_models.py swinir_light --steps 10 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" -print -quit)
python3 tools/step_breakdown.py $f 40 > $O/breakdown.txt && cat $O/breakdown.txt
