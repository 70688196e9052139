#!/bin/bash
# round 6: where a B = 4 fp32x3 step goes (the N = 8 per-GPU shape): the bench line at per-GPU batch 4 under
# rocprofv3 --kernel-trace --stats
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6i; mkdir -p $O
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b4 -- \
  python3 $R/bench.py --per-gpu-batch 4 --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_b4_line.txt 2> $P/bench_b4_err.txt || { echo "stats pass failed"; tail -5 $P/bench_b4_err.txt; exit 1; }
cd $R
grep -o '"value": [0-9.]*' $P/bench_b4_line.txt | head -1
echo done
