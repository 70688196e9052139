#!/bin/bash
# round 6: rocprofv3 kernel traces of the B = 4 and B = 32 bench steps (grouped fp32x3 weight gradients)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6m; mkdir -p $O
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for b in 4 32; do
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b$b -- \
  python3 $R/bench.py --per-gpu-batch $b --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles \
  > $P/bench_b${b}_line.txt 2> $P/bench_b${b}_err.txt || { echo "stats pass failed"; tail -5 $P/bench_b${b}_err.txt; exit 1; }
grep -o '"value": [0-9.]*' $P/bench_b${b}_line.txt | head -1
done
echo done
