#!/bin/bash
# round 6 checkpoint: the whole GPU suite, smoke(), the default bench line (100 steps, every extra line), the
# per-GPU batch 16 / 8 / 4 lines, and a rocprofv3 --kernel-trace --stats pass of the headline bench step
# (tools/roofline_check.py compares the line's roofline with that summary).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6fin; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
rc=$?; tail -3 $O/t_all.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A15 "Error\|assert" $O/t_all.log | head -60; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python3 bench.py > $O/bench_default.txt 2> $O/bench_default_err.txt || { tail -5 $O/bench_default_err.txt; exit 1; }
echo "default $(grep -o '"value": [0-9.]*' $O/bench_default.txt | head -1)"
for b in 16 8 4; do
  timeout -k 10 300 python3 bench.py --per-gpu-batch $b --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs \
    --no-fp32-line --no-psnr > $O/bench_b$b.txt 2>&1 || { tail -3 $O/bench_b$b.txt; exit 1; }
  echo "b$b $(grep -o '"value": [0-9.]*' $O/bench_b$b.txt | head -1)"
done
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
cd $R
python3 tools/roofline_check.py $P/bench_line.txt $P/stats/b_kernel_stats.csv
python3 tools/step_breakdown.py $P/stats/b_kernel_trace.csv 30 > $O/step_breakdown_b32.txt
rm -f $P/stats/b_kernel_trace.csv
echo done
