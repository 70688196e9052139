#!/bin/bash
# round 6: measurement tests, then the bench line (kernel table from a gated eager pass) under rocprofv3
# --kernel-trace --stats; tools/roofline_check.py compares the line with the summary.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_measure_gpu.py -x -v --timeout 60 --timeout-method thread > $O/t_meas.log 2>&1
rc=$?; tail -6 $O/t_meas.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
cd $R
python3 tools/roofline_check.py $P/bench_line.txt $P/stats/b_kernel_stats.csv
echo done
