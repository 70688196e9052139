#!/bin/bash
# round 6: re-run of the fixed tests, then the headline bench line (graph-timed roofline) and a rocprofv3
# --kernel-trace --stats pass of the same command (the roofline kernel's mean must agree with the line).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6c; mkdir -p $O
run_tests() {   # $1 = log name, rest = pytest args; a test failure (rc 1) goes on, anything else stops
  local log=$O/$1.log; shift
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > $log 2>&1
  local rc=$?
  tail -3 $log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
}
run_tests t_range tests/test_x3_range_gpu.py -s
run_tests t_var tests/test_swinir_variants_gpu.py -k "trainer or vs_golden"

timeout -k 10 400 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $O/bench.log 2>&1 || { grep -v "^frame" $O/bench.log | tail -12; exit 1; }
grep -h "^{" $O/bench.log | cut -c1-300
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
find $P -name "*stats*.csv" | head
echo done
