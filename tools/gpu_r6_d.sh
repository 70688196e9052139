#!/bin/bash
# round 6: fp16-pair block operands (LN / row-copy / attention / fc1 / fc2-dgrad producers, TN-ring pair reads):
# the x3 kernel + network tests, the range / variant / world-2 x3 tests, then a short bench line.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r6d}; mkdir -p $O
run_tests() {   # $1 = log name, rest = pytest args; a test failure (rc 1) goes on, anything else stops
  local log=$O/$1.log; shift
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > $log 2>&1
  local rc=$?
  tail -3 $log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
}
run_tests t_x3 tests/test_x3_gpu.py -s
run_tests t_range tests/test_x3_range_gpu.py
run_tests t_var tests/test_swinir_variants_gpu.py -k "fp32x3"
run_tests t_dist tests/test_dist_gpu.py -s -k "fp32x3"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $O/bench.log 2>&1 || { grep -v "^frame" $O/bench.log | tail -12; exit 1; }
grep -h "^{" $O/bench.log | cut -c1-200
echo done
