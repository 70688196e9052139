#!/bin/bash
# round 6, first GPU pass: the range-guard / fp32x3 variant / dist tests, smoke(), and a short headline bench line
# (graph-timed roofline).  A test FAILURE (pytest rc 1) does not stop the script; anything else (fault, abort,
# time limit) does.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6a; mkdir -p $O
run_tests() {   # $1 = log name, rest = pytest args
  local log=$O/$1.log; shift
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > $log 2>&1
  local rc=$?
  tail -3 $log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
}
run_tests t_range tests/test_x3_range_gpu.py -s
run_tests t_x3 tests/test_x3_gpu.py -s -k "classical_full or trajectory or injected"
run_tests t_var tests/test_swinir_variants_gpu.py
run_tests t_dist tests/test_dist_gpu.py -s
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line \
  > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -h "^{" $O/bench.log | cut -c1-400
echo done
