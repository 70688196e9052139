#!/bin/bash
# round 6 checkpoint: the whole -m gpu suite (one process), smoke(), the default bench line, and rocprofv3
# --kernel-trace --stats of the headline bench command (the roofline kernel's mean must agree with the line).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r6full}; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench_default.log 2>&1 || { grep -v "^frame" $O/bench_default.log | tail -12; exit 1; }
grep -h "^{" $O/bench_default.log | cut -c1-300
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
find $P -name "*stats*.csv" | head -3
echo done
