#!/bin/bash
# State check: full -m gpu suite, the default bench line, and the B=4 kernel-trace breakdown.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
[ -n "$SKIPTESTS" ] || { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/st_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/st_tests.log; exit 1; }; }
tail -3 $R/gpurun_out/st_tests.log
SECONDS=0; timeout -k 10 400 python bench.py > $R/gpurun_out/st_bench.log 2>$R/gpurun_out/st_bench.err || { echo "bench failed"; tail -20 $R/gpurun_out/st_bench.err; exit 1; }
tail -1 $R/gpurun_out/st_bench.log
echo "bench wall $SECONDS s"
B=4 bash tools/gpu_prof4.sh && head -40 gpurun_out/tr4_breakdown.txt
