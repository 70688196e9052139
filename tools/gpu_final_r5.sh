#!/bin/bash
# round-5 closing evidence, part 2 (part 1: tools/gpu_tests.sh + smoke): the default bench line (all fields), the
# per-call-site step breakdown, rocprofv3 kernel-trace stats of the headline bench command, and separate
# FETCH_SIZE / WRITE_SIZE PMC passes over the fp32x3 training step alone (summarised by tools/pmc_traffic.py)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/final5; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep -h "^{" $O/bench_default.log | cut -c1-300
timeout -k 10 200 python -u tools/roles.py 32 --dtype fp32x3 > $O/roles32.txt 2>&1 || exit 1
P=$O/prof; rm -rf $P; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $P/pmc32 -o f -- \
  python3 $R/tools/prof_step.py 32 4 fp32x3 > $P/logf.txt 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $P/pmc32 -o w -- \
  python3 $R/tools/prof_step.py 32 4 fp32x3 > $P/logw.txt 2>&1 || { echo "write pass failed"; exit 1; }
cd $R && python3 tools/pmc_traffic.py $P/pmc32 > $P/pmc_traffic_b32.json
find $P -name "*stats*.csv" | head
echo profile done
