#!/bin/bash
# round 6: the whole GPU suite after the launch-macro change (every libkair launch goes through KAIR_LAUNCH), then
# the headline bench line (kernel table from dispatch-packet timestamps) and a rocprofv3 --kernel-trace --stats pass
# of the same command; tools/roofline_check.py compares the two.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6g; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
rc=$?; tail -3 $O/t_all.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
cd $R
python3 tools/roofline_check.py $P/bench_line.txt $P/stats/b_kernel_stats.csv

# A/B: 64-row NT ring tiles at B = 32 (KAIR_X3_BM=64) against the default
timeout -k 10 300 python3 tools/x3_micro.py > $O/micro_default.txt 2>&1 && \
KAIR_X3_BM=64 timeout -k 10 300 python3 tools/x3_micro.py > $O/micro_bm64.txt 2>&1 && \
paste <(cut -c1-30 $O/micro_default.txt) <(cut -c1-30 $O/micro_bm64.txt) | head -30
echo done
