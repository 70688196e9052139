#!/bin/bash
# round-4 evidence: rocprofv3 kernel-trace stats of the bench command (its JSON line kept beside) for the
# bf16 headline and the fp32 parity line, and separate FETCH_SIZE / WRITE_SIZE PMC passes over the
# training step alone (B = 32 and B = 4)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/prof4; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o b -- \
  python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $O/bench_line.txt 2> $O/bench_err.txt || { echo "stats pass failed"; tail -5 $O/bench_err.txt; exit 1; }
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats32 -o f -- \
  python3 $R/bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $O/bench_fp32_line.txt 2> $O/bench_fp32_err.txt || { echo "fp32 stats pass failed"; tail -5 $O/bench_fp32_err.txt; exit 1; }
for B in 32 4; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc$B -o f -- \
    python3 $R/tools/prof_step.py $B 4 > $O/logf$B.txt 2>&1 || { echo "fetch pass failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc$B -o w -- \
    python3 $R/tools/prof_step.py $B 4 > $O/logw$B.txt 2>&1 || { echo "write pass failed"; exit 1; }
  cd $R && python3 tools/pmc_traffic.py $O/pmc$B > $O/pmc_traffic_b$B.json; cd /tmp
done
find $O -name "*stats*.csv" | head
echo profile done
