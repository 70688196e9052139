#!/bin/bash
# round 6: in-kernel trace timing of the bench roofline vs rocprofv3 of the same command; x3 tests after the kernel
# signature change; per-GPU batch 16 / 8 / 4 lines (the 2 / 4 / 8-GPU strong-scaling shapes)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r6f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_x3_gpu.py tests/test_x3_range_gpu.py \
  > $O/t_x3.log 2>&1; rc=$?; tail -2 $O/t_x3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
P=$O/prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/stats -o b -- \
  python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
  > $P/bench_line.txt 2> $P/bench_err.txt || { echo "stats pass failed"; tail -5 $P/bench_err.txt; exit 1; }
cd $R
python3 - <<'PY'
import csv, json, glob
line = json.loads([l for l in open("gpurun_out/r6f/prof/bench_line.txt") if l.startswith("{")][0])
r = line["roofline"]
print("bench roofline:", r["kernel"], r["kernel_ms"], r.get("frac"), r.get("timed_by"), "value", line["value"])
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r6f/prof/stats/*kernel_stats.csv")[0])))
for x in rows[:5]:
    print("rocprof:", x["Calls"], round(float(x["AverageNs"]) / 1e3, 2), x["Percentage"], x["Name"][:90])
PY
for b in 16 8 4; do
  timeout -k 10 300 python -u bench.py --global-batch $b --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs \
    --no-fp32-line --no-psnr > $O/bench_b$b.log 2>&1 || { grep -v "^frame" $O/bench_b$b.log | tail -12; exit 1; }
  echo "B=$b: $(grep -h '^{' $O/bench_b$b.log | cut -c1-110)"
done
echo done
