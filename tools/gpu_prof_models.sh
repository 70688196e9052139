#!/bin/bash
# rocprofv3 kernel stats of the other BASELINE configs (tools/bench_models.py), one run per config
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in ${@:-swinir_light rrdbnet usrnet}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pm_$m -o run -- \
    python3 $R/tools/bench_models.py $m --steps 5 --warmup 2 > $R/gpurun_out/pm_$m.log 2>&1 || { echo "profile $m failed"; exit 1; }
  rm -f $R/gpurun_out/pm_$m/run_kernel_trace.csv
  echo "== $m: $(tail -1 $R/gpurun_out/pm_$m.log | cut -c1-160)"
  python3 - "$R/gpurun_out/pm_$m/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("  %5.1f%%  %6d x %8.1f us  %s" % (100 * float(r["TotalDurationNs"]) / tot, int(r["Calls"]), float(r["AverageNs"]) / 1e3, r["Name"][:90]))
PY
done
