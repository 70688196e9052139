#!/bin/bash
set -o pipefail
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr"
for sc in 0 -2 -4; do
  for pb in 4 32; do
    timeout -k 10 300 $B --per-gpu-batch $pb --side-ctas $sc > gpurun_out/r4s_$pb_$sc.log 2>&1 || exit 1
    echo "B=$pb side_ctas=$sc $(grep -h '^{' gpurun_out/r4s_$pb_$sc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
