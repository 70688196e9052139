#!/bin/bash
# B=4 A/B of engine switches (bench.py at the per-GPU shape of the N=8 run).
# usage: bash tools/gpu_b4_ab.sh "ENV=1 ENV2=2" "ENV=0" ...   (B via $AB_B, default 4)
set -o pipefail
mkdir -p gpurun_out
B=${AB_B:-4}
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python bench.py --global-batch $B --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-other-configs 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
done
