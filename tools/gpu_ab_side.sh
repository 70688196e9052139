#!/bin/bash
# A/B: side-stream workgroup budget at B=32 and B=4
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > gpurun_out/ab.log
Q="--no-cpu-baseline --no-fp32-line --no-other-configs --no-roles"
for b in 32 4; do for c in 0 48 96 144 0 48 96 144; do
  st=$([ $b = 4 ] && echo 60 || echo 30)
  v=$(timeout -k 10 300 python bench.py --global-batch $b --steps $st --warmup 10 $Q --side-ctas $c 2>/dev/null | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') || exit 1
  echo "B=$b side_ctas=$c $v" | tee -a gpurun_out/ab.log
done; done
