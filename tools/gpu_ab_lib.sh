#!/bin/bash
# A/B of two library builds on the bench (B=32, B=4): $1 = variant .so (swapped in for the second arm)
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
Q="--no-cpu-baseline --no-fp32-line --no-other-configs --no-roles"
for arm in base variant; do
  if [ $arm = variant ]; then cp "$1" kair_amd/lib/libkair_hip.so; fi
  for b in 32 4; do
    timeout -k 10 300 python bench.py --global-batch $b --steps 40 --warmup 10 $Q > gpurun_out/ab_$arm$b.log 2>&1 || { tail -5 gpurun_out/ab_$arm$b.log; exit 1; }
    echo "$arm B=$b $(tail -1 gpurun_out/ab_$arm$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_lib.txt
  done
done
