#!/bin/bash
# A/B over library variants x bench flags, B=32 and B=4, two rounds (ABAB order):
#   tools/gpu_ab_multi.sh "lib1.so lib2.so ..." "flags1|flags2|..."   (lib "base" = libkair_hip.so as built)
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; OUT=gpurun_out/ab_multi.txt; rm -f $OUT
cp kair_amd/lib/libkair_hip.so /tmp/kair_base.so
Q="--no-cpu-baseline --no-fp32-line --no-other-configs --no-roles"
IFS='|' read -ra FL <<< "${2:-}"; [ ${#FL[@]} -eq 0 ] && FL=("")
for rep in 1 2; do
  for lib in $1; do
    if [ "$lib" = base ]; then cp /tmp/kair_base.so kair_amd/lib/libkair_hip.so; else cp "kair_amd/lib/$lib" kair_amd/lib/libkair_hip.so; fi
    for f in "${FL[@]}"; do
      for b in 32 4; do
        timeout -k 10 300 python bench.py --global-batch $b --steps 30 --warmup 10 $Q $f > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; cp /tmp/kair_base.so kair_amd/lib/libkair_hip.so; exit 1; }
        echo "$lib [$f] B=$b $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT
      done
    done
  done
done
cp /tmp/kair_base.so kair_amd/lib/libkair_hip.so
