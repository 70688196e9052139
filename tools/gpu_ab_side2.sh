#!/bin/bash
# Side-stream scheduling A/B: splits scale (--side-ctas < 0) x stream priorities, B=32 and B=4
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; rm -f gpurun_out/ab2.txt
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" | tee -a gpurun_out/ab2.txt
Q="--no-cpu-baseline --no-fp32-line --no-other-configs --no-roles"
for cfg in "" "--side-ctas -4" "--main-priority -1" "--side-ctas -4 --main-priority -1" "--side-ctas -2 --main-priority -1" "--no-graph --main-priority -1 --side-ctas -4" "--no-graph"; do
  for b in 32 4; do
    timeout -k 10 300 python bench.py --global-batch $b --steps 30 --warmup 8 $Q $cfg > gpurun_out/ab2.log 2>&1 || { tail -5 gpurun_out/ab2.log; exit 1; }
    echo "B=$b [$cfg] $(tail -1 gpurun_out/ab2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab2.txt
  done
done
