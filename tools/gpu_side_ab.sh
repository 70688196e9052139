#!/bin/bash
# A/B: deferred per-RSTB weight gradients on the side stream vs in place (bench.py --no-side-stream)
set -o pipefail
O=gpurun_out/side_ab; mkdir -p $O
for i in 1 2; do
  for mode in side inline; do
    f=""; [ $mode = inline ] && f="--no-side-stream"
    timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr $f > $O/b32_${mode}_$i.log 2>&1 || exit 1
    grep -h "^{" $O/b32_${mode}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r={k:v for k,v in d.get('kernels_in_step',{}).items()} if isinstance(d.get('kernels_in_step'),dict) else d.get('kernels_in_step'); print('B32 $mode $i', d['value'], d['ms_per_step'])"
  done
done
for mode in side inline; do
  f=""; [ $mode = inline ] && f="--no-side-stream"
  timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --per-gpu-batch 4 $f > $O/b4_${mode}.log 2>&1 || exit 1
  grep -h "^{" $O/b4_${mode}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B4 $mode', d['value'], d['ms_per_step'])"
done
