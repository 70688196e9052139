#!/bin/bash
# bench.py at B=32 and B=4 (30 timed steps): throughput + the fused kernels' HIP-event times
set -o pipefail
mkdir -p gpurun_out
for B in ${KMS_BATCHES:-32 4}; do
  timeout -k 10 300 python bench.py --global-batch $B --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-other-configs \
    > gpurun_out/kms_$B.log 2>&1 || { tail -20 gpurun_out/kms_$B.log; exit 1; }
  tail -1 gpurun_out/kms_$B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['ms_per_step'], 'mlp', d['roofline']['kernel_ms'], 'attn', d['roofline_attention']['kernel_ms'], 'psnr', d['psnr']['bf16_delta_db'], d['psnr']['uint8_bf16_delta_db'])"
done
