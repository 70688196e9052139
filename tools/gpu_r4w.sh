#!/bin/bash
# A/B: 2-wave vs 4-wave workgroups of the bf16 attention backward (B = 4, B = 32)
set -o pipefail
timeout -k 10 200 env KAIR_ATTN_BWD_NW=2 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_swinir_gpu.py -k "attention or engine or train" > gpurun_out/r4w_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4w_tests.log; [ $rc -eq 0 ] || exit 1
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for nw in 4 2; do for b in 4 32; do
  KAIR_ATTN_BWD_NW=$nw timeout -k 10 200 $B --global-batch $b > gpurun_out/r4w_b${b}_nw$nw.log 2>&1 || exit 1
  echo "nw $nw B $b: $(grep -h '^{' gpurun_out/r4w_b${b}_nw$nw.log | cut -c80-125)"
done; done
KAIR_ATTN_BWD_NW=2 timeout -k 10 200 python -u tools/roles.py 4 > gpurun_out/r4w_roles4.txt 2>&1; grep -E "attn" gpurun_out/r4w_roles4.txt
