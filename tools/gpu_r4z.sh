#!/bin/bash
# same-box A/B: KAIR_LIB=base (HEAD library) vs the working tree's, B = 32 / B = 4 and C5 RRDBNet
set -o pipefail
B="python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
for rep in 1 2; do for lib in base new; do for b in 32 4; do
  KAIR_LIB=$lib timeout -k 10 200 $B --global-batch $b > gpurun_out/r4z_${lib}_b$b.log 2>&1 || exit 1
  echo "$lib B $b: $(grep -h '^{' gpurun_out/r4z_${lib}_b$b.log | cut -c80-115)"
done; done; done
for lib in base new; do
  KAIR_LIB=$lib timeout -k 10 200 python -u tools/bench_models.py rrdbnet --steps 8 --warmup 3 > gpurun_out/r4z_${lib}_c5.log 2>&1 || exit 1
  echo "$lib C5: $(grep -h '^{' gpurun_out/r4z_${lib}_c5.log | cut -c1-90)"
done
