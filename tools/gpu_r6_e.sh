#!/bin/bash
# round 6: x3 GEMM micro-benchmarks at B = 32 / 4 (pair vs fp32 operands, 64-row ring tiles at B = 4), the debug-
# ablation breakdown of the NT ring (KAIR_RING_DBG: 1 no epilogue, 2 no MFMA, 64 no fragment loads, 128 no stores),
# and a B = 4 bench line.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r6e}; mkdir -p $O
X3_MICRO_B=32 timeout -k 10 200 python -u tools/x3_micro.py --reps 20 > $O/micro_b32.log 2>&1 || { tail -5 $O/micro_b32.log; exit 1; }
grep -v amdgpu.ids $O/micro_b32.log
X3_MICRO_B=4 timeout -k 10 200 python -u tools/x3_micro.py --reps 50 > $O/micro_b4.log 2>&1 || { tail -5 $O/micro_b4.log; exit 1; }
grep -v amdgpu.ids $O/micro_b4.log
DBGS="0 1 2 64 128" bash tools/gpu_abl.sh ${TAG:-r6e}/abl nt_ || exit 1
timeout -k 10 300 python -u bench.py --global-batch 4 --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs \
  --no-fp32-line --no-psnr > $O/bench_b4.log 2>&1 || { grep -v "^frame" $O/bench_b4.log | tail -12; exit 1; }
grep -h "^{" $O/bench_b4.log | cut -c1-200
echo done
