#!/bin/bash
# round 6: x3 GEMM micro-benchmarks at B = 32 / 4 (pair vs fp32 operands, 64-row ring tiles at B = 4), the debug-
# ablation breakdown of the NT ring (KAIR_RING_DBG: 1 no epilogue, 2 no MFMA, 64 no fragment loads, 128 no stores),
# and a B = 4 bench line.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${TAG:-r6e}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_full_configs_gpu.py -k c5 \
  tests/test_dist_gpu.py > $O/t_c5.log 2>&1; rc=$?; tail -4 $O/t_c5.log; grep -h "rrdbnet-c5 params" $O/t_c5.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
X3_MICRO_B=32 timeout -k 10 200 python -u tools/x3_micro.py --reps 20 > $O/micro_b32.log 2>&1 || { tail -5 $O/micro_b32.log; exit 1; }
grep -v amdgpu.ids $O/micro_b32.log
X3_MICRO_B=4 timeout -k 10 200 python -u tools/x3_micro.py --reps 50 > $O/micro_b4.log 2>&1 || { tail -5 $O/micro_b4.log; exit 1; }
grep -v amdgpu.ids $O/micro_b4.log
DBGS="0 1 2 64 128" bash tools/gpu_abl.sh ${TAG:-r6e}/abl nt_ || exit 1
timeout -k 10 300 python -u bench.py --global-batch 4 --steps 40 --warmup 10 --no-cpu-baseline --no-other-configs \
  --no-fp32-line --no-psnr > $O/bench_b4.log 2>&1 || { grep -v "^frame" $O/bench_b4.log | tail -12; exit 1; }
grep -h "^{" $O/bench_b4.log | cut -c1-200
echo done
for sc in 0 128 192; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr \
    --no-roles --side-ctas $sc > $O/bench_sc$sc.log 2>&1 || { grep -v "^frame" $O/bench_sc$sc.log | tail -12; exit 1; }
  echo "side-ctas $sc: $(grep -h '^{' $O/bench_sc$sc.log | cut -c1-120)"
done
timeout -k 10 400 python -u tools/bench_models.py rrdbnet usrnet dncnn --dtype fp32 --steps 10 --warmup 3 > $O/models_fp32.log 2>&1 \
  || { tail -5 $O/models_fp32.log; exit 1; }
grep "^{" $O/models_fp32.log
timeout -k 10 300 python -u tools/bench_models.py rrdbnet --dtype fp32x3 --steps 10 --warmup 3 > $O/models_x3.log 2>&1 \
  || { tail -5 $O/models_x3.log; exit 1; }
grep "^{" $O/models_x3.log
echo done2
