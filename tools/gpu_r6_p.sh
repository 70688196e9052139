#!/bin/bash
# round 6: the LayerNorm backward fused into the q/k/v / fc1 input-gradient NT ring (kair_gemm_nt_x3_lnbwd): kernel
# and engine parity tests, then bench lines fused vs unfused (KAIR_X3_LNFUSE=0) at B = 32 and B = 4
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -x -v --timeout 120 --timeout-method thread -k "lnbwd" > $O/t_k.log 2>&1
rc=$?; tail -5 $O/t_k.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A12 "Error\|assert" $O/t_k.log | head -60; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_x3_gpu.py tests/test_x3_range_gpu.py tests/test_swinir_variants_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A12 "Error\|assert" $O/t.log | head -60; exit $rc; fi
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
run() {   # label, KAIR_X3_LNFUSE, args
  local l=$1 f=$2; shift 2
  KAIR_X3_LNFUSE=$f timeout -k 10 300 $B "$@" > $O/$l.txt 2>&1 || { echo "$l failed"; tail -3 $O/$l.txt; exit 1; }
  echo "$l $(grep -o '"value": [0-9.]*' $O/$l.txt)"
}
run b32_fused 1
run b32_unfused 0
run b4_fused 1 --per-gpu-batch 4
run b4_unfused 0 --per-gpu-batch 4
echo done
