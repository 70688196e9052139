#!/bin/bash
# round 6: NT ring last-round split (128-row tiles, then 64-row tiles from m_base): tests, then bench lines
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x3_gpu.py tests/test_swinir_variants_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B5 "Error\|assert" $O/t.log | head -40; exit $rc; fi
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
run() {   # label, args
  local l=$1; shift
  timeout -k 10 300 $B "$@" > $O/$l.txt 2>&1 || { echo "$l failed"; tail -3 $O/$l.txt; exit 1; }
  echo "$l $(grep -o '"value": [0-9.]*' $O/$l.txt)"
}
run b32
run b16 --per-gpu-batch 16
run b8 --per-gpu-batch 8
run b4 --per-gpu-batch 4
echo done
