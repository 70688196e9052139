#!/bin/bash
# round 6: chunked pair packing (tests), then bench lines: B = 32 default, B = 4 with x3 weight-gradient row splits of
# at least KAIR_X3_WG_ROWS rows (0 = the 128-row rule)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_x3_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
B="python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles"
timeout -k 10 300 $B > $O/b32.txt 2>&1 || exit 1
echo "B32 $(grep -o '"value": [0-9.]*' $O/b32.txt)"
for r in 0 512 1024 2048; do
  KAIR_X3_WG_ROWS=$r timeout -k 10 300 $B --per-gpu-batch 4 > $O/b4_$r.txt 2>&1 || exit 1
  echo "B4 rows $r $(grep -o '"value": [0-9.]*' $O/b4_$r.txt)"
done
echo done
