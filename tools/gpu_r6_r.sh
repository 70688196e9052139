#!/bin/bash
# round 6: channel-chunk-major im2col k order in the generic x3 NT kernel: tests, then the B = 32 step with and
# without it (KAIR_X3_TAPMAJOR=1) under rocprofv3 kernel stats (the 96^2 PixelUnshuffle input gradient)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_tail_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A12 "Error\|assert" $O/t.log | head -50; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  KAIR_X3_TAPMAJOR=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$v -o p -- \
    python3 $R/tools/prof_step.py 32 6 > $O/log$v.txt 2>&1 || { echo "pass $v failed"; tail -3 $O/log$v.txt; exit 1; }
  echo "tapmajor=$v"; grep -h "gemm_nt_x3_kernel" $O/s$v/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
cd $R
timeout -k 10 300 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --no-roles > $O/b.txt 2>&1
echo "b32 $(grep -o '"value": [0-9.]*' $O/b.txt)"
echo done
