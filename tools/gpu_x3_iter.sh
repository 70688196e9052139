# fp32x3 iteration loop on the GPU box: x3 parity tests, the x3 GEMM micro-benchmark, a short bench line and
# the per-call-site kernel times of one B = 32 step.  Stops at the first crash / timeout (a test failure,
# rc 1, still runs the measurements).   usage: bash tools/gpu_x3_iter.sh OUTDIR [pytest -k expr]
set -o pipefail
out=gpurun_out/${1:-x3}
mkdir -p $out
sel=${2:+-k "$2"}
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_tail_gpu.py -v -x $sel --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $out/tests.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u tools/x3_micro.py > $out/micro.log 2>&1 || exit $?
cat $out/micro.log
timeout -k 10 400 python -u bench.py --dtype fp32x3 --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-psnr --no-roles > $out/bench.log 2>&1 || exit $?
grep -h "^{" $out/bench.log | cut -c1-300
timeout -k 10 300 python -u tools/roles.py 32 --dtype fp32x3 > $out/roles32.txt 2>&1 || exit $?
head -30 $out/roles32.txt
exit $rc
