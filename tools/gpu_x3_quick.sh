# split-fp16 (fp32x3) engine: kernel + network parity tests, the gradient-error diagnostic, a short bench
# line and the per-call-site kernel times of one step
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u tools/x3_grad_diag.py > gpurun_out/r5a/diag.log 2>&1; echo "diag rc $?"
head -12 gpurun_out/r5a/diag.log
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r5a/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r5a/tests.log | tail -30
timeout -k 10 400 python -u bench.py --dtype fp32x3 --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-psnr --no-roles > gpurun_out/r5a/bench.log 2>&1; rc2=$?
grep -h "^{" gpurun_out/r5a/bench.log | cut -c1-300
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 300 python -u tools/roles.py 32 --dtype fp32x3 > gpurun_out/r5a/roles32.txt 2>&1; rc3=$?
head -40 gpurun_out/r5a/roles32.txt
exit $rc3
