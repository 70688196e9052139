# one GPU call: x3 parity tests, the NT-ring store ablation (debug build: bits 0 / 128 / 1), the bench line and
# the per-role times.   usage: bash tools/gpu_r5_combo.sh OUTDIR
set -o pipefail
out=gpurun_out/${1:-combo}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_tail_gpu.py -v -x --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAIL" $out/tests.log | tail -5
[ $rc -le 1 ] || exit $rc
for d in 0 128 1; do
  KAIR_LIB=debug KAIR_RING_DBG=$d timeout -k 10 120 python -u tools/x3_micro.py nt_ --reps 10 > $out/abl_$d.log 2>&1 || exit $?
done
timeout -k 10 240 python -u tools/x3_micro.py > $out/micro.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --dtype fp32x3 --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-psnr --no-roles > $out/bench.log 2>&1 || exit $?
grep -h "^{" $out/bench.log | cut -c1-300
timeout -k 10 300 python -u tools/roles.py 32 --dtype fp32x3 > $out/roles32.txt 2>&1 || exit $?
exit $rc
