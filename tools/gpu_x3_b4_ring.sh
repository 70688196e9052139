# fp32x3 at B = 4 per GPU (the 8-GPU strong-scaling shape): ring kernels on / off (KAIR_X3_RING=0), 20-step lines
set -o pipefail
out=gpurun_out/${1:-b4ring}; mkdir -p $out
for r in 1 0 1 0; do
  KAIR_X3_RING=$r timeout -k 10 300 python -u bench.py --dtype fp32x3 --per-gpu-batch 4 --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-psnr --no-roles --no-fp32-line > $out/b.log 2>&1 || exit $?
  echo "[ring=$r] $(grep -h '^{' $out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python -u tools/roles.py 4 --dtype fp32x3 > $out/roles4.txt 2>&1 || exit $?
head -30 $out/roles4.txt
