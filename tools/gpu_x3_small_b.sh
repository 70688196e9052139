# the fp32x3 headline at the per-GPU batches of the 2 / 4 / 8-GPU strong-scaling runs (16 / 8 / 4), 20-step lines
set -o pipefail
out=gpurun_out/${1:-smallb}; mkdir -p $out
for b in 16 8 4; do
  timeout -k 10 300 python -u bench.py --dtype fp32x3 --per-gpu-batch $b --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-psnr --no-roles --no-fp32-line > $out/b$b.log 2>&1 || exit $?
  echo "[B=$b] $(grep -h '^{' $out/b$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
done
