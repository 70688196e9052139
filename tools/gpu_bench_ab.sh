# bench A/B: fused MLP on/off at B=32 and B=4, then a B=4 kernel-trace profile
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > $R/gpurun_out/ab.log
for b in 32 4; do for f in 0 1; do
  echo "B=$b fused_mlp=$f $(KAIR_FUSED_MLP=$f timeout -k 10 300 python bench.py --global-batch $b --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line 2>/dev/null | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["psnr"].get("bf16_delta_db"), d["psnr"].get("uint8_bf16_delta_db"))')" >> $R/gpurun_out/ab.log || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o run -- \
    python3 $R/bench.py --global-batch 4 --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/p4.log 2>&1 || { echo "profile failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof32 -o run -- \
    python3 $R/bench.py --global-batch 32 --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/p32.log 2>&1 || { echo "profile failed"; exit 1; }
echo done
