set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > $R/gpurun_out/tn_ab.log
for d in 1 2 4; do
  KAIR_TN_SPLIT_DIV=$d timeout -k 10 120 python tools/bwd_micro.py 32 30 2>/dev/null | tail -1 >> $R/gpurun_out/tn_ab.log || exit 1
done
for d in 1 2; do
  echo "bench div=$d $(KAIR_TN_SPLIT_DIV=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line 2>/dev/null | tail -1 | cut -c1-120)" >> $R/gpurun_out/tn_ab.log || exit 1
done
echo ok
