set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > $R/gpurun_out/attn_ab.log
for d in 0 1 2 3; do
  echo "dbg=$d $(KAIR_SPLIT=0 KAIR_ATTN_DBG=$d timeout -k 10 120 python tools/fused_micro.py 32 30 2>/dev/null | tail -1)" >> $R/gpurun_out/attn_ab.log || exit 1
done
echo ok
