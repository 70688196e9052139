# MLP fused kernel ablations (KAIR_MLP_DBG bits) at B=32, split and plain weights
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > $R/gpurun_out/mlp_ab.log
for sp in 0 1; do for d in 0 1 2 3 4 7; do
  echo "split=$sp dbg=$d $(KAIR_SPLIT=$sp KAIR_MLP_DBG=$d timeout -k 10 120 python tools/fused_micro.py 32 30 2>/dev/null | tail -1)" >> $R/gpurun_out/mlp_ab.log || exit 1
done; done
echo ok
