set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out; : > $R/gpurun_out/bwd_micro.log
for d in 0 1 2 4; do
  KAIR_RING_DBG=$d timeout -k 10 120 python tools/bwd_micro.py 32 30 2>/dev/null | tail -1 >> $R/gpurun_out/bwd_micro.log || exit 1
done
echo ok
