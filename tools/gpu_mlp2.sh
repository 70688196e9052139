set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_f.log 2>&1 || { tail -30 $R/gpurun_out/t_f.log; exit 1; }
tail -1 $R/gpurun_out/t_f.log
for d in 0 3 4 7; do
  echo "dbg=$d $(KAIR_FUSED_MLP=1 KAIR_SPLIT=0 KAIR_MLP_DBG=$d timeout -k 10 120 python tools/fused_micro.py 32 30 2>/dev/null | tail -1)"
done
echo "B4 $(KAIR_FUSED_MLP=1 KAIR_SPLIT=0 timeout -k 10 120 python tools/fused_micro.py 4 50 2>/dev/null | tail -1)"
