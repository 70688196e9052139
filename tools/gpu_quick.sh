#!/bin/bash
# Quick iteration: selected -m gpu tests ($1: pytest -k expression, "" = test files in $2), bench lines
# at B=32 / B=4 (roles table), and a B=32 rocprofv3 step breakdown.
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
K="$1"; FILES="${2:-tests}"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; echo "tests failed"; exit 1; }
  tail -1 gpurun_out/t.log
fi
Q="--no-cpu-baseline --no-fp32-line --no-other-configs"
timeout -k 10 300 python bench.py --steps 30 --warmup 10 $Q > gpurun_out/b32.log 2>&1 || { tail -20 gpurun_out/b32.log; echo "bench failed"; exit 1; }
tail -1 gpurun_out/b32.log > gpurun_out/b32.json; cut -c1-300 gpurun_out/b32.json
timeout -k 10 300 python bench.py --global-batch 4 --steps 50 --warmup 10 $Q > gpurun_out/b4.log 2>&1 || { tail -20 gpurun_out/b4.log; echo "bench4 failed"; exit 1; }
tail -1 gpurun_out/b4.log > gpurun_out/b4.json; cut -c1-300 gpurun_out/b4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr32 -o run -- \
  python3 $R/bench.py --steps 8 --warmup 3 $Q --no-roles > $R/gpurun_out/tr32.log 2>&1 || { echo "profile failed"; exit 1; }
cd $R
python3 tools/step_breakdown.py gpurun_out/tr32/run_kernel_trace.csv 6 > gpurun_out/b32_breakdown.txt
for k in "rowgemm_kernel<12, 2, 4, 1" "attn_bwd_bf16"; do
  python3 tools/overlap.py gpurun_out/tr32/run_kernel_trace.csv "$k" 6 > gpurun_out/ovl_$(echo $k | cut -c1-8).txt
done
rm -f gpurun_out/tr32/run_kernel_trace.csv
head -24 gpurun_out/b32_breakdown.txt
echo done
