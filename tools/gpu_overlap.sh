#!/bin/bash
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
Q="--no-cpu-baseline --no-fp32-line --no-other-configs --no-roles"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr32 -o run -- \
  python3 $R/bench.py --steps 8 --warmup 3 $Q > $R/gpurun_out/tr32.log 2>&1 || { echo "profile failed"; exit 1; }
cd $R
for k in "rowgemm_kernel<12, 4, 4, 1>" "rowgemm_kernel<36" "rowgemm_kernel<24" "swin_mlp_fwd" "attn_bwd_bf16"; do
  python3 tools/overlap.py gpurun_out/tr32/run_kernel_trace.csv "$k" 6
done
python3 tools/step_breakdown.py gpurun_out/tr32/run_kernel_trace.csv 6 | head -20
rm -f gpurun_out/tr32/run_kernel_trace.csv
