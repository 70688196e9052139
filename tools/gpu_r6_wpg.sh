#!/bin/bash
# round 6: attention-backward windows per group from the groups per head that fit one round (C2) -- parity, C2, trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wpg; mkdir -p $O; cd $R
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py tests/test_x3_gpu.py -k "attention or attn" > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -1 $O/kern.txt
timeout -k 10 400 $T tests/test_full_configs_gpu.py -k c2 -s > $O/c2.txt 2>&1 || { tail -30 $O/c2.txt; exit 1; }
grep "C2 bf16" $O/c2.txt; tail -1 $O/c2.txt
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 > $O/b_$i.txt 2>&1 || { tail -5 $O/b_$i.txt; exit 1; }
  echo "c2 $(grep -o '"patches_per_s": [0-9.]*' $O/b_$i.txt)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c2 -- python3 tools/bench_models.py swinir_light --steps 10 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" -print -quit)
python3 tools/step_breakdown.py $f 16 > $O/breakdown.txt && cut -c1-160 $O/breakdown.txt
