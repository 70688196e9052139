#!/bin/bash
# round 6: the 128-pixel halo tile (C2's W = 64 RSTB convs) -- parity, C2 + C1/C3/C5 throughput, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/halo128; mkdir -p $O; cd $R
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -1 $O/kern.txt
timeout -k 10 500 $T tests/test_full_configs_gpu.py tests/test_swinir_variants_gpu.py -s > $O/full.txt 2>&1 || { tail -30 $O/full.txt; exit 1; }
grep "C2 bf16" $O/full.txt; tail -1 $O/full.txt
timeout -k 10 600 python3 tools/bench_models.py --steps 20 --warmup 5 > $O/models.txt 2>&1 || { tail -5 $O/models.txt; exit 1; }
cut -c1-110 $O/models.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c2 -- python3 tools/bench_models.py swinir_light --steps 10 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" -print -quit)
python3 tools/step_breakdown.py $f 16 > $O/breakdown.txt && cut -c1-160 $O/breakdown.txt
