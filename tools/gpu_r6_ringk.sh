#!/bin/bash
# round 6: ring GEMM partial-K chunks (K % 64 != 0: C2's K = 96 / 288) + 128-wide N tile, narrow linears in the
# grouped TN-ring weight gradient -- parity, C2 A/Bs, the other configs, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ringk; mkdir -p $O; cd $R
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -1 $O/kern.txt
timeout -k 10 500 $T tests/test_full_configs_gpu.py tests/test_fused_gpu.py -s > $O/full.txt 2>&1 || { tail -30 $O/full.txt; exit 1; }
grep "C2 bf16" $O/full.txt; tail -1 $O/full.txt
for t in 1 0 1 0; do
  export KAIR_RING_BN128=$t
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 > $O/b_$t.txt 2>&1 || { tail -5 $O/b_$t.txt; exit 1; }
  echo "bn128 $t $(grep -o '"patches_per_s": [0-9.]*' $O/b_$t.txt)"
done
unset KAIR_RING_BN128
for t in 1 0 1 0; do
  a=""; [ $t = 0 ] && a="--no-grouped-wgrad"
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 $a > $O/g_$t.txt 2>&1 || { tail -5 $O/g_$t.txt; exit 1; }
  echo "grouped $t $(grep -o '"patches_per_s": [0-9.]*' $O/g_$t.txt)"
done
timeout -k 10 600 python3 tools/bench_models.py dncnn rrdbnet usrnet --steps 20 --warmup 5 > $O/models.txt 2>&1 || { tail -5 $O/models.txt; exit 1; }
cut -c1-110 $O/models.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c2 -- python3 tools/bench_models.py swinir_light --steps 10 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" -print -quit)
python3 tools/step_breakdown.py $f 22 > $O/breakdown.txt && cut -c1-160 $O/breakdown.txt
