# A/B of the fp32x3 bench line and the NT micro-benchmark: the baseline library (tools/build_base.py REV) vs the
# working tree's, alternating twice on one box.   usage: bash tools/gpu_ab_bench.sh OUTDIR
set -o pipefail
out=gpurun_out/${1:-abb}; mkdir -p $out
for lib in base cur base cur; do
  if [ $lib = base ]; then export KAIR_LIB=base; else unset KAIR_LIB; fi
  timeout -k 10 300 python -u bench.py --dtype fp32x3 --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-psnr --no-roles --no-fp32-line > $out/b_$lib.log 2>&1 || exit $?
  echo "[$lib] $(grep -h '^{' $out/b_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
done
for lib in base cur; do
  if [ $lib = base ]; then export KAIR_LIB=base; else unset KAIR_LIB; fi
  timeout -k 10 180 python -u tools/x3_micro.py nt_ > $out/micro_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -v amdgpu.ids $out/micro_$lib.log
done
