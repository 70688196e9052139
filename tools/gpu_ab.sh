# A/B of the x3 GEMM micro-benchmark: the baseline library (tools/build_base.py REV) vs the working tree's
#   usage: bash tools/gpu_ab.sh OUTDIR [filter]
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p $out
for lib in base cur; do
  echo "== $lib"
  if [ $lib = base ]; then export KAIR_LIB=base; else unset KAIR_LIB; fi
  timeout -k 10 180 python -u tools/x3_micro.py ${2:-} > $out/micro_$lib.log 2>&1 || exit $?
  grep -v amdgpu.ids $out/micro_$lib.log
done
