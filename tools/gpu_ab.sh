#!/bin/bash
# A/B on the GPU box: gpu tests, then bench.py at B=32 (and B=4 with AB_B4=1) once per variant.
#   AB_VARIANTS="base KAIR_X=1 KAIR_Y=2" bash tools/gpu_ab.sh    (base = no extra env)
set -o pipefail
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
fi
for v in ${AB_VARIANTS:-base}; do
  envs=""; [ "$v" != base ] && envs="$v"
  if [ -z "$AB_ONLY_B4" ]; then
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b32_$v.log 2>&1 || { echo "b32 $v failed"; exit 1; }
  fi
  if [ -n "$AB_B4$AB_ONLY_B4" ]; then
    env $envs timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b4_$v.log 2>&1 || { echo "b4 $v failed"; exit 1; }
  fi
done
echo done
