#!/bin/bash
# One perf iteration on the GPU box: selected GPU tests ($TESTS, default: all -m gpu), then bench A/B
# configs at B=4 and B=32 given as arguments (each an env assignment list, e.g. "KAIR_X=1").
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-tests}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { tail -30 gpurun_out/it_tests.log; echo "TESTS FAILED"; exit 1; }
tail -2 gpurun_out/it_tests.log
for B in ${AB_BATCHES:-4 32}; do
  for cfg in "$@"; do
    echo "== B=$B $cfg"
    env $cfg timeout -k 10 200 python bench.py --global-batch $B --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --no-fp32-line 2>gpurun_out/it_err.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['psnr']['bf16_delta_db'])" || { tail -20 gpurun_out/it_err.log; exit 1; }
  done
done
