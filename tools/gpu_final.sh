#!/bin/bash
# round-4 closing evidence: the full -m gpu suite, the default bench line (all fields), the B = 4 line,
# per-call-site step breakdowns, then the rocprofv3 stats / PMC passes (tools/gpu_profile_r4.sh)
set -o pipefail
mkdir -p gpurun_out/final4
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/final4/smoke.log 2>&1 || { tail -5 gpurun_out/final4/smoke.log; exit 1; }
tail -1 gpurun_out/final4/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final4/bench_default.log 2>&1 || { tail -5 gpurun_out/final4/bench_default.log; exit 1; }
grep -h "^{" gpurun_out/final4/bench_default.log | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --per-gpu-batch 4 > gpurun_out/final4/bench4.log 2>&1 || exit 1
grep -h "^{" gpurun_out/final4/bench4.log | cut -c1-200
for b in 8 16; do   # the per-GPU shapes of the N = 4 / N = 2 strong-scaling runs
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs --no-fp32-line --no-psnr --per-gpu-batch $b > gpurun_out/final4/bench$b.log 2>&1 || exit 1
  grep -h "^{" gpurun_out/final4/bench$b.log | cut -c1-200
done
timeout -k 10 200 python -u tools/roles.py 32 > gpurun_out/final4/roles32.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/roles.py 4 > gpurun_out/final4/roles4.txt 2>&1 || exit 1
bash tools/gpu_profile_r4.sh
