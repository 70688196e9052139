#!/bin/bash
# round 6: narrow-N GEMMs on the ring in one N tile (C2's Cp = 64 / Hdp = 128 projections) -- parity, then the
# other configs' throughput (regression check: C1 / C3 / C5 also run bf16 row GEMMs)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/ring64; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -2 $O/kern.txt
timeout -k 10 500 $T tests/test_full_configs_gpu.py -s > $O/full.txt 2>&1 || { tail -30 $O/full.txt; exit 1; }
grep "C2 bf16" $O/full.txt; tail -2 $O/full.txt
timeout -k 10 600 python3 tools/bench_models.py --steps 20 --warmup 5 > $O/models.txt 2>&1 || { tail -5 $O/models.txt; exit 1; }
cut -c1-150 $O/models.txt
echo done
