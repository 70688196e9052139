#!/bin/bash
# round 6: C2's side-stream workgroup cap (grouped narrow weight gradients beside the next RSTB's chain)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/c2side; mkdir -p $O
for c in 0 96 128 192 0 96 128 192; do
  timeout -k 10 300 python3 tools/bench_models.py swinir_light --steps 20 --warmup 5 --side-ctas $c > $O/b_$c.txt 2>&1 || { tail -5 $O/b_$c.txt; exit 1; }
  echo "side-ctas $c $(grep -o '"patches_per_s": [0-9.]*' $O/b_$c.txt)"
done
echo done
