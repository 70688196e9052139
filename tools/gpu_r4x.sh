#!/bin/bash
# kernel stats of the other configs' training steps (C2 SwinIR-light, C5 RRDBNet)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/prof_oc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-swinir_light rrdbnet}; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o s -- \
    python3 $R/tools/bench_models.py $c --steps 5 --warmup 3 > $O/$c.log 2>&1 || { echo "$c failed"; tail -5 $O/$c.log; exit 1; }
  tail -2 $O/$c.log
done
