#!/bin/bash
# HBM traffic per kernel launch: separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE over a
# short bench run (MI355X_MICROARCH.md: FETCH_SIZE x2 on gfx950), summarised by tools/pmc_traffic.py
set -o pipefail
R=$(pwd); O=$R/gpurun_out/pmc2; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O -o f -- \
  python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-fp32-line --no-other-configs --no-roles > $O/logf.txt 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O -o w -- \
  python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-fp32-line --no-other-configs --no-roles > $O/logw.txt 2>&1 || { echo "write pass failed"; exit 1; }
cd $R && python3 tools/pmc_traffic.py $O > $R/gpurun_out/pmc_traffic.json && echo pmc done
