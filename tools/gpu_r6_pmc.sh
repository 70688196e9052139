#!/bin/bash
# round 6: HBM traffic per kernel launch over the fp32x3 B = 32 training step alone (tools/prof_step.py): one
# rocprofv3 pass for FETCH_SIZE, one for WRITE_SIZE (MI355X_MICROARCH.md rocprofv3 PMC slots), summarised by
# tools/pmc_traffic.py (FETCH_SIZE x 2 on gfx950)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O -o f -- \
  python3 $R/tools/prof_step.py 32 4 > $O/log_f.txt 2>&1 || { echo "fetch pass failed"; tail -3 $O/log_f.txt; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O -o w -- \
  python3 $R/tools/prof_step.py 32 4 > $O/log_w.txt 2>&1 || { echo "write pass failed"; tail -3 $O/log_w.txt; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O > $O/r06_pmc_traffic.json && echo "pmc ok"
rm -f $O/*_counter_collection.csv.gz
echo done
