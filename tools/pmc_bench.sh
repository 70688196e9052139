#!/bin/bash
# PMC counters (one pass per counter group, MI355X_MICROARCH.md "rocprofv3 PMC slots") over a short
# bench run at B=32; summarise with tools/pmc_summary.py gpurun_out/pmc.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
N=0
run() {
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O -o p$N -- \
    python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/log$N.txt 2>&1 || { echo "pmc pass $N failed"; exit 1; }
  N=$((N+1))
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
run FETCH_SIZE
run WRITE_SIZE
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
echo pmc done
