# SQ counters of the x3 NT ring on two shapes (tools/x3_micro.py filters), one rocprofv3 --pmc pass per counter
# group (each group within the per-pass hardware limits), summarised by tools/pmc_sq.py.
#   usage: bash tools/gpu_pmc_sq.sh OUTDIR
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${1:-pmc_sq}; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for shape in nt_conv_fwd nt_fc1_fwd; do
  for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/$shape -o p$i -- \
      python3 $R/tools/x3_micro.py $shape --reps 3 > $O/log$i.txt 2>&1 || { echo "pass $i failed"; exit 1; }
  done
done
cd $R && python3 tools/pmc_sq.py $O/nt_conv_fwd $O/nt_fc1_fwd > $O/summary.json && echo pmc done
