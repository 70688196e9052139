set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C=proj_fwd
for S in 0 1; do
  KAIR_GEMM_STREAM=$S timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc$S -o a -- python3 $R/tools/gemm_micro.py $C --no-torch --reps 5 > $R/gpurun_out/pmc${S}a.log 2>&1
  KAIR_GEMM_STREAM=$S timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc$S -o b -- python3 $R/tools/gemm_micro.py $C --no-torch --reps 5 > $R/gpurun_out/pmc${S}b.log 2>&1
  KAIR_GEMM_STREAM=$S timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc$S -o c -- python3 $R/tools/gemm_micro.py $C --no-torch --reps 5 > $R/gpurun_out/pmc${S}c.log 2>&1
  KAIR_GEMM_STREAM=$S timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc$S -o d -- python3 $R/tools/gemm_micro.py $C --no-torch --reps 5 > $R/gpurun_out/pmc${S}d.log 2>&1
done
