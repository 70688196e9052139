# Ablations of the x3 ring GEMMs (debug-ablation build, KAIR_RING_DBG bits: 1 no epilogue, 2 no MFMA, 4 no DMA,
# 16 no B (weight) DMA, 32 no A DMA, 64 no fragment loads, 128 no epilogue stores)
#   usage: bash tools/gpu_abl.sh OUTDIR [filter]
set -o pipefail
out=gpurun_out/${1:-abl}
mkdir -p $out
for d in ${DBGS:-0 1 2 4 3 6}; do
  echo "== dbg $d"
  KAIR_LIB=debug KAIR_RING_DBG=$d timeout -k 10 120 python -u tools/x3_micro.py ${2:-} --reps 10 > $out/abl_$d.log 2>&1 || exit $?
  grep -v amdgpu.ids $out/abl_$d.log
done
