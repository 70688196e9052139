# NT ring chunk timelines (debug-ablation build) for the main block shapes
#   usage: bash tools/gpu_stamps.sh OUTDIR
set -o pipefail
out=gpurun_out/${1:-stamps}
mkdir -p $out
for c in nt_qkv_fwd nt_proj_fwd nt_fc1_dgrad nt_conv_fwd; do
  KAIR_LIB=debug KAIR_RING_DBG=8 timeout -k 10 120 python -u tools/x3_stamps.py $c >> $out/stamps.log 2>&1 || exit $?
done
grep -v amdgpu.ids $out/stamps.log
