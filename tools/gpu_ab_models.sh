set -o pipefail
mkdir -p gpurun_out
for v in base KAIR_NT_N32=1 KAIR_NT_N32=2; do
  envs=""; [ "$v" != base ] && envs="$v"
  env $envs timeout -k 10 300 python tools/bench_models.py rrdbnet --steps 20 --warmup 5 > gpurun_out/m_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  env $envs KAIR_NT_N32_TEST=1 timeout -k 10 300 python -m pytest tests/test_convnets_gpu.py -m gpu -x -q > gpurun_out/tc_$v.log 2>&1 || { echo "$v tests failed"; exit 1; }
done
echo done
