set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b32.log 2>&1 || { echo "b32 failed"; exit 1; }
KAIR_WGRAD_OVERLAP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b32off.log 2>&1 || { echo "b32off failed"; exit 1; }
timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b4.log 2>&1 || { echo "b4 failed"; exit 1; }
KAIR_WGRAD_OVERLAP=0 timeout -k 10 300 python bench.py --global-batch 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b4off.log 2>&1 || { echo "b4off failed"; exit 1; }
echo done
