set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_data_gpu.py -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_data.log 2>&1 || { tail -30 $R/gpurun_out/t_data.log; exit 1; }
tail -1 $R/gpurun_out/t_data.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/q32.log 2>&1 || { echo "b32 failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$R/gpurun_out/q32.log').read().strip().split(chr(10))[-1]); print(d['value'], d['ms_per_step'])"
