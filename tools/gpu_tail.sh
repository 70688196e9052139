set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/t_full.log 2>&1 || { tail -30 $R/gpurun_out/t_full.log; exit 1; }
tail -1 $R/gpurun_out/t_full.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/q32.log 2>&1 || { echo "b32 failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/qprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qprof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line > $R/gpurun_out/qp.log 2>&1 || { echo "profile failed"; exit 1; }
echo done
