set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_rowgemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rg_test.log 2>&1
rc=$?
tail -5 gpurun_out/rg_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/rowgemm_bench.py > gpurun_out/rg_bench.log 2>&1
rc=$?
cat gpurun_out/rg_bench.log
exit $rc
