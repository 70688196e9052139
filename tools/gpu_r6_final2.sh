#!/bin/bash
# round 6 checkpoints after the C2 work: the whole GPU suite, smoke(), the default bench line
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6fin5; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
rc=$?; tail -3 $O/t_all.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -B2 -A15 "Error\|assert" $O/t_all.log | head -60; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python3 bench.py > $O/bench_default.txt 2> $O/bench_default_err.txt || { tail -5 $O/bench_default_err.txt; exit 1; }
echo "default $(grep -o '"value": [0-9.]*' $O/bench_default.txt | head -1)"
echo done
