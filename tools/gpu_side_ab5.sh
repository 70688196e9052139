# side-stream knobs A/B on the fp32x3 headline (10-step lines, same box)
set -o pipefail
out=gpurun_out/${1:-side5}; mkdir -p $out
for v in "" "--side-ctas 128" "--side-ctas -2" "--side-priority -1" "--main-priority -1" ""; do
  timeout -k 10 300 python -u bench.py --dtype fp32x3 --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-psnr --no-roles --no-fp32-line $v > $out/b.log 2>&1 || exit $?
  echo "[$v] $(grep -h '^{' $out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
done
