set -o pipefail
for d in 0 1 2 3 4 7; do
  KAIR_MLPB_DBG=$d timeout -k 10 120 python tools/mlpbwd_micro.py 32 30 2>/dev/null | tail -1 || exit 1
done
