#!/bin/bash
# Short bench lines (B=32, B=4) with the in-step per-role kernel table
set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out
Q="--no-cpu-baseline --no-fp32-line --no-other-configs"
timeout -k 10 300 python bench.py --steps 30 --warmup 10 $Q > gpurun_out/b32.log 2>&1 || { tail -20 gpurun_out/b32.log; echo "bench failed"; exit 1; }
tail -1 gpurun_out/b32.log > gpurun_out/b32.json
timeout -k 10 300 python bench.py --global-batch 4 --steps 50 --warmup 10 $Q > gpurun_out/b4.log 2>&1 || { tail -20 gpurun_out/b4.log; echo "bench4 failed"; exit 1; }
tail -1 gpurun_out/b4.log > gpurun_out/b4.json
python3 - <<'PY'
import json
for f in ("gpurun_out/b32.json", "gpurun_out/b4.json"):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], "roof:", {k: d["roofline"].get(k) for k in ("kernel", "role", "kernel_ms", "frac")})
    for k in d.get("kernels_in_step", []):
        print("   %-40s %-48s %4d x %8.4f ms  frac %s" % (k["kernel"][:40], k["role"][:48], k["launches_per_step"], k["kernel_ms"], k.get("frac")))
    print("   attn mfma", d.get("attention_gemm_mfma"))
PY
