"""Print value / ms_per_step of every gpurun_out/b*_*.log written by tools/gpu_ab.sh."""
import glob
import json

for f in sorted(glob.glob("gpurun_out/b*_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f"{f:45s} {d['value']:9.2f} patches/s {d['ms_per_step']:8.3f} ms/step")
    except Exception as e:  # noqa: BLE001
        print(f, "no result", e)
