"""Per-kernel medians of SQ / TCP / TCC counters from rocprofv3 --pmc passes (tools/gpu_pmc_sq.sh).

    python tools/pmc_sq.py DIR [DIR ...]      one JSON object per directory: {kernel: {counter: median}}
"""
import collections
import csv
import glob
import json
import sys


def summarize(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/**/*_counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in acc.items():
        out[k] = {n: sorted(v)[len(v) // 2] for n, v in c.items()}
        out[k]["dispatches"] = max(len(v) for v in c.values())
    return out


if __name__ == "__main__":
    json.dump({d: summarize(d) for d in sys.argv[1:]}, sys.stdout, indent=1)
