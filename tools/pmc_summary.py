"""Average rocprofv3 --pmc counter values per kernel over the dispatches in *_counter_collection.csv.

    python tools/pmc_summary.py <dir> [kernel-substring]
"""
import collections
import csv
import glob
import sys


def main(d, sub=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if sub and sub not in k:
                continue
            vals[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
