"""HBM traffic per kernel launch from rocprofv3 PMC passes (tools/pmc_bench.sh output).

    python tools/pmc_traffic.py gpurun_out/pmc > profiles/r01_pmc_traffic.json

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads, so it is doubled (MI355X_MICROARCH.md, HBM / rocprofv3 section);
WRITE_SIZE is exact for 16-byte-per-lane streaming stores.  Averages over every dispatch of a kernel.
"""
import collections
import csv
import glob
import json
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                acc[r["Kernel_Name"]][r["Counter_Name"]].append((dur, float(r["Counter_Value"])))
    out = {}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        # the profiled program runs full-batch steps only (tools/prof_step.py): the median over every
        # dispatch of the kernel (robust to a cold first launch), with the dispatch count
        def avg(v):
            xs = sorted(x for _, x in v)
            return xs[len(xs) // 2], len(xs)
        fetch, nf = avg(c["FETCH_SIZE"])
        write, nw = avg(c["WRITE_SIZE"])
        fetch *= 2.0 * 1024
        write *= 1024.0
        out[k[:160]] = {"fetch_bytes_corrected": round(fetch), "write_bytes": round(write),
                        "hbm_bytes_per_launch": round(fetch + write), "dispatches": [nf, nw]}
    json.dump({"source": d, "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes; median over all dispatches of "
               "the kernel (the profiled program runs full-batch training steps only)", "kernels": out},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
