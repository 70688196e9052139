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
        # the bench's full-batch launches only: the same kernel also runs at the PSNR evaluation's
        # smaller batch (same persistent grid size), so keep dispatches at >= half the longest duration
        def avg(v):
            top = max(t for t, _ in v)
            sel = [x for t, x in v if t >= 0.5 * top]
            return sum(sel) / len(sel), len(sel)
        fetch, nf = avg(c["FETCH_SIZE"])
        write, nw = avg(c["WRITE_SIZE"])
        fetch *= 2.0 * 1024
        write *= 1024.0
        out[k[:160]] = {"fetch_bytes_corrected": round(fetch), "write_bytes": round(write),
                        "hbm_bytes_per_launch": round(fetch + write), "dispatches": [nf, nw]}
    json.dump({"source": d, "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes; full-batch dispatches "
               "(>= half the kernel's longest duration) averaged", "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
