"""Where a training step's GPU time goes, from a rocprofv3 --kernel-trace CSV of bench.py.

    python tools/step_breakdown.py KERNEL_TRACE_CSV [TOP]

Takes the middle of the run (40 %..85 % of the dispatches: graph-replayed timed steps), counts steps by the Adam
kernel, and prints per step: the span, the GPU-busy union of all kernels, the summed kernel time, and the kernels by
summed duration (launches per step, mean duration).
"""
import collections
import csv
import sys


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    w = rows[int(len(rows) * 0.40):int(len(rows) * 0.85)]
    steps = sum(1 for r in w if "adam_ema" in r["Kernel_Name"])
    t0 = int(w[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in w)
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in w]
    busy = union(iv)
    ksum = sum(e - s for s, e in iv)
    print(f"{steps} steps: {(t1 - t0) / steps / 1e3:.1f} us span per step, GPU busy {busy / steps / 1e3:.1f} us, "
          f"kernel time {ksum / steps / 1e3:.1f} us, {len(w) / steps:.1f} launches")
    per = collections.defaultdict(lambda: [0, 0])
    for r in w:
        d = per[r["Kernel_Name"]]
        d[0] += 1
        d[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, (n, ns) in sorted(per.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{ns / steps / 1e3:9.1f} us/step {n / steps:6.1f}x {ns / n / 1e3:8.2f} us  {name[:110]}")


if __name__ == "__main__":
    main()
