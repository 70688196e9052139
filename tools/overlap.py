"""Which kernels run concurrently with a given kernel in a rocprofv3 kernel trace (one step).

    python tools/overlap.py run_kernel_trace.csv KERNEL_SUBSTRING [step_index]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\((.*)", "", n)[:60]


def main(path, key, k=6):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    idx = [i for i, n in enumerate(names) if "swin_attn_fwd" in n]
    a, b = idx[::36][k], idx[::36][k + 1]
    step = rows[a:b]
    tot = collections.Counter()
    cnt = 0
    dur = []
    for r in step:
        if key not in r["Kernel_Name"]:
            continue
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur.append((e0 - s0) / 1e3)
        cnt += 1
        for o in step:
            if o is r:
                continue
            s1, e1 = int(o["Start_Timestamp"]), int(o["End_Timestamp"])
            ov = min(e0, e1) - max(s0, s1)
            if ov > 0:
                tot[short(o["Kernel_Name"])] += ov / 1e3
    print(f"{key}: {cnt} launches, mean {sum(dur) / max(1, cnt):.1f} us, min {min(dur):.1f}, max {max(dur):.1f}")
    print("  durations:", " ".join(f"{d:.0f}" for d in dur))
    for n, v in tot.most_common(8):
        print(f"  overlapped by {n:60s} {v:8.1f} us total")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 6)
