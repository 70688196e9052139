"""Per-step kernel time breakdown from a rocprofv3 kernel trace of bench.py.

    python tools/step_breakdown.py gpurun_out/qprof/run_kernel_trace.csv [step_index]
A step is delimited by consecutive first-block launches of the fused attention kernel (or the first
LayerNorm when the fused path is off)."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\((.*)", "", n)
    return n[:70]


def main(path, k=5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    key = "swin_attn_fwd" if any("swin_attn_fwd" in n for n in names) else "layernorm_fwd"
    idx = [i for i, n in enumerate(names) if key in n]
    per = 36 if key == "swin_attn_fwd" else None
    starts = idx[::per] if per else idx
    a, b = starts[k], starts[k + 1]
    t = collections.defaultdict(float)
    c = collections.Counter()
    for r in rows[a:b]:
        s = short(r["Kernel_Name"])
        t[s] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c[s] += 1
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    tot = sum(t.values())
    print(f"step span {span / 1e3:.3f} ms, kernel time {tot / 1e3:.3f} ms, {b - a} launches")
    for s, v in sorted(t.items(), key=lambda x: -x[1]):
        print(f"{v / 1e3:8.3f} ms {100 * v / tot:5.1f}% {c[s]:4d}x {v / c[s]:8.1f} us  {s}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
