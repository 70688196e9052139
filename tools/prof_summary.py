"""Summarise a rocprofv3 kernel-trace database: per-kernel totals, per-step share.

    python tools/prof_summary.py <run_results.db> [steps]
"""
import collections
import sqlite3
import sys


def main(db, steps=None):
    con = sqlite3.connect(db)
    rows = con.execute("select name, grid_x, duration from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, gx, d in rows:
        short = n.replace("(anonymous namespace)::", "")
        short = short.split("(")[0] if short.startswith("void") is False else short[5:].split("(")[0]
        agg[short][0] += 1
        agg[short][1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot / 1e6:.2f} ms over {len(rows)} dispatches")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        per = f" {t / 1e6 / steps:8.3f} ms/step" if steps else ""
        print(f"{t / 1e6:9.2f} ms {100 * t / tot:5.1f}% n={n:6d} avg={t / n / 1e3:8.1f} us{per}  {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
