"""Does the bench line's roofline follow from the committed rocprofv3 summary of the same command?

    python tools/roofline_check.py BENCH_LINE_FILE KERNEL_STATS_CSV

For the kernel rocprofv3 ranks first (largest summed duration), prints its mean duration there and the line's
kernel_ms for it, and the HBM fraction each implies with the line's algorithmic bytes per launch
(bytes / mean / 8 TB/s).  Exit status 1 when the line's roofline kernel is not rocprof's first, or the two
fractions differ by more than 5 %.
"""
import csv
import json
import sys

PEAK_HBM_GBS = 8000.0


def main():
    line_path, stats_path = sys.argv[1], sys.argv[2]
    with open(line_path) as f:
        line = json.loads(next(ln for ln in f if ln.startswith("{")))
    with open(stats_path) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    top = rows[0]
    roof = line["roofline"]
    sym = roof.get("symbol", "")
    same = sym == top["Name"] or roof["kernel"] in top["Name"]
    rp_ms = float(top["AverageNs"]) * 1e-6
    print(f"rocprof first : {top['Name'][:110]}")
    print(f"                calls {top['Calls']}, mean {rp_ms * 1e3:.2f} us, {top['Percentage']} % of kernel time")
    print(f"line roofline : {roof['kernel']}  kernel_ms {roof['kernel_ms'] * 1e3:.2f} us, frac {roof.get('frac')}")
    ok = same
    if roof.get("bytes_per_launch"):
        f_rp = roof["bytes_per_launch"] / (rp_ms * 1e-3) / 1e9 / PEAK_HBM_GBS
        dev = abs(roof["frac"] - f_rp) / f_rp
        print(f"bytes / rocprof mean / 8 TB/s = {f_rp:.4f}; the line's frac deviates {100 * dev:.1f} %")
        ok = ok and dev <= 0.05
    if roof.get("flops_per_launch"):
        print(f"FLOPs / rocprof mean = {roof['flops_per_launch'] / (rp_ms * 1e-3) / 1e12:.1f} TFLOP/s "
              f"(line: {roof.get('achieved_tflops')})")
    for r in rows[1:6]:
        print(f"  next: {float(r['AverageNs']) / 1e3:8.2f} us x {r['Calls']:>6}  {r['Percentage']:>6} %  {r['Name'][:90]}")
    print("kernel" + (" matches" if same else " DIFFERS") + ("; agreement within 5 %" if ok else "; NOT within 5 %"))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
