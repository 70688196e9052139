"""Per-step kernel time vs wall time from a rocprofv3 kernel trace of bench.py (graph replays).

    python tools/step_gaps.py <run_kernel_trace.csv> [kernels_per_step_marker]

Finds the adam_ema launches (one per training step), and for each step between two of them
reports the wall span, the summed kernel durations and the idle gaps between kernels."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_ema" in r["Kernel_Name"]]
    for a, b in zip(ends[-4:-1], ends[-3:]):
        seg = rows[a + 1:b + 1]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        gaps, last = [], int(seg[0]["Start_Timestamp"])
        for r in seg:
            s = int(r["Start_Timestamp"])
            gaps.append(max(0, s - last))
            last = max(last, int(r["End_Timestamp"]))
        gaps.sort()
        print(f"kernels {len(seg)} wall {(t1 - t0) / 1e6:.3f} ms busy {busy / 1e6:.3f} ms idle {sum(gaps) / 1e6:.3f} ms "
              f"median gap {gaps[len(gaps) // 2] / 1e3:.1f} us p90 {gaps[int(len(gaps) * .9)] / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
