"""Kernel timeline of one bench step from a rocprofv3 kernel_trace.csv: durations and
the idle gaps between kernels (host-bound stretches show up as gaps).
python tools/step_gaps.py <kernel_trace.csv> <substring of the step's first kernel>"""
import csv
import sys


def main(path, anchor):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    a, b = idx[-3], idx[-2]
    t0 = int(rows[a]["Start_Timestamp"])
    prev = None
    busy = gaps = 0.0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        busy += (e - s) / 1e3
        gaps += max(gap, 0.0)
        print(f"{(s - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} gap {gap:7.1f}  {r['Kernel_Name'][:70]}")
        prev = e
    print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us: kernels {busy:.1f} us, "
          f"gaps {gaps:.1f} us, {b - a} launches")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
