"""Kernel timeline of the last train step in a rocprofv3 kernel trace
(results .db or kernel_trace .csv): start offset, gap to the previous
kernel's end, duration, workgroups.  Usage:
    python tools/step_timeline.py <trace.db|kernel_trace.csv> [n_kernels] [first_kernel_substring]
The step starts at the last launch whose name contains first_kernel_substring
(default: the last n_kernels launches)."""
import csv
import re
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, s, e, gx, wx) for n, s, e, gx, wx in
                c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start")]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                     int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)))
    rows.sort(key=lambda r: r[1])
    return rows


def main():
    rows = load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    first = sys.argv[3] if len(sys.argv) > 3 else None
    if first:
        idx = max(i for i, r in enumerate(rows) if first in r[0])
        sel = rows[idx:idx + n]
    else:
        sel = rows[-n:]
    t0, prev, busy = sel[0][1], None, 0
    for name, s, e, gx, wx in sel:
        short = re.sub(r"\(.*", "", name)[:60]
        gap = (s - prev) / 1000 if prev is not None else 0.0
        busy += e - s
        print(f"{(s - t0) / 1000:8.2f}  gap {gap:6.2f}  dur {(e - s) / 1000:7.2f}  wg {gx // max(wx, 1):6d}  {short}")
        prev = e
    print(f"span {(sel[-1][2] - t0) / 1000:.2f} us, kernels {busy / 1000:.2f} us")


if __name__ == "__main__":
    main()
