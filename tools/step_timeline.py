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
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        gy = int(r.get("Grid_Size_Y", 1) or 1) // max(1, int(r.get("Workgroup_Size_Y", 1) or 1))
        rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), gx * gy, wx))
    rows.sort(key=lambda r: r[1])
    return rows


def main():
    rows = load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    first = sys.argv[3] if len(sys.argv) > 3 else None
    if first:
        # "name" or "name@workgroups"; the last such launch with n launches after it
        name, _, wg = first.partition("@")
        hit = [i for i, r in enumerate(rows) if name in r[0] and (not wg or r[3] // max(r[4], 1) == int(wg))]
        full = [i for i in hit if i + n <= len(rows)]
        idx = max(full or hit)
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
