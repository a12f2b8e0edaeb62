"""Average duration per (kernel, grid size) from a rocprofv3 kernel_trace.csv,
so one kernel's launches at different shapes (the train engine's forward and
backward launches, the bench's three workloads) are not mixed.
    python tools/kernel_by_grid.py <run_kernel_trace.csv> [name substring]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(list)
for r in csv.DictReader(open(path)):
    if match in r["Kernel_Name"]:
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0))) * int(r.get("Grid_Size_Y", 1) or 1)
        w = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1))) * int(r.get("Workgroup_Size_Y", 1) or 1)
        acc[(r["Kernel_Name"][:70], g // max(1, w))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, wg), d in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    d.sort()
    print(f"{name:70s} wg {wg:7d} n {len(d):6d} avg {sum(d) / len(d):9.3f} us  median {d[len(d) // 2]:9.3f} us  "
          f"total {sum(d) / 1e3:9.3f} ms")
