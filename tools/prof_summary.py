"""Summarise a rocprofv3 kernel_stats.csv (and per-step view from kernel_trace)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    per = f"{float(r['TotalDurationNs']) / 1e3 / steps:8.2f}us/step" if steps else ""
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms n={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:9.2f}us "
          f"{per} {r['Name'][:100]}")
print(f"total {tot/1e6:.3f} ms")
