"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv:
python tools/pmc_kernel.py <csv> [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for r in rows:
    k = r["Kernel_Name"]
    if sub not in k:
        continue
    key = (k[:48], r["Grid_Size"])
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[key][r["Counter_Name"]] += 1
for key, v in agg.items():
    print(key[0], key[1], " ".join(f"{c}={v[c] / cnt[key][c]:.0f}" for c in sorted(v)))
