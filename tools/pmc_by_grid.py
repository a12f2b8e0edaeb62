"""Per (kernel, workgroup count) averages of rocprofv3 PMC passes
(<root>/<pass>/**/*counter_collection.csv), so one kernel's launches at
different shapes (e.g. upd_kernel's B=20 update and its large-batch slab
pass) are not mixed.  FETCH_SIZE is doubled (gfx950 tallies 128-B requests
at 64 B, MI355X_MICROARCH.md); derived: HBM MB per dispatch, wait and LDS
conflict fractions, VALU per MFMA.
    python tools/pmc_by_grid.py <root> [name substring] [--json out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
jout = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if match and match not in k:
            continue
        g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        w = int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 1)) or 1)
        acc[(k.split("(")[0][:70], g // max(1, w))][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for (k, wg), cs in sorted(acc.items(), key=lambda kv: -max(len(v) for v in kv[1].values())):
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    n = max(len(v) for v in cs.values())
    d = {}
    if "FETCH_SIZE" in a:
        d["fetch_MB"] = 2 * a["FETCH_SIZE"] / 1024
    if "WRITE_SIZE" in a:
        d["write_MB"] = a["WRITE_SIZE"] / 1024
    if "fetch_MB" in d and "write_MB" in d:
        d["hbm_MB"] = d["fetch_MB"] + d["write_MB"]
    if a.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in a:
                d[c + "/wave_cycles"] = a[c] / a["SQ_WAVE_CYCLES"]
    if a.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_frac"] = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"]
    if a.get("SQ_INSTS_MFMA"):
        d["valu_per_mfma"] = a.get("SQ_INSTS_VALU", 0.0) / a["SQ_INSTS_MFMA"]
    if a.get("TCC_HIT_sum") is not None and a.get("TCC_MISS_sum") is not None:
        d["tcc_hit_rate"] = a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
    print(f"{k}  wg {wg}  (dispatches {n})")
    for c in sorted(a):
        print(f"    {c:28s} {a[c]:16.1f}")
    for c, v in d.items():
        print(f"    = {c:26s} {v:16.4f}")
    out[f"{k} wg {wg}"] = dict(counters=a, derived=d, dispatches=n)
if jout:
    json.dump(out, open(jout, "w"), indent=1)
