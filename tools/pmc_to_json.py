"""Turn rocprofv3 PMC passes (tools/pmc_passes.sh output) into the per-launch
HBM traffic records bench.py reports as roofline.traffic.

FETCH_SIZE is in KiB per dispatch and is doubled (gfx950 tallies a 128-B wide
streaming request as 64 B: MI355X_MICROARCH.md, HBM section); WRITE_SIZE is
taken as is (exact for 16-B-per-lane streaming stores).

    python tools/pmc_to_json.py <pmc dir> <kernel name substring> <out.json> <label> [grid: threads | max | min | rank:n]

The record is merged into out.json under `label` (the kernel label bench.py
uses); the grid size separates launches of one kernel with different roles
(the train engine's forward and backward launches)."""
import csv
import glob
import json
import os
import sys

root, match, out, label = sys.argv[1:5]
grid = sys.argv[5] if len(sys.argv) > 5 else None     # threads, or "max" / "min" over the matching launches
rows = [r for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)
        for r in csv.DictReader(open(f)) if match in r.get("Kernel_Name", "")]
if grid in ("max", "min"):
    sizes = {int(r["Grid_Size"]) for r in rows}
    grid = max(sizes) if grid == "max" else min(sizes)
elif grid is not None and grid.startswith("rank:"):        # the n-th largest grid (0 = max)
    sizes = sorted({int(r["Grid_Size"]) for r in rows}, reverse=True)
    grid = sizes[int(grid[5:])]
elif grid is not None:
    grid = int(grid)
vals = {}
for r in rows:
    if grid is None or int(r["Grid_Size"]) == grid:
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
rec = {
    "kernel_match": match,
    "grid_size": grid,
    "dispatches": len(vals.get("FETCH_SIZE", [])),
    "fetch_bytes": 2 * avg["FETCH_SIZE"] * 1024,
    "write_bytes": avg["WRITE_SIZE"] * 1024,
    "note": "per launch; FETCH_SIZE x2 (gfx950 128-B request tally), WRITE_SIZE as is; rocprofv3 --pmc passes "
            "of tools/pmc_passes.sh over the bench's train-step command (no NLL, no CPU leg)",
}
rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
for k in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES",
          "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_WAVES"):
    if k in avg:
        rec[k] = avg[k]
data = {}
if os.path.exists(out):
    with open(out) as fh:
        data = json.load(fh)
    if "kernel_match" in data:          # older single-record layout
        data = {}
data[label] = rec
with open(out, "w") as fh:
    json.dump(data, fh, indent=1)
print(label, json.dumps(rec, indent=1))
