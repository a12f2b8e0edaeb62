"""Turn rocprofv3 PMC passes (tools/pmc_passes.sh output) into the per-launch
HBM traffic record bench.py reports as roofline.traffic.

FETCH_SIZE is in KiB per dispatch and is doubled (gfx950 tallies a 128-B wide
streaming request as 64 B: MI355X_MICROARCH.md, HBM section); WRITE_SIZE is
taken as is (exact for 16-B-per-lane streaming stores).

    python tools/pmc_to_json.py gpurun_out/pmc_train "gemm_kernel<2, 2, 1, 1, false, false, 2," profiles/r01_pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys

root, match, out = sys.argv[1], sys.argv[2], sys.argv[3]
vals = {}
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if match in r.get("Kernel_Name", ""):
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
rec = {
    "kernel_match": match,
    "dispatches": len(vals.get("FETCH_SIZE", [])),
    "fetch_bytes": 2 * avg["FETCH_SIZE"] * 1024,
    "write_bytes": avg["WRITE_SIZE"] * 1024,
    "note": "per launch; FETCH_SIZE x2 (gfx950 128-B request tally), WRITE_SIZE as is; rocprofv3 --pmc passes "
            "of tools/pmc_passes.sh over the same bench command (no NLL, no CPU leg)",
}
rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
for k in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"):
    if k in avg:
        rec[k] = avg[k]
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
