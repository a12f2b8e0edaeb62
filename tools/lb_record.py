"""Large-batch (configs[4] share: B=512, k=50, 25,600 sample rows) kernel record
for bench.py's `large_batch.kernels`: per kernel of the step its average
duration (rocprofv3 kernel trace of tools/train_large.py), its algorithmic
work per launch and the fraction of the roofline that bounds it, plus the HBM
bytes per launch from the PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
tools/pmc_by_grid.py) where present.
    python tools/lb_record.py <kernel_trace.csv> <pmc_by_grid.json|-> <out.json>"""
import csv
import json
import re
import sys
from collections import defaultdict

ROWS = 512 * 50
BF16X3_PEAK = 2500.0 / 3          # TFLOP/s: bf16 dense / 3 MFMAs per bf16x3 product
HBM_PEAK = 8000.0                 # GB/s
# algorithmic FLOP per launch (2 x rows x MACs per row of the kernel's Dense products)
SAMPLE_MACS = 281_800             # forward: every sample-row Dense layer (2L, k=50)
OUT_BWD_MACS = 784 * 200 + 200 * 200 + 200 * 100
ENC_PRIOR_BWD_MACS = 200 * 100 + 100 * 100 + 100 * 50 + 100 * 100 + 100 * 100 + 100 * 100
WGRAD_MACS = 3 * 101 * 100 + 51 * 100 + 101 * 100 + 101 * 200 + 101 * 200 + 201 * 200 + 201 * 784
KERNELS = [
    # (label, kernel-name regex, workgroups or None, bound, algorithmic work per launch)
    ("ring forward, train mode (nring_kernel)", r"nring_kernel<0, false, true>", None, "mfma",
     2.0 * ROWS * SAMPLE_MACS),
    ("output-MLP backward-data (nrb_kernel)", r"nrb_kernel<0>", None, "mfma", 2.0 * ROWS * OUT_BWD_MACS),
    ("encoder / prior backward-data (nre_kernel)", r"nre_kernel", None, "mfma", 2.0 * ROWS * ENC_PRIOR_BWD_MACS),
    ("weight gradients (dw_kernel)", r"dw_kernel", None, "mfma", 2.0 * ROWS * WGRAD_MACS),
    ("weight gradients (upd_kernel slab pass)", r"upd_kernel", 600, "mfma", 2.0 * ROWS * WGRAD_MACS),
    ("Adam over the slabs (adam_kernel)", r"adam_kernel", None, "hbm", None),
]


def main():
    trace, pmc_path, out = sys.argv[1], sys.argv[2], sys.argv[3]
    dur = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        w = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        dur[(r["Kernel_Name"].split("(")[0], g // max(1, w))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = json.load(open(pmc_path)) if pmc_path != "-" else {}
    rec = {}
    for label, rx, wg, bound, work in KERNELS:
        hits = [(k, v) for k, v in dur.items() if re.search(rx, k[0]) and (wg is None or k[1] == wg)]
        if not hits:
            continue
        (name, nwg), d = max(hits, key=lambda kv: len(kv[1]))
        d = sorted(d)[1:] if len(d) > 3 else d           # drop the first (cold) launch
        us = sum(d) / len(d)
        e = dict(kernel=name, workgroups=nwg, launches=len(d), avg_us=round(us, 2), bound=bound)
        p = next((v for k, v in pmc.items() if k.startswith(name.replace("void ", "")[:60]) and k.endswith(f"wg {nwg}")),
                 None)
        if p and "hbm_MB" in p["derived"]:
            e["hbm_MB_per_launch"] = round(p["derived"]["hbm_MB"], 2)
            e["hbm_GBps"] = round(p["derived"]["hbm_MB"] / 1e3 / (us * 1e-6), 1)
        if work is not None:
            tf = work / (us * 1e-6) / 1e12
            e.update(flop_per_launch=work, tflops=round(tf, 2), peak_tflops=round(BF16X3_PEAK, 1),
                     frac=round(tf / BF16X3_PEAK, 4))
        elif "hbm_GBps" in e:
            e.update(frac=round(e["hbm_GBps"] / HBM_PEAK, 4), peak_GBps=HBM_PEAK)
        rec[label] = e
    json.dump(dict(source=trace, rows=ROWS, kernels=rec), open(out, "w"), indent=1)
    for k, v in rec.items():
        print(f"{k:48s} {v['avg_us']:8.2f} us  frac {v.get('frac')}")


if __name__ == "__main__":
    main()
