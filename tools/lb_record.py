"""Large-batch (configs[4] share: B=512, k=50, 25,600 sample rows) kernel record
for bench.py's `large_batch.kernels`: per kernel of the step its average
duration (rocprofv3 kernel trace of tools/train_large.py), its algorithmic
work per launch (bench.kernel_work: FLOP and algorithmic HBM bytes) and the
fraction of the roofline its FLOP / byte ratio puts it under, plus the HBM
bytes per launch from the PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
tools/pmc_by_grid.py) where present.
    python tools/lb_record.py <kernel_trace.csv> <pmc_by_grid.json|-> <out.json>"""
import csv
import os
import json
import re
import sys
from collections import defaultdict

ROWS, IMAGES = 512 * 50, 512
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (the roofline model: kernel_work, roofline_of)

KERNELS = [
    # (label, kernel-name regex, workgroups or None, bench.kernel_work kind or None)
    ("ring forward, train mode (nring_kernel)", r"nring_kernel<0, false, true>", None, "fwd"),
    ("output-MLP backward-data (nrb_kernel)", r"nrb_kernel<0>", None, "nrb"),
    ("encoder / prior backward-data (nre_kernel)", r"nre_kernel", None, "nre"),
    ("ring backward-data, output MLP + encoder / prior (nrbe_kernel)", r"nrbe_kernel", None, "nrbe"),
    ("weight gradients (dw_kernel)", r"dw_kernel", None, "dw"),
    ("first-layer weight gradients + Adam + FX copies (upd_kernel)", r"upd_kernel", None, None),
    ("first encoder layer input GEMM, split-K slabs (gemm_kernel)", r"gemm_kernel", None, None),
    ("bound / loss reduction (bound_kernel)", r"bound_kernel", None, None),
    ("first encoder layer l2 / head, image rows (tc_kernel I)", r"tc_kernel<1>#0", 256, "img_fwd"),
    ("first encoder layer backward, image rows (tc_kernel I')", r"tc_kernel<1>#1", 256, "img_bwd"),
    ("Adam over the slabs (adam_kernel)", r"adam_kernel", None, None),
]


def work(kind):
    if kind == "nrbe":
        f1, b1 = bench.kernel_work("nrb", ROWS, IMAGES)
        f2, b2 = bench.kernel_work("nre", ROWS, IMAGES)
        return f1 + f2, b1 + b2
    return bench.kernel_work(kind, ROWS, IMAGES)


def main():
    trace, pmc_path, out = sys.argv[1], sys.argv[2], sys.argv[3]
    dur = defaultdict(list)
    seen = defaultdict(int)
    for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"])):
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        w = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        name = r["Kernel_Name"].split("(")[0]
        if re.search(r"tc_kernel<1(, \d+u)?>$", name) and g // max(1, w) == 256:
            # the step's two image-row launches alternate: job I (forward) then job I' (backward);
            # the kind-mask template argument (kTcKindsFwd / kTcKindsImgBwd) is dropped from the label
            base = re.sub(r"tc_kernel<1(, \d+u)?>$", "tc_kernel<1>", name)
            name = base + f"#{seen[base] % 2}"
            seen[base] += 1
        dur[(name, g // max(1, w))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = json.load(open(pmc_path)) if pmc_path != "-" else {}
    rec = {}
    for label, rx, wg, kind in KERNELS:
        hits = [(k, v) for k, v in dur.items() if re.search(re.escape(rx) if "#" in rx else rx, k[0])
                and (wg is None or k[1] == wg)]
        if not hits:
            continue
        (name, nwg), d = max(hits, key=lambda kv: len(kv[1]))
        d = sorted(d)[1:] if len(d) > 3 else d           # drop the first (cold) launch
        us = sum(d) / len(d)
        e = dict(kernel=name, workgroups=nwg, launches=len(d), avg_us=round(us, 2))
        p = next((v for k, v in pmc.items() if k.startswith(name.replace("void ", "")[:60]) and k.endswith(f"wg {nwg}")),
                 None)
        if p and "hbm_MB" in p["derived"]:
            e["hbm_MB_per_launch"] = round(p["derived"]["hbm_MB"], 2)
            e["hbm_GBps"] = round(p["derived"]["hbm_MB"] / 1e3 / (us * 1e-6), 1)
        if kind is not None:
            fl, nb = work(kind)
            r = bench.roofline_of(fl, nb, us)
            e.update(bound=r["bound"], frac=r["frac"], achieved=r["achieved"], unit=r["unit"], peak=r["peak"],
                     flop_per_launch=fl, alg_MB_per_launch=round(nb / 1e6, 2), flop_per_byte=r["flop_per_byte"],
                     tflops=round(fl / (us * 1e-6) / 1e12, 2), mfma_frac=round(fl / (us * 1e-6) / 1e12 / 833.3, 4))
            if "hbm_MB_per_launch" in e:
                e["traffic_over_alg"] = round(e["hbm_MB_per_launch"] * 1e6 / nb, 2)
        elif "hbm_GBps" in e:
            e.update(bound="hbm", frac=round(e["hbm_GBps"] / 8000.0, 4), peak=8000.0, unit="GB/s")
        rec[label] = e
    json.dump(dict(source=trace, rows=ROWS, kernels=rec), open(out, "w"), indent=1)
    for k, v in rec.items():
        print(f"{k:48s} {v['avg_us']:8.2f} us  frac {v.get('frac')}")


if __name__ == "__main__":
    main()
