"""Per-stage cycle timeline (s_memtime) of the fused NLL kernel for 4 sampled
workgroups, every wave.  Needs the -DIWAE_MG_TRACE debug library:

    OUT=libiwae_mgtrace.so bash tools/build_debug.sh -DIWAE_MG_TRACE
    IWAE_HIP_LIB=tools/_dbg/libiwae_mgtrace.so python tools/mg_trace.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

x, pi = bench.synthetic_images(400, 99)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2)
xd = m._x(x)
m.log_px(xd, 5000)
m.log_px(xd, 5000)
torch.cuda.synchronize()
dump = m._lib.iwae_mg_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 4096)()
n = dump(buf, 4096)
a = np.array(buf[:n], dtype=np.int64).reshape(4, 8, 128)
names = ["enc l1", "enc l2", "enc head", "dec l1", "dec l2", "dec head", "out l1", "out l2", "out 784"]
for b in range(4):
    t0 = a[b, :, 0].min()
    if t0 <= 0:
        continue
    end = a[b, :, 127].max() - t0
    print(f"workgroup sample {b}: total {end} cycles; prologue {a[b, :, 1].max() - t0}")
    for s, nm in enumerate(names):
        ent = a[b, :, 2 + 3 * s] - t0
        dn = a[b, :, 3 + 3 * s] - t0
        br = a[b, :, 4 + 3 * s] - t0
        work = dn - ent
        print(f"  {nm:9s} enter {ent.min():7d}  work per wave min/max {work.min():6d}/{work.max():6d}  "
              f"barrier done {br.max():7d}  (stage {br.max() - ent.min():6d})")
        f0, f1, f2 = a[b, :, 64 + 4 * s], a[b, :, 65 + 4 * s], a[b, :, 66 + 4 * s]
        ok = (f0 > 0) & (f1 > 0) & (f2 > 0)
        if ok.any():
            fetch = (f0 - (a[b, :, 2 + 3 * s]))[ok]
            mma = (f1 - f0)[ok]
            epi = (f2 - f1)[ok]
            print(f"            first tile: fetch-wait {int(np.median(fetch)):6d}  mfma-loop {int(np.median(mma)):6d}  "
                  f"epilogue {int(np.median(epi)):6d}  (medians over waves)")
