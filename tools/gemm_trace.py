"""Per-workgroup phase times of the train step's Bernoulli GEMM (one eager
step of the bench workload).  Needs the -DIWAE_GEMM_TRACE debug library:

    bash tools/build_debug.sh -DIWAE_GEMM_TRACE
    IWAE_HIP_LIB=tools/_dbg/libiwae_dbg.so python tools/gemm_trace.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

x, pi = bench.synthetic_images(bench.B_PER_GPU * 8, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K,
                   seed=2, use_graphs=False)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
dump = m._lib.iwae_gemm_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 32768)()
for i in range(6):
    m.train_step(x[i * 20:(i + 1) * 20])
    n = dump(buf, 32768)
a = np.array(buf[:n], dtype=np.int64).reshape(-1, 8)
t0 = a[:, 1].min()
st = (a[:, 1] - t0) / 100.0
pro = (a[:, 2] - a[:, 1]) / 100.0
loop = (a[:, 3] - a[:, 2]) / 100.0
epi = (a[:, 4] - a[:, 3]) / 100.0
ecomp = (a[:, 5] - a[:, 3]) / 100.0
ered = (a[:, 6] - a[:, 5]) / 100.0
etail = (a[:, 4] - a[:, 6]) / 100.0
end = (a[:, 4] - t0) / 100.0
print(f"workgroups {len(a)}; span {end.max():.2f} us (first start -> last end)")
rows = [("start offset", st), ("prologue load", pro), ("main loop", loop), ("epilogue", epi)]
if (a[:, 5] > 0).all() and (a[:, 6] > 0).all():      # debug builds with the finer epilogue stamps
    rows += [("  elementwise", ecomp), ("  row reduce", ered), ("  tail", etail)]
rows.append(("end", end))
for name, v in rows:
    print(f"  {name:14s} min {v.min():6.2f}  med {np.median(v):6.2f}  max {v.max():6.2f} us")
