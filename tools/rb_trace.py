"""Phase timeline of workgroup 0 of every fused-kernel job in one eager train
step of the bench workload.  Needs a library built with -DIWAE_RB_TRACE:

    IWAE_HIPCC_FLAGS=-DIWAE_RB_TRACE python -c "import __graft_entry__ as g; g.build(True)"
    python tools/rb_trace.py
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
dump = m._lib.iwae_rb_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16384)()
for i in range(5):
    m.train_step(x[i * 20:(i + 1) * 20])
    n = dump(buf, 16384)
a = np.array(buf[:n], dtype=np.int64).reshape(-1, 32)
t0 = a[:, 1].min()
for r in a:
    kind, jb = int(r[0]) >> 8, int(r[0]) & 255
    start = int(r[1])
    ph = " ".join(f"{j}:{(int(r[j]) - start) / 100:.2f}" for j in list(range(2, 8)) + [31] if r[j] > 0)
    print(f"{'fwd' if kind == 1 else 'bwd'} job{jb} @{(start - t0) / 100:8.2f}us  {ph}")
    for s in range(5):
        b = 8 + 4 * s
        if r[b] > 0:
            print(f"      stage{s}: enter {(int(r[b]) - start) / 100:.2f} issued +{(int(r[b + 1]) - int(r[b])) / 100:.2f} "
                  f"mfma-done +{(int(r[b + 2]) - int(r[b + 1])) / 100:.2f} epilogue +{(int(r[b + 3]) - int(r[b + 2])) / 100:.2f}")
