"""Per-workgroup timeline of the combined image-row backward + update launch
(tcu_kernel) in eager B=20 train steps: job I' blocks (start, body done, after
the publish), update tiles (start, in-launch wait done for the first encoder
layer's tiles, end).  Needs a -DIWAE_TCU_TRACE build (tools/build_debug.sh),
run with IWAE_HIP_LIB pointing at it.  Usage: python tools/tcu_trace.py [B]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else bench.B_PER_GPU
x, pi = bench.synthetic_images(B * 8, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K,
                   seed=2, use_graphs=False)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
dump = m._lib.iwae_tcu_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * (512 * 4))()
for i in range(6):
    m.train_step(x[(i % 8) * B:(i % 8 + 1) * B])
    dump(buf, 512 * 4)
a = np.array(buf[:], dtype=np.int64).reshape(512, 4)
live = a[:, 0] > 0
t0 = a[live, 0].min()
names = {0: "I'", 1: "heavy", 2: "light"}
for role in (0, 1, 2):
    sel = np.where(live & (a[:, 3] == role))[0]
    if len(sel) == 0:
        continue
    st = (a[sel, 0] - t0) / 100.0
    mid = (a[sel, 1] - t0) / 100.0
    en = (a[sel, 2] - t0) / 100.0
    print(f"{names[role]:6s} n={len(sel):4d}  start {st.min():6.2f}..{st.max():6.2f}  "
          f"mid {mid.min() if role != 1 else 0:6.2f}..{mid.max() if role != 1 else 0:6.2f}  end {en.min():6.2f}..{en.max():6.2f} us")
print(f"launch span {((a[live, 2].max() - t0) / 100.0):.2f} us")
