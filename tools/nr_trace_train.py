"""Per-unit timeline of the ring forward in TRAIN mode (nring_kernel<..., TR>)
at the large-batch step (B = 512, k = 50) from a -DIWAE_NR_TRACE build
(OUT=libnrtr.so bash tools/build_debug.sh -DIWAE_NR_TRACE; run with
IWAE_HIP_LIB=<that library>): waves 0 and 7 of workgroup 0, s_memtime cycles
per unit in the group wait, the MFMA phase and the epilogue, summed per stage."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
x, pi = bench.synthetic_images(B, 1)
# the ring backward kernels share the trace buffer: the engine backward instead
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                   tuning={"nring_bwd": 0})
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
for i in range(3):
    m.train_step(xd)
torch.cuda.synchronize()
dump = m._lib.iwae_nr_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NU = 512
buf = (ctypes.c_ulonglong * (4 * NU * 3))()
n = dump(buf, 4 * NU * 3)
T = np.array(buf[:n], dtype=np.int64).reshape(4, NU, 3)
STAGES = [("e1", 7), ("e2", 7), ("eh", 7), ("p1", 7), ("p2", 7), ("ph", 13), ("o1", 13), ("o2", 13), ("bern", 49)]
for rec in range(2):
    t0 = T[rec, NU - 1, 0]
    if t0 == 0:
        continue
    nu = int(np.max(np.nonzero(T[rec, :NU - 1, 0])[0])) + 1
    e, b, d = T[rec, :nu, 0], T[rec, :nu, 1], T[rec, :nu, 2]
    wait, mma, epi = b - e, d - b, np.append(e[1:] - d[:-1], 0)
    print(f"rec {rec}: units {nu}, total {T[rec, nu - 1, 2] - t0} cyc, prologue {T[rec, NU - 1, 1] - t0}; "
          f"sum wait {wait.sum()} mma {mma.sum()} epi {epi.sum()}")
    u = 0
    for name, cnt in STAGES:
        sl = slice(u, min(u + cnt, nu))
        print(f"  {name:5s} units {cnt:3d}: wait {wait[sl].sum():7d} mma {mma[sl].sum():7d} epi {epi[sl].sum():7d}"
              f"  per unit {(wait[sl].sum() + mma[sl].sum() + epi[sl].sum()) / cnt:7.0f}")
        u += cnt
