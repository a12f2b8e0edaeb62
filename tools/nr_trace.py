"""Per-unit timeline of the weight-ring NLL kernel (nring_kernel) from a
-DIWAE_NR_TRACE build (OUT=libiwae_nrtrace.so bash tools/build_debug.sh
-DIWAE_NR_TRACE; run with IWAE_HIP_LIB=tools/_dbg/libiwae_nrtrace.so):
waves 0 and 7 of workgroups 0 and 3000, s_memtime cycles per unit spent
waiting (vmcnt + barrier), multiplying, and in the epilogue until the next unit."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

x, pi = bench.synthetic_images(209, 3)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2)
m.log_px(x, 5000)
m.log_px(x, 5000)
dump = m._lib.iwae_nr_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NU = 512
buf = (ctypes.c_ulonglong * (4 * NU * 3))()
n = dump(buf, 4 * NU * 3)
T = np.array(buf[:n], dtype=np.int64).reshape(4, NU, 3)
for rec in range(4):
    t0 = T[rec, NU - 1, 0]
    if t0 == 0:
        continue
    nu = int(np.max(np.nonzero(T[rec, :NU - 1, 0])[0])) + 1
    e, b, d = T[rec, :nu, 0], T[rec, :nu, 1], T[rec, :nu, 2]
    wait = b - e
    mma = d - b
    epi = np.append(e[1:] - d[:-1], 0)
    print(f"rec {rec}: units {nu}, total {T[rec, nu - 1, 2] - t0} cyc, prologue {T[rec, NU - 1, 1] - t0}, "
          f"first unit entry {e[0] - t0}; sum wait {wait.sum()} mma {mma.sum()} epi {epi.sum()}")
    for u in range(nu):
        print(f"  u{u:3d} wait {wait[u]:6d} mma {mma[u]:6d} epi {epi[u]:6d}")
