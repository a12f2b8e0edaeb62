"""Per-unit timeline of the ring encoder / prior backward (nre_kernel) of a
B = 512 train step, from the -DIWAE_NR_TRACE build (s_memtime, waves 0 and 7
of workgroup 0): prologue (Gaussian backward of the prior), ring phase A,
drain + the encoder's Gaussian backward, ring phase B.
  OUT=libiwae_nrtrace.so bash tools/build_debug.sh -DIWAE_NR_TRACE
  IWAE_HIP_LIB=tools/_dbg/libiwae_nrtrace.so python tools/nre_trace.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

x, pi = bench.synthetic_images(512, 3)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                   use_graphs=False)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
for _ in range(3):
    m.train_step(x)
dump = m._lib.iwae_nr_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NU = 512
buf = (ctypes.c_ulonglong * (4 * NU * 3))()
n = dump(buf, 4 * NU * 3)
T = np.array(buf[:n], dtype=np.int64).reshape(4, NU, 3)
NUNITS = 39
for rec in range(2):
    t0 = T[rec, NU - 1, 0]
    e, b, d = T[rec, :NUNITS, 0], T[rec, :NUNITS, 1], T[rec, :NUNITS, 2]
    print(f"rec {rec}: total {d[-1] - t0} cyc; prologue (P1) {T[rec, NU - 1, 1] - t0}; phase A {T[rec, NU - 2, 0] - T[rec, NU - 1, 1]}; "
          f"drain + E1 {T[rec, NU - 2, 1] - T[rec, NU - 2, 0]}; phase B {d[-1] - T[rec, NU - 2, 1]}")
    wait, mma = b - e, d - b
    epi = np.append(e[1:] - d[:-1], 0)
    for u in range(NUNITS):
        print(f"  u{u:3d} wait {wait[u]:6d} mma {mma[u]:6d} epi {epi[u]:6d}")
