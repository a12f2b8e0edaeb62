"""Op timeline of the first workgroup of every train-engine job (tc_kernel) in
eager train steps of the bench workload.  Needs a library built with
-DIWAE_TC_TRACE (tools/build_debug.sh), run with IWAE_HIP_LIB pointing at it.
Usage: python tools/tc_trace.py [B] [k]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else bench.B_PER_GPU
K = int(sys.argv[2]) if len(sys.argv) > 2 else bench.K
x, pi = bench.synthetic_images(B * 8, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=K,
                   seed=2, use_graphs=False)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
dump = m._lib.iwae_tc_trace_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * (256 * 64))()
udump = m._lib.iwae_tc_utrace_dump
udump.restype = ctypes.c_int
udump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
ubuf = (ctypes.c_ulonglong * (256 * 8 * 16 * 3))()
for i in range(4):
    m.train_step(x[i * B:(i + 1) * B])
    n = dump(buf, 256 * 64)
    udump(ubuf, 256 * 8 * 16 * 3)
a = np.array(buf[:n], dtype=np.int64).reshape(-1, 64)
for r in a:
    t0 = int(r[1])
    ops = []
    for s in range(31):
        b, e = int(r[2 + 2 * s]), int(r[3 + 2 * s])
        if b == 0:
            break
        ops.append(f"op{s}:{(b - t0) / 100:.2f}+{(e - b) / 100:.2f}")
    print(f"job {int(r[0])}: " + "  ".join(ops))
U = np.array(ubuf[:], dtype=np.int64).reshape(256, 8, 16, 3)
nrec = a.shape[0]
for rec in range(nrec):
    t0 = int(a[rec, 1])
    for op in range(8):
        us = [(u, U[rec, op, u]) for u in range(16) if U[rec, op, u, 0] > 0]
        if not us:
            continue
        print(f"  rec{rec} job{int(a[rec, 0])} op{op}: " + " ".join(
            f"u{u}[{(v[0] - t0) / 100:.2f} mma+{(v[1] - v[0]) / 100:.2f} epi+{(v[2] - v[1]) / 100:.2f}]" for u, v in us))
# per op: kind read (descriptor loads), after the LDS padding, dense-op entry (wave 0)
pdump = getattr(m._lib, "iwae_tc_ptrace_dump", None)
if pdump is not None:
    pdump.restype = ctypes.c_int
    pdump.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    pbuf = (ctypes.c_ulonglong * (256 * 32 * 4))()
    pdump(pbuf, 256 * 32 * 4)
    P = np.array(pbuf[:], dtype=np.int64).reshape(256, 32, 4)
    for rec in range(nrec):
        t0 = int(a[rec, 1])
        parts = []
        for s in range(31):
            b = int(a[rec, 2 + 2 * s])
            if b == 0:
                break
            k, pd, de = (int(v) for v in P[rec, s, :3])
            f = lambda v: f"{(v - b) / 100:.2f}" if v > 0 else "-"
            parts.append(f"op{s}[kind+{f(k)} pad+{f(pd)} dense+{f(de)}]")
        print(f"  prologue rec{rec} job{int(a[rec, 0])}: " + " ".join(parts))
