"""Fixed cost of one train_steps call (fit's loop, iwae_train_steps) at B=20:
for n steps, the host time until the call returns and the time until its
stream drained, graphs captured beforehand (iwae_train_steps_prepare).  The
intercept of wall time over n is the per-call latency that a short timed
region (the driver's --steps 20) pays once.
    python tools/steps_call_overhead.py [steps_first]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from iwae_replication_project_amd import Adam, Flexible_Model

rng = np.random.default_rng(0)
pi = rng.uniform(0.02, 0.4, 784)
m = Flexible_Model([200, 100], [100, 200], [100, 50], [100, 784], dataset_bias=pi, loss_function="IWAE", k=50,
                   seed=2, use_graphs=True,
                   tuning={"steps_first": int(sys.argv[1])} if len(sys.argv) > 1 else {})
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
X = m._x((rng.random((64 * 20, 784)) < pi).astype(np.float32))
ns = [1, 2, 4, 8, 16, 20, 32, 64]
for n in ns:
    m.prepare_train_steps(X[:n * 20], 20)
    m.train_steps(X[:n * 20], 20, sync=False)
torch.cuda.synchronize()
res = {}
for rep in range(5):
    for n in ns:
        m._stream.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.train_steps(X[:n * 20], 20, sync=False)
        t1 = time.perf_counter()
        m._stream.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res.setdefault(n, []).append((t1 - t0, t2 - t0))
for n in ns:
    h = min(r[0] for r in res[n]) * 1e6
    w = min(r[1] for r in res[n]) * 1e6
    print(f"n={n:3d}  host {h:8.1f} us  wall {w:9.1f} us  per step {w / n:7.2f} us", flush=True)
a = np.array([[n, 1.0] for n in ns])
b = np.array([min(r[1] for r in res[n]) * 1e6 for n in ns])
slope, icpt = np.linalg.lstsq(a, b, rcond=None)[0]
print(f"fit: wall = {slope:.2f} us * n + {icpt:.1f} us")
