"""Host-side cost of a replayed train step: the same graph replayed with one
batch (the captured x) against cycling batches (the input-layer launch is
re-pointed with hipGraphExecKernelNodeSetParams every call)."""
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
                   seed=2, use_graphs=True)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xs = [m._x((rng.random((20, 784)) < pi).astype(np.float32)) for _ in range(16)]
for i in range(30):
    m.train_step(xs[i % 16], sync=False)
torch.cuda.synchronize()
for mode in ("cycle", "one", "cycle", "one"):
    n = 400
    m._stream.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        m.train_step(xs[i % 16] if mode == "cycle" else xs[0], sync=False)
    t1 = time.perf_counter()
    m._stream.synchronize()
    t2 = time.perf_counter()
    print(f"{mode:6s} {1e6 * (t2 - t0) / n:8.2f} us/step  (host issue {1e6 * (t1 - t0) / n:7.2f} us/step)", flush=True)
