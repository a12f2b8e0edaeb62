"""A few train_steps calls (B=20, 20 steps, graphs prepared) for a
rocprofv3 --kernel-trace --hip-trace run: where the per-call fixed cost goes
(host API calls against the kernels they feed).
    rocprofv3 --kernel-trace --hip-trace --output-format csv -d <dir> -o run -- python tools/steps_call_trace.py"""
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
X = m._x((rng.random((20 * 20, 784)) < pi).astype(np.float32))
m.prepare_train_steps(X, 20)
m.train_steps(X, 20, sync=False)
torch.cuda.synchronize()
for rep in range(4):
    time.sleep(0.01)
    t0 = time.perf_counter()
    m.train_steps(X, 20, sync=False)
    t1 = time.perf_counter()
    m._stream.synchronize()
    t2 = time.perf_counter()
    print(f"call {rep}: host {1e6 * (t1 - t0):.1f} us, wall {1e6 * (t2 - t0):.1f} us", flush=True)
