"""Config C4: gradient SNR over R noise draws for the 2L model at
k = 64 (IWAE, PIWAE / MIWAE with M = K = 8, CIWAE with beta = 0.5: two
independent draws per estimate, F:382-F:383), batch 20; prints draws/s and
the median SNR of the encoder and decoder parameters, and the train step's
time for the same loss (graph-replayed Philox steps, Adam included).  Under
torchrun the R draws are split over the ranks (one all-reduce of the moments)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
x, pi = bench.synthetic_images(20, 1)
for loss, kw in (("IWAE", {}), ("PIWAE", dict(k1=8, k2=8)), ("MIWAE", dict(k1=8, k2=8)), ("CIWAE", dict(beta=0.5))):
    m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function=loss, k=64, seed=2,
                       **kw)
    m.get_gradient_snr(x, R=4, seed=1)                 # warm-up (workspace, graph capture)
    torch.cuda.synchronize()
    t = time.perf_counter()
    snr, _ = m.get_gradient_snr(x, R=R, seed=7)
    el = time.perf_counter() - t
    # Keras order: per Dense (name, fan_in, fan_out) a kernel then a bias
    names = [d[0] for d in m.dense for _ in (0, 1)]
    flat = [np.asarray(s).ravel() for s in snr]
    enc = np.concatenate([f for f, nm in zip(flat, names) if nm.startswith("enc")])
    dec = np.concatenate([f for f, nm in zip(flat, names) if not nm.startswith("enc")])
    from iwae_replication_project_amd import Adam
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    xd = m._x(x)
    n0 = m._lib.iwae_debug_count(m._h, 2)
    for _ in range(10):
        m.train_step(xd, sync=False)
    engine = m._lib.iwae_debug_count(m._h, 2) > n0
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        m.train_step(xd, sync=False)
    torch.cuda.synchronize()
    st = (time.perf_counter() - t) / 200
    print(f"{loss:6s} k=64 R={R}: {R / el:8.1f} draws/s  median SNR encoder {np.median(enc[np.isfinite(enc)]):.3f}"
          f"  decoder {np.median(dec[np.isfinite(dec)]):.3f}   train step {st * 1e3:.4f} ms "
          f"({20 * 64 / st / 1e6:.2f} M image*samples/s, engine {engine})", flush=True)
