"""k=5000 NLL images/s of the bench model right after some train steps (the
bench's order), timed twice -- to separate one-time costs from throughput."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
x, pi = bench.synthetic_images(max(n, 400), 99)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
for i in range(20):
    m.train_step(xd[(i % 20) * 20:(i % 20 + 1) * 20], sync=False)
torch.cuda.synchronize()
m.log_px(xd[:64], 5000)
torch.cuda.synchronize()
for rep in range(3):
    t = time.perf_counter()
    lp = m.log_px(xd[:n], 5000)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(f"rep {rep}: {n / el:9.1f} images/s ({el:.3f} s)", flush=True)
