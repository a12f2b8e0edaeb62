"""k=5000 NLL images/s of the bench model over N synthetic images (one warm-up
call first); library chosen by IWAE_HIP_LIB like every tool."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
tag = sys.argv[2] if len(sys.argv) > 2 else ""
x, pi = bench.synthetic_images(n, 99)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2)
xd = m._x(x)
m.log_px(xd[:64], 5000)
torch.cuda.synchronize()
t = time.perf_counter()
lp = m.log_px(xd, 5000)
torch.cuda.synchronize()
el = time.perf_counter() - t
print(f"{tag} {n / el:9.1f} images/s  nll {-lp.mean().item():.4f}", flush=True)
