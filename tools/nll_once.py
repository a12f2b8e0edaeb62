"""One k=5000 NLL evaluation over N synthetic images (bench model) -- a short
target for rocprofv3 passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
x, pi = bench.synthetic_images(n, 99)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                   precision=prec)
lp = m.log_px(m._x(x), 5000)
torch.cuda.synchronize()
print(f"nll {-lp.mean().item():.4f} over {n} images ({prec})")
