"""NLL throughput vs chunk size (tuning knob nll_rows) on the bench model (2L, k=5000)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Flexible_Model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
x, pi = bench.synthetic_images(n, 99)
for prec in ("bf16x3", "f32"):
    m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                       precision=prec)
    xd = m._x(x)
    for rows in (1 << 20, 1 << 18, 1 << 17, 1 << 16, 1 << 15):
        m.set_tuning("nll_rows", rows)
        m.log_px(xd[:64], 5000)
        torch.cuda.synchronize()
        t = time.perf_counter()
        lp = m.log_px(xd, 5000)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        print(f"{prec:7s} rows/chunk {rows:8d}: {n / el:9.1f} images/s  nll {-lp.mean().item():.4f}", flush=True)
