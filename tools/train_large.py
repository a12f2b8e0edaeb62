"""Train-step throughput of the 2L model (k=50) at a large per-GPU batch --
config C5's per-rank share (global B=4096 over 8 GPUs = 512 per GPU)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
path = sys.argv[3] if len(sys.argv) > 3 else "auto"
tuning = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[4:]}     # knob=value ... (A/B runs)
x, pi = bench.synthetic_images(4 * B, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                   kernel_path=path, tuning=tuning)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
if os.environ.get("LOOP", "steps") == "calls":      # one train_step call (graph launch) per step
    for i in range(3):
        m.train_step(xd[(i % 4) * B:(i % 4 + 1) * B], sync=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(steps):
        m.train_step(xd[(i % 4) * B:(i % 4 + 1) * B], sync=False)
else:                                               # fit's loop: train_steps over the steps' batches
    xs = xd.repeat((steps + 3) // 4, 1)[:steps * B].contiguous()
    m.train_steps(xs, B, sync=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    m.train_steps(xs, B, sync=False)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / steps
rows = B * 50
print(f"B={B} k=50 path={path}: {el * 1e3:.3f} ms/step, {rows / el / 1e6:.3f} M image*samples/s, "
      f"{1712944 * rows / el / 1e12:.1f} TFLOP/s, loss {float(m._loss_buf.item()):.3f}", flush=True)
