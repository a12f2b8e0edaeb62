"""Host-side cost of one Flexible_Model.train_steps call (the bench's timed
call, 20 steps of B=20 from prepared graphs) and of its pieces, in us:
python tools/host_overhead.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model, _lib  # noqa: E402

B, n = bench.B_PER_GPU, 20
x, pi = bench.synthetic_images(n * B * 4, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K, seed=2)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
xs = xd[:n * B]
m.prepare_train_steps(xs, B)
m.train_steps(xs, B, sync=False)
torch.cuda.synchronize()


def timeit(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    el = (time.perf_counter() - t) / reps * 1e6
    torch.cuda.synchronize()
    return el


lc = m._lc()
losses = torch.empty(n, device=m.device)
res = {
    "stream ctx enter/exit": timeit(lambda: torch.cuda.stream(m._stream).__enter__() or None, 2000),
    "_x(device tensor)": timeit(lambda: m._x(xs), 2000),
    "torch.empty under stream": timeit(lambda: [torch.empty(n, device=m.device) for _ in [0] if torch.cuda.stream(m._stream)], 2000),
    "_lc()": timeit(lambda: m._lc(), 2000),
    "iwae_train_steps ctypes call only (enqueue)": timeit(lambda: m._lib.iwae_train_steps(m._h, lc, _lib.fptr(xs), B, n, _lib.fptr(losses)), 50),
    "train_steps(sync=False) (enqueue)": timeit(lambda: m.train_steps(xs, B, sync=False), 50),
}
t = time.perf_counter()
for _ in range(20):
    m.train_steps(xs, B, sync=False)
    m._stream.synchronize()
res["train_steps + stream sync, per call"] = (time.perf_counter() - t) / 20 * 1e6
for k, v in res.items():
    print(f"{k:50s} {v:9.2f} us", flush=True)
