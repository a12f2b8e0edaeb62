"""One configs[1] train step through the library's data-parallel path (RCCL
communicator owned by the handle, world size 1 on one GPU) for a rocprofv3
kernel trace: shows where the gradient all-reduce sits in the captured step
(two buckets: the output MLP bucket all-reduced on a side stream beside the
other layers' gradient pass, then one Adam + FX / GX launch).
    rocprofv3 --kernel-trace -d gpurun_out/dp -o run -- python tools/dp_timeline.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model, distributed  # noqa: E402

x, pi = bench.synthetic_images(bench.B_PER_GPU * 8, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K,
                   seed=2)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
d = distributed.enable_data_parallel(m, comm="library")
assert d.comm == "library"
X = m._x(x)
for i in range(30):
    m.train_step(X[(i % 8) * bench.B_PER_GPU:(i % 8 + 1) * bench.B_PER_GPU], sync=False)
m._stream.synchronize()
print("dp steps done, loss", float(m._loss_buf.item()))
