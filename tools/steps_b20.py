"""The bench's headline workload alone (configs[1]: 2L, k=50, B=20, IWAE),
fit's loop through train_steps with graphs, for kernel traces of replayed
steps (tools/prof_step.sh).  Usage: python tools/steps_b20.py [steps] [knob=value ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
# further arguments: library knobs, knob=value (include/iwae.h enum iwae_knob)
tuning = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}
x, pi = bench.synthetic_images(n * bench.B_PER_GPU, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K, seed=2,
                   tuning=tuning or None)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
m.train_steps(xd, bench.B_PER_GPU, sync=False)
m.train_steps(xd, bench.B_PER_GPU, sync=False)
torch.cuda.synchronize()
print("steps done", flush=True)
