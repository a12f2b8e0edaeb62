"""Replay one train step from the same state (weights, Adam moments, noise
position, batch) R times and report which outputs differ between replays:
the loss, each parameter tensor's gradient and its updated value.  Every
kernel on the path is meant to be bitwise reproducible, so a tensor that
differs names the launch with a race (its producer).
    python tools/replay_determinism.py [B] [replays] [knob=value ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from iwae_replication_project_amd import Adam, Flexible_Model

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
R = int(sys.argv[2]) if len(sys.argv) > 2 else 200
tuning = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[3:])
rng = np.random.default_rng(7)
xs = (rng.random((3 * B, 784)) < 0.3).astype(np.float32)
m = Flexible_Model([200, 100], [100, 200], [100, 50], [100, 784], dataset_bias=None, loss_function="IWAE", k=50,
                   seed=3, use_graphs=True, tuning=tuning)
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
X = torch.from_numpy(xs).to(m.device)
for i in range(2):
    m.train_step(X[i * B:(i + 1) * B])
w0 = m.get_weights()
m0, v0, st0 = m.get_optimizer_state()
Xs = X[2 * B:3 * B]
shapes = [tuple(np.shape(w)) for w in w0]
ref = None
ndiff = 0
bad = {}
for r in range(R):
    m.set_weights(w0)
    m.set_optimizer_state(m0, v0, st0)
    m.set_seed(11)
    loss = np.float32(m.train_step(Xs)["IWAE"])
    g = [np.asarray(t, np.float32) for t in m.get_gradients()]
    w = [np.asarray(t, np.float32) for t in m.get_weights()]
    mm, vv, _ = m.get_optimizer_state()
    if ref is None:
        ref = (loss, g, w, np.asarray(mm), np.asarray(vv))
        continue
    diffs = []
    if loss != ref[0]:
        diffs.append(f"loss {ref[0]!r}->{loss!r}")
    for kind, cur, base in (("grad", g, ref[1]), ("weight", w, ref[2])):
        for i, (a, b) in enumerate(zip(cur, base)):
            d = a != b
            if d.any():
                idx = np.argwhere(d)
                key = (kind, i)
                bad.setdefault(key, []).append(int(d.sum()))
                diffs.append(f"{kind}[{i}]{shapes[i]}: {int(d.sum())} elems, max |d| {float(np.abs(a - b).max()):.3g},"
                             f" first {idx[0].tolist()} last {idx[-1].tolist()}")
    if not np.array_equal(np.asarray(mm), ref[3]) or not np.array_equal(np.asarray(vv), ref[4]):
        diffs.append("adam state")
    if diffs:
        ndiff += 1
        if ndiff <= 12:
            print(f"replay {r}: " + "; ".join(diffs), flush=True)
print(f"B={B} tuning={tuning}: {ndiff} of {R - 1} replays differ from the first", flush=True)
for (kind, i), v in sorted(bad.items()):
    print(f"  {kind}[{i}] {shapes[i]}: differs in {len(v)} replays, elems {min(v)}..{max(v)}", flush=True)
