"""Run-to-run determinism of the train step: the same model, data and noise
trained for a few steps R times per tuning configuration (a fresh model each
time); prints how many runs differ from the first and, for each, the first
step where it does and which outputs differ there (the loss, each parameter
tensor's gradient, its updated value).  Every path is meant to be bitwise
reproducible, so a difference names a race (or a read of memory nothing
wrote).
    python tools/determinism_stress.py [B] [repeats] [steps] [knob=v,knob=v ...]
NLL=1: instead, the k=5000 NLL of B images (device Philox) per fresh model.
LOSS=<name> [K=<k>]: another loss function (default IWAE, k=50)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from iwae_replication_project_amd import Adam, Flexible_Model

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
S = int(sys.argv[3]) if len(sys.argv) > 3 else 3
CONFIGS = [{}]
if len(sys.argv) > 4:
    CONFIGS = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in c.split(",") if kv) for c in sys.argv[4:]]

KEEP = os.environ.get("KEEP") == "1"        # keep every model alive (no reuse of freed device memory)
SETTLE = os.environ.get("SETTLE") == "1"    # device synchronize + 50 ms before the first step
kept = []
rng = np.random.default_rng(7)
xs = (rng.random((S * B, 784)) < 0.3).astype(np.float32)


def run_nll(cfg):
    m = Flexible_Model([200, 100], [100, 200], [100, 50], [100, 784], dataset_bias=None, loss_function="IWAE", k=50,
                       seed=3, use_graphs=True, tuning=cfg)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    X = torch.from_numpy(xs[:B]).to(m.device)
    m.set_seed(5)
    v = np.float32(m.get_NLL(X, k=5000))
    del m
    return [(v, [], [])], [0, 0, 0]


LOSS = os.environ.get("LOSS", "IWAE")
KS = int(os.environ.get("K", "50"))
LOSS_KW = {"CIWAE": {"beta": 0.5}, "L_alpha": {"alpha": 0.5}, "L_power_p": {"p": 2.0},
           "MIWAE": {"k1": 8, "k2": 8}, "PIWAE": {"k1": 8, "k2": 8}}.get(LOSS, {})


def run(cfg):
    if os.environ.get("NLL") == "1":
        return run_nll(cfg)
    m = Flexible_Model([200, 100], [100, 200], [100, 50], [100, 784], dataset_bias=None, loss_function=LOSS, k=KS,
                       seed=3, use_graphs=True, tuning=cfg, **LOSS_KW)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    X = torch.from_numpy(xs).to(m.device)
    if SETTLE:
        import time
        torch.cuda.synchronize()
        time.sleep(0.05)
    steps = []
    for i in range(S):
        loss = np.float32(m.train_step(X[i * B:(i + 1) * B])[LOSS])
        g = [np.asarray(t, np.float32).copy() for t in m.get_gradients()]
        w = [np.asarray(t, np.float32).copy() for t in m.get_weights()]
        steps.append((loss, g, w))
    dbg = [int(m._lib.iwae_debug_count(m._h, i)) for i in (2, 8, 9)]
    if KEEP:
        kept.append(m)
    del m
    return steps, dbg


def compare(a, b):
    """First step where runs a and b differ and what differs there."""
    for s, ((la, ga, wa), (lb, gb, wb)) in enumerate(zip(a, b)):
        d = []
        if la != lb:
            d.append(f"loss {la!r}/{lb!r}")
        for kind, xa, xb in (("grad", ga, gb), ("weight", wa, wb)):
            for i, (u, v) in enumerate(zip(xa, xb)):
                ne = (u != v) & ~(np.isnan(u) & np.isnan(v))
                if ne.any():
                    idx = np.argwhere(ne)
                    d.append(f"{kind}[{i}]{u.shape}: {int(ne.sum())} elems max|d| {float(np.nanmax(np.abs(u - v))):.3g}"
                             f" first {idx[0].tolist()} last {idx[-1].tolist()}")
        if d:
            return s, d
    return None, []


for cfg in CONFIGS:
    base = None
    ndiff = 0
    nonfinite = 0
    for r in range(R):
        steps, dbg = run(cfg)
        if not all(np.isfinite(l) for l, _, _ in steps):
            nonfinite += 1
        if base is None:
            base = steps
            continue
        s, d = compare(base, steps)
        if s is not None:
            ndiff += 1
            print(f"  {cfg} run {r}: first differs at step {s}: " + "; ".join(d), flush=True)
    print(f"{cfg}: {ndiff} of {R - 1} runs differ from the first, non-finite {nonfinite}  (last run: tc {dbg[0]}, "
          f"spin give-ups {dbg[1]}, tcu {dbg[2]})", flush=True)
