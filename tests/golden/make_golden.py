"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (TF 2.4 + TFP + tfds) cannot run in this container, and it holds
no tests or fixtures of its own, so these vectors are produced by the oracle's
float64 restatement (parity unpinned -- see oracle/iwae_oracle.py).  They pin
the oracle against regressions and give the GPU parity tests fixed cases.

Inputs are float32-representable (weights, x, eps rounded to float32 first) so
the float32 HIP path and the float64 oracle start from identical values.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import iwae_oracle as O  # noqa: E402

CASES = {
    # name: (he, hd, le, ld, x_dim, B, k, k1, k2)
    "g1L": ([32], [32], [8], [64], 64, 4, 6, 3, 2),
    "g2L": ([32, 16], [16, 32], [16, 8], [16, 64], 64, 3, 6, 2, 3),
    "g2L784": ([48, 24], [24, 48], [20, 10], [20, 784], 784, 5, 8, 4, 2),
}
LOSS_KW = {
    "VAE": {}, "IWAE": {}, "L_power_p": dict(p=2.5), "L_median": {}, "L_alpha": dict(alpha=0.3),
    "VAE_V1": {}, "CIWAE": dict(beta=0.3), "MIWAE": {}, "PIWAE": {},
}


FULL_GRADS_784 = ("IWAE", "VAE", "CIWAE", "PIWAE")   # keep the 784-wide fixture small


def f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def make(name, he, hd, le, ld, x_dim, B, k, k1, k2, seed):
    rng = np.random.default_rng(seed)
    spec = O.ModelSpec(he, hd, le, ld, x_dim=x_dim)
    mean = rng.uniform(0.05, 0.5, x_dim)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [f32(w), f32(b)] for n, (w, b) in params.items()}
    x = (rng.random((B, x_dim)) < mean).astype(np.float64)
    eps = [f32(e) for e in O.draw_eps(spec, k, B, rng)]
    eps2 = [f32(e) for e in O.draw_eps(spec, k, B, rng)]
    out = dict(he=np.array(he), hd=np.array(hd), le=np.array(le), ld=np.array(ld),
               x_dim=np.int64(x_dim), B=np.int64(B), k=np.int64(k), k1=np.int64(k1), k2=np.int64(k2),
               params=O.flatten_params(spec, params).astype(np.float32), x=x.astype(np.float32))
    for i, e in enumerate(eps):
        out[f"eps{i}"] = e.astype(np.float32)
    for i, e in enumerate(eps2):
        out[f"eps2_{i}"] = e.astype(np.float32)
    c = O.forward(params, spec, x, eps, need_bce=True)
    out["lw"] = c["lw"]
    out["bce_mean"] = np.float64(np.mean(c["bce_row"]))
    for loss, kw in LOSS_KW.items():
        kw = dict(kw)
        if loss in ("MIWAE", "PIWAE"):
            kw.update(k1=k1, k2=k2)
        if loss == "CIWAE":
            kw["eps2"] = eps2
        J, g = O.objective_and_grads(params, spec, x, eps, loss, k, **kw)
        out[f"{loss}.J"] = np.float64(J)
        if x_dim <= 64 or loss in FULL_GRADS_784:
            out[f"{loss}.grad_loss"] = (-O.flatten_params(spec, g)).astype(np.float32)
    out["logpx"] = O.log_px_per_image(params, spec, x, k, eps=eps)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {kk: float(v) for kk, v in out.items() if kk.endswith(".J")})


if __name__ == "__main__":
    for i, (name, case) in enumerate(CASES.items()):
        make(name, *case, seed=100 + i)
