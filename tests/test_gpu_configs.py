"""The BASELINE.json configurations at their own sizes, each against the
float64 oracle on identical injected noise and weights (north_star: losses
and gradients within 1e-4 relative):

* configs[0]: 1 stochastic layer 784-200-200-50, k=5, batch 20 -- every loss
  of the train_step dispatch (F:228-F:241) plus MIWAE/PIWAE;
* configs[3]: 2 layers, k=64 = M*K with M=K=8, beta=0.5 -- MIWAE, CIWAE
  (two independent draws, F:382-F:383) and PIWAE (PDF p7);
* configs[4]: the per-GPU share of the large-batch data-parallel step, B=512,
  k=50 (25,600 sample rows; the output layer's GEMMs take bf16x3 products
  there), loss, gradients and post-Adam weights.

The configs[2] k=5000 NLL on that architecture is in test_gpu_edges.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-4
ADAM_ATOL = 6e-5     # test_gpu_parity.py: Adam's first step amplifies near-zero gradient errors by lr/eps
ARCH1 = ([200], [200], [50], [784])
ARCH2 = ([200, 100], [100, 200], [100, 50], [100, 784])


def _flat(ws):
    return np.concatenate([np.asarray(w, np.float64).ravel() for w in ws])


def _rel_l2(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-30))


def _case(arch, B, k, seed, n_draws=1):
    from oracle import iwae_oracle as O
    he, hd, le, ld = arch
    rng = np.random.default_rng(seed)
    mean = rng.uniform(0.01, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    x = (rng.random((B, 784)) < mean).astype(np.float64)
    draws = [[e.astype(np.float32).astype(np.float64) for e in O.draw_eps(spec, k, B, rng)] for _ in range(n_draws)]
    return O, spec, params, mean, x, draws


def _run(arch, loss, B, k, seed, engine_launches=None, **kw):
    """One train step on the GPU and in the oracle; returns the comparisons
    (engine_launches: a list that receives the step's train-engine launches)."""
    from iwae_replication_project_amd import Adam, Flexible_Model
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    n_draws = 2 if loss == "CIWAE" else 1
    O, spec, params, mean, x, draws = _case(arch, B, k, seed, n_draws)
    he, hd, le, ld = arch
    m = Flexible_Model(he, hd, le, ld, dataset_bias=mean, loss_function=loss, k=k, seed=1, **kw)
    m.set_weights(_split(O.flatten_params(spec, params).astype(np.float32), weight_shapes(m.dense)))
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    eps_gpu = [e.astype(np.float32) for d in draws for e in d]
    n0 = m._lib.iwae_debug_count(m._h, 2)
    loss_gpu = m.train_step(x.astype(np.float32), eps=eps_gpu)[loss]
    if engine_launches is not None:
        engine_launches.append(m._lib.iwae_debug_count(m._h, 2) - n0)
    okw = {n: kw[n] for n in ("p", "alpha", "beta", "k1", "k2") if n in kw}
    if loss == "CIWAE":
        okw["eps2"] = draws[1]
    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    ref_loss, ref_new, ref_g = O.train_step(params, spec, x, draws[0], loss, k, opt, **okw)
    g = _flat(m.get_gradients())
    w0 = O.flatten_params(spec, params)
    return loss_gpu, ref_loss, g, ref_g, _flat(m.get_weights()), O.flatten_params(spec, ref_new), \
        O.Adam(1e-3, 0.9, 0.999, 1e-4).apply(w0, g)


def _check(res):
    loss, ref_loss, g, ref_g, w, ref_w, w_from_g = res
    assert abs(loss - ref_loss) <= REL * abs(ref_loss), (loss, ref_loss)
    assert _rel_l2(g, ref_g) <= REL, _rel_l2(g, ref_g)
    # Adam on the device == Adam applied to the device gradient; against the oracle's
    # weights within 10x the gradient error (lr/eps = 10 amplification at step 1)
    np.testing.assert_allclose(w, w_from_g, atol=2e-6)
    np.testing.assert_allclose(w, ref_w, atol=max(ADAM_ATOL, 10 * np.abs(g - ref_g).max()))


C0_LOSSES = [("VAE", {}), ("IWAE", {}), ("VAE_V1", {}), ("L_alpha", dict(alpha=0.5)),
             ("L_power_p", dict(p=2.0)), ("L_median", {}), ("CIWAE", dict(beta=0.5)),
             ("MIWAE", dict(k1=5, k2=1)), ("PIWAE", dict(k1=5, k2=1))]


@pytest.mark.parametrize("loss,kw", C0_LOSSES, ids=[c[0] for c in C0_LOSSES])
def test_configs0_1L_full_width_k5_b20_every_loss(loss, kw):
    """BASELINE configs[0] (experiment_example.py's IWAE k=5, 784-200-200-50,
    batch 20) for every loss of the train_step dispatch."""
    _check(_run(ARCH1, loss, 20, 5, 300 + len(loss), **kw))


@pytest.mark.parametrize("loss", ["MIWAE", "CIWAE", "PIWAE"])
def test_configs3_k64_m8_k8_beta05(loss):
    """BASELINE configs[3]: 2L, k=64 with M=K=8 (MIWAE / PIWAE), beta=0.5 (CIWAE)."""
    kw = dict(k1=8, k2=8) if loss in ("MIWAE", "PIWAE") else dict(beta=0.5)
    n = []
    _check(_run(ARCH2, loss, 20, 64, 400 + len(loss), engine_launches=n, **kw))
    # on the train engine (forward, backward and the image-row jobs; PIWAE: one
    # unit-weight backward chain serves both weightings, knob piwae_one)
    assert n[0] >= 3, n


def test_configs4_per_gpu_share_b512_k50():
    """BASELINE configs[4]'s per-GPU share (4096 images over 8 GPUs): B=512,
    k=50, 25,600 sample rows -- the bench's large_batch leg."""
    _check(_run(ARCH2, "IWAE", 512, 50, 512))
