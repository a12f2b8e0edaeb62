"""GPU parity of the evaluation-statistics suite (SURVEY.md s8(f) rank 1,
F:249-F:300, F:466-F:526): reconstruction probabilities and loss, encoder
means / unit activity / PCA eigenvalues / active units, and the NLL with
inactive units zeroed -- the HIP path through the C ABI against the float64
oracle on identical injected noise and weights.  Parity unpinned (no TF here):
the oracle restates the reference's lines, cited per function."""
import numpy as np
import pytest

from test_gpu_parity import REL, make_model, weights_from_flat

pytestmark = pytest.mark.gpu

ARCHS = [([64], [64], [16], [784]), ([64, 32], [32, 64], [32, 16], [32, 784]),
         ([48, 32, 24], [24, 32, 48], [20, 12, 8], [12, 20, 784])]


def _setup(arch, seed, B):
    from oracle import iwae_oracle as O
    he, hd, le, ld = arch
    rng = np.random.default_rng(seed)
    mean = rng.uniform(0.02, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    m = make_model(he, hd, le, ld, loss="IWAE", k=5)
    m.set_weights(weights_from_flat(m, O.flatten_params(spec, params)))
    x = (rng.random((B, 784)) < mean).astype(np.float32)
    return O, spec, params, m, x, rng


def _eps(rng, shape):
    return rng.standard_normal(shape).astype(np.float32)


@pytest.mark.parametrize("arch", ARCHS)
def test_reconstruction_matches_oracle(arch):
    """reconstructed_x_probs / get_reconstruction_loss with injected encoder and
    prior draws (generate_x re-samples h_{L-1}..h_1 from the prior)."""
    O, spec, params, m, x, rng = _setup(arch, 5, 9)
    L = spec.L
    le = spec.n_latent_encoder
    B = x.shape[0]
    e_enc = [_eps(rng, (1, B, d)) for d in le]
    e_pri = [_eps(rng, (1, B, le[L - 2 - j])) for j in range(L - 1)]
    eps = e_enc + e_pri
    probs = m.reconstructed_x_probs(x, eps=eps).cpu().numpy()
    loss = m.get_reconstruction_loss(x, eps=eps)
    rp, rl = O.reconstruct(params, spec, x.astype(np.float64), [e.astype(np.float64) for e in e_enc],
                           [e.astype(np.float64) for e in e_pri])
    assert probs.shape == (1, B, 784)
    np.testing.assert_allclose(probs, rp, rtol=2e-4, atol=2e-6)
    assert abs(loss - rl) <= REL * abs(rl), (loss, rl)


def test_reconstruction_philox_is_reproducible_and_fresh_per_call():
    O, spec, params, m, x, rng = _setup(ARCHS[1], 6, 8)
    m.set_seed(123)
    a = m.reconstructed_x_probs(x).cpu().numpy()
    b = m.reconstructed_x_probs(x).cpu().numpy()
    m.set_seed(123)
    c = m.reconstructed_x_probs(x).cpu().numpy()
    np.testing.assert_array_equal(a, c)
    assert np.abs(a - b).max() > 1e-4
    assert np.isfinite(m.get_reconstruction_loss(x)) and m.get_reconstruction_loss(x) > 0


@pytest.mark.parametrize("arch", ARCHS)
def test_unit_activity_matches_oracle(arch):
    """Encoder means over n draws, their batch variances, PCA eigenvalues and
    the active-unit decision (F:264-F:300)."""
    O, spec, params, m, x, rng = _setup(arch, 7, 24)
    n = 40
    B = x.shape[0]
    eps = [_eps(rng, (n, B, d)) for d in spec.n_latent_encoder]
    means = [t.cpu().numpy() for t in m.encoder_means(x, n, eps=eps)]
    ref = O.encoder_means(params, spec, x.astype(np.float64), [e.astype(np.float64) for e in eps])
    for a, r in zip(means, ref):
        np.testing.assert_allclose(a, r, rtol=1e-4, atol=2e-5)
    var, eig = m.get_levels_of_units_activity(x, n, eps=eps)
    rvar, reig = O.levels_of_units_activity(ref)
    for a, r in zip(var, rvar):
        np.testing.assert_allclose(a, r, rtol=1e-3, atol=1e-6)
    for a, r in zip(eig, reig):
        np.testing.assert_allclose(a, r, rtol=1e-3, atol=1e-6)
    thr = float(np.median(np.concatenate(rvar)))       # a threshold that splits the units
    au, nau, npca = m.get_active_units(var, eig, thr)
    rau, rnau, rnpca = O.active_units(rvar, reig, thr)
    for a, r, v in zip(au, rau, rvar):
        sure = np.abs(v - thr) > 1e-3 * thr
        assert np.array_equal(np.asarray(a)[sure], np.asarray(r)[sure])


def test_encoder_means_philox_chunks_match_single_pass_statistics():
    """Philox means over many images (several 2^20-row chunks) agree with the
    analytic mean of q(h_1|x) for a 1-layer model: E[h_1] = mu(x)."""
    import torch
    O, spec, params, m, x, rng = _setup(ARCHS[0], 8, 4)
    N, n = 300, 4000                                    # 1.2 M rows -> 2 chunks
    xs = np.repeat(x, N // 4, axis=0)
    means = m.encoder_means(xs, n)[0].cpu().numpy()
    q0 = O._stoch_forward(params, "enc0", x.astype(np.float64))
    mu, sc = q0["mu"], q0["scale"]
    ref = np.repeat(mu, N // 4, axis=0)
    tol = 6 * np.repeat(sc, N // 4, axis=0) / np.sqrt(n)
    assert np.all(np.abs(means - ref) <= tol + 1e-5)
    torch.cuda.synchronize()


@pytest.mark.parametrize("arch", ARCHS)
def test_nll_without_inactive_units_matches_oracle(arch):
    """iwae_nll_masked with injected noise against the oracle's masked forward
    (F:466-F:494: log q at the masked sample, later layers and the decoder read
    it)."""
    O, spec, params, m, x, rng = _setup(arch, 9, 6)
    k = 40
    B = x.shape[0]
    masks = [(rng.random(d) < 0.6).astype(np.float32) for d in spec.n_latent_encoder]
    for mk in masks:
        mk[0] = 1.0
    eps = [_eps(rng, (k, B, d)) for d in spec.n_latent_encoder]
    lp = m.log_px_masked(x, masks, k, eps=eps).cpu().numpy()
    ref = O.log_px_per_image(params, spec, x.astype(np.float64), k, eps=[e.astype(np.float64) for e in eps],
                             masks=[mk.astype(np.float64) for mk in masks])
    np.testing.assert_allclose(lp, ref, rtol=REL, atol=1e-3)


def test_masked_nll_with_all_units_active_equals_plain_nll():
    """All-ones masks: the masked (layer-wise) path draws the same Philox stream
    as the fused NLL path, so both estimates agree to rounding."""
    O, spec, params, m, x, rng = _setup(ARCHS[1], 10, 5)
    ones = [np.ones(d, np.float32) for d in spec.n_latent_encoder]
    m.set_seed(77)
    a = m.log_px(x, 500).cpu().numpy()
    m.set_seed(77)
    b = m.log_px_masked(x, ones, 500).cpu().numpy()
    np.testing.assert_allclose(a, b, rtol=2 * REL, atol=2e-3)


def test_training_statistics_has_the_reference_keys():
    O, spec, params, m, x, rng = _setup(ARCHS[1], 11, 20)
    res, res2 = m.get_training_statistics(x, 5, batch_size=10)
    for key in ["VAE", "IWAE", "NLL", "E_q(h|x)[log(p(x|h))]", "D_kl(q(h|x),p(h))", "D_kl(q(h|x),p(h|x))",
                "reconstruction_loss", "LL_pruned"]:
        assert key in res and np.isfinite(res[key]), key
    assert res["reconstruction_loss"] > 0 and res["LL_pruned"] > 0
    assert [len(a) for a in res2["active_units"]] == list(spec.n_latent_encoder)
    assert res2["number_of_active_units"] == [sum(a) for a in res2["active_units"]]
    assert len(res2["number_of_PCA_active_units"]) == spec.L and len(res2["variances"]) == spec.L


def test_batched_training_statistics_keep_the_per_batch_reductions(monkeypatch):
    """The batched statistics (many batches per call, every k=5000 NLL over
    all images in one launch series) equal the reference loop's mean of batch
    means: with each per-call statistic replaced by a deterministic function
    of its images (the mean pixel), both paths give the same numbers; on the
    real model both give finite estimates within the NLL's sampling noise."""
    O, spec, params, m, x, rng = _setup(ARCHS[1], 12, 40)

    def fake(b, *a, **kw):
        return float(m._x(b).double().mean().item())
    for name in ("get_L", "get_L_k", "get_NLL", "get_E_qhIx_log_pxIh", "get_reconstruction_loss"):
        monkeypatch.setattr(m, name, fake)
    monkeypatch.setattr(m, "get_NLL_without_inactive_units", lambda b, *a, **kw: 1.0)
    ra, _ = m.get_training_statistics(x, 5, batch_size=10, batched=False)
    rb, _ = m.get_training_statistics(x, 5, batch_size=10, batched=True, chunk_images=20)
    for key in ra:
        assert abs(ra[key] - rb[key]) <= 1e-9 * max(1.0, abs(ra[key])), (key, ra[key], rb[key])
    monkeypatch.undo()
    r1, _ = m.get_training_statistics(x, 5, batch_size=10, batched=False)
    r2, _ = m.get_training_statistics(x, 5, batch_size=10, batched=True)
    assert abs(r1["NLL"] - r2["NLL"]) < 0.5, (r1["NLL"], r2["NLL"])
    for key in r2:
        assert np.isfinite(r2[key]), key
