"""CPU tests of the oracle (test infrastructure): golden fixtures, finite
differences, an independent torch.distributions + autograd restatement, the
known-answer identities implied by the reference's definitions, closed-form
densities and the Adam kernel form."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import iwae_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def tiny(seed=0, L=2, x_dim=16):
    rng = np.random.default_rng(seed)
    if L == 1:
        spec = O.ModelSpec([12], [12], [6], [x_dim], x_dim=x_dim)
    else:
        spec = O.ModelSpec([12, 8], [8, 12], [6, 4], [6, x_dim], x_dim=x_dim)
    params = O.glorot_init(spec, rng, out_bias=rng.normal(size=x_dim) * 0.5)
    return rng, spec, params


LOSS_CASES = [("VAE", {}), ("IWAE", {}), ("L_power_p", dict(p=2.5)), ("L_median", {}),
              ("L_alpha", dict(alpha=0.3)), ("VAE_V1", {}), ("CIWAE", dict(beta=0.3)),
              ("MIWAE", dict(k1=3, k2=2)), ("PIWAE", dict(k1=3, k2=2))]


# ------------------------------------------------------------- golden
@pytest.mark.parametrize("name", ["g1L", "g2L", "g2L784"])
def test_oracle_reproduces_golden(name):
    z = np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)
    spec = O.ModelSpec(list(z["he"]), list(z["hd"]), list(z["le"]), list(z["ld"]), x_dim=int(z["x_dim"]))
    params = O.unflatten_params(spec, z["params"].astype(np.float64))
    x = z["x"].astype(np.float64)
    L = spec.L
    eps = [z[f"eps{i}"].astype(np.float64) for i in range(L)]
    eps2 = [z[f"eps2_{i}"].astype(np.float64) for i in range(L)]
    k, k1, k2 = int(z["k"]), int(z["k1"]), int(z["k2"])
    np.testing.assert_allclose(O.forward(params, spec, x, eps)["lw"], z["lw"], rtol=1e-12)
    for loss, kw in LOSS_CASES:
        kw = dict(kw)
        if loss in ("MIWAE", "PIWAE"):
            kw.update(k1=k1, k2=k2)
        if loss == "CIWAE":
            kw["eps2"] = eps2
        J, g = O.objective_and_grads(params, spec, x, eps, loss, k, **kw)
        assert J == pytest.approx(float(z[f"{loss}.J"]), rel=1e-12)
        if f"{loss}.grad_loss" in z:
            np.testing.assert_allclose(-O.flatten_params(spec, g), z[f"{loss}.grad_loss"], rtol=1e-5, atol=1e-7)


# -------------------------------------------------- finite differences
@pytest.mark.parametrize("loss,kw", LOSS_CASES)
@pytest.mark.parametrize("L", [1, 2])
def test_gradients_match_finite_differences(loss, kw, L):
    rng, spec, params = tiny(1, L)
    B, k = 3, 6
    x = (rng.random((B, spec.x_dim)) < 0.4).astype(np.float64)
    eps = O.draw_eps(spec, k, B, rng)
    kw = dict(kw)
    if loss == "CIWAE":
        kw["eps2"] = O.draw_eps(spec, k, B, rng)
    _, g = O.objective_and_grads(params, spec, x, eps, loss, k, **kw)
    flat, gf = O.flatten_params(spec, params), O.flatten_params(spec, g)
    if loss == "PIWAE":
        # PIWAE's update is not the gradient of one scalar: check each half
        n_enc = sum(fin * fout + fout for n, fin, fout in spec.dense if n.startswith("enc"))
        checks = [("IWAE", {}, slice(n_enc, None)), ("MIWAE", dict(k1=3, k2=2), slice(0, n_enc))]
    else:
        checks = [(loss, kw, slice(None))]
    for l2, kw2, sl in checks:
        idx = np.arange(flat.size)[sl]
        idx = rng.choice(idx, size=min(25, idx.size), replace=False)
        for i in idx:
            h = 1e-6 * max(1.0, abs(flat[i]))
            fp, fm = flat.copy(), flat.copy()
            fp[i] += h
            fm[i] -= h
            Jp, _ = O.objective_and_grads(O.unflatten_params(spec, fp), spec, x, eps, l2, k, with_grads=False, **kw2)
            Jm, _ = O.objective_and_grads(O.unflatten_params(spec, fm), spec, x, eps, l2, k, with_grads=False, **kw2)
            fd = (Jp - Jm) / (2 * h)
            assert abs(fd - gf[i]) <= 1e-5 * max(1.0, abs(fd)), (l2, i, fd, gf[i])


# ------------------------------------ independent torch restatement
def torch_objective(params, spec, x, eps, loss, k, p=1.0, alpha=1.0, beta=0.5, k1=None, k2=None, eps2=None):
    """Independent restatement with torch.distributions and autograd (float64)."""
    from torch.distributions import Bernoulli, Normal
    P = {n: [torch.tensor(w, requires_grad=True), torch.tensor(b, requires_grad=True)] for n, (w, b) in params.items()}

    def stoch(prefix, X):
        y1 = torch.tanh(X @ P[prefix + ".l1"][0] + P[prefix + ".l1"][1])
        y2 = torch.tanh(y1 @ P[prefix + ".l2"][0] + P[prefix + ".l2"][1])
        mu = y2 @ P[prefix + ".lmu"][0] + P[prefix + ".lmu"][1]
        sd = torch.exp(y2 @ P[prefix + ".lstd"][0] + P[prefix + ".lstd"][1])
        return Normal(mu, sd + 1e-6)

    xt = torch.tensor(x)

    def lw_of(ep, need_bce=False):
        L = spec.L
        q = stoch("enc0", xt)
        h = [q.mean + q.stddev * torch.tensor(ep[0])]
        lq = q.log_prob(h[0]).sum(-1)
        dists = [q]
        for i in range(1, L):
            qi = stoch(f"enc{i}", h[-1])
            h.append(qi.mean + qi.stddev * torch.tensor(ep[i]))
            lq = lq + qi.log_prob(h[-1]).sum(-1)
            dists.append(qi)
        o1 = torch.tanh(h[0] @ P["out.l1"][0] + P["out.l1"][1])
        o2 = torch.tanh(o1 @ P["out.l2"][0] + P["out.l2"][1])
        pr = torch.sigmoid(o2 @ P["out.l3"][0] + P["out.l3"][1]) * (1 - 1e-6) + 1e-7
        lpx = Bernoulli(probs=pr).log_prob(xt).sum(-1)
        lp = Normal(0.0, 1.0).log_prob(h[-1]).sum(-1)
        for i in range(L - 1):
            lp = lp + stoch(f"dec{i}", h[L - 1 - i]).log_prob(h[L - 2 - i]).sum(-1)
        lw = lp + lpx - lq
        bce = None
        if need_bce:
            pc = torch.clamp(pr, 1e-7, 1 - 1e-7)
            bce = (xt * torch.log(pc + 1e-7) + (1 - xt) * torch.log(1 - pc + 1e-7)).sum(-1)
        return lw, bce, dists[-1]

    def lse(lw, axis=0):
        return torch.logsumexp(lw, axis) - math.log(lw.shape[axis])

    if loss == "CIWAE":
        J = beta * lw_of(eps)[0].mean() + (1 - beta) * lse(lw_of(eps2)[0]).mean()
    elif loss in ("L_alpha", "VAE_V1"):
        lw, bce, qL = lw_of(eps, need_bce=True)
        if loss == "L_alpha":
            J = (1 - alpha) * bce.mean() + alpha * lw.mean()
        else:
            kl = -0.5 * (1 + 2 * torch.log(qL.stddev) - qL.mean ** 2 - qL.stddev ** 2)
            J = bce.mean() - kl.sum(-1).mean()
    else:
        lw, _, _ = lw_of(eps)
        if loss == "VAE":
            J = lw.mean()
        elif loss in ("IWAE", "PIWAE"):
            J = lse(lw).mean()
        elif loss == "L_power_p":
            J = (lse(lw * p) / p).mean()
        elif loss == "L_median":
            s = torch.sort(lw, 0).values
            J = ((s[(k - 1) // 2] + s[k // 2]) / 2).mean()
        elif loss == "MIWAE":
            J = lse(lw.reshape(k2, k1, -1), 1).mean()
    J.backward()

    def g(t):
        return np.zeros(tuple(t.shape)) if t.grad is None else t.grad.numpy()
    return float(J.detach()), {n: [g(v[0]), g(v[1])] for n, v in P.items()}


@pytest.mark.parametrize("loss,kw", [c for c in LOSS_CASES if c[0] != "PIWAE"])
@pytest.mark.parametrize("L", [1, 2])
def test_oracle_matches_torch_autograd(loss, kw, L):
    rng, spec, params = tiny(2, L)
    B, k = 4, 6
    x = (rng.random((B, spec.x_dim)) < 0.4).astype(np.float64)
    eps = O.draw_eps(spec, k, B, rng)
    kw = dict(kw)
    if loss == "CIWAE":
        kw["eps2"] = O.draw_eps(spec, k, B, rng)
    J, g = O.objective_and_grads(params, spec, x, eps, loss, k, **kw)
    Jt, gt = torch_objective(params, spec, x, eps, loss, k, **kw)
    assert J == pytest.approx(Jt, rel=1e-10)
    np.testing.assert_allclose(O.flatten_params(spec, g), O.flatten_params(spec, gt), rtol=1e-7, atol=1e-10)


# ------------------------------------------------- known-answer identities
def test_identities_from_reference_definitions():
    rng, spec, params = tiny(3, 2)
    B = 5
    x = (rng.random((B, spec.x_dim)) < 0.4).astype(np.float64)
    eps1 = O.draw_eps(spec, 1, B, rng)
    # L_1 == VAE at k = 1 (F:369 vs F:430)
    J1, _ = O.objective_and_grads(params, spec, x, eps1, "IWAE", 1)
    Jv, _ = O.objective_and_grads(params, spec, x, eps1, "VAE", 1)
    assert J1 == pytest.approx(Jv, rel=1e-12)
    k = 6
    eps = O.draw_eps(spec, k, B, rng)
    eps2 = O.draw_eps(spec, k, B, rng)
    Jiw, giw = O.objective_and_grads(params, spec, x, eps, "IWAE", k)
    Jva, gva = O.objective_and_grads(params, spec, x, eps, "VAE", k)
    Jiw2, _ = O.objective_and_grads(params, spec, x, eps2, "IWAE", k)
    # CIWAE(beta=1) == VAE (draw 1), CIWAE(beta=0) == IWAE (draw 2)  (F:383)
    assert O.objective_and_grads(params, spec, x, eps, "CIWAE", k, beta=1.0, eps2=eps2)[0] == pytest.approx(Jva)
    assert O.objective_and_grads(params, spec, x, eps, "CIWAE", k, beta=0.0, eps2=eps2)[0] == pytest.approx(Jiw2)
    # power-p with p = 1 == IWAE (F:408 vs F:369)
    Jp, gp = O.objective_and_grads(params, spec, x, eps, "L_power_p", k, p=1.0)
    assert Jp == pytest.approx(Jiw)
    np.testing.assert_allclose(O.flatten_params(spec, gp), O.flatten_params(spec, giw), rtol=1e-10, atol=1e-12)
    # L_alpha with alpha = 1 == VAE (F:401)
    assert O.objective_and_grads(params, spec, x, eps, "L_alpha", k, alpha=1.0)[0] == pytest.approx(Jva)
    # MIWAE(1, k) == VAE, MIWAE(k, 1) == IWAE (PDF p12 Table 9 caption)
    assert O.objective_and_grads(params, spec, x, eps, "MIWAE", k, k1=1, k2=k)[0] == pytest.approx(Jva)
    assert O.objective_and_grads(params, spec, x, eps, "MIWAE", k, k1=k, k2=1)[0] == pytest.approx(Jiw)
    # PIWAE(k, 1) == IWAE including gradients
    _, gpi = O.objective_and_grads(params, spec, x, eps, "PIWAE", k, k1=k, k2=1)
    np.testing.assert_allclose(O.flatten_params(spec, gpi), O.flatten_params(spec, giw), rtol=1e-10, atol=1e-12)


def test_bound_ordering_in_expectation():
    """L_1 <= L_5 <= L_50 (PDF p5 eq. 3), averaged over draws."""
    rng, spec, params = tiny(4, 1)
    B = 8
    x = (rng.random((B, spec.x_dim)) < 0.4).astype(np.float64)
    vals = {}
    for k in (1, 5, 50):
        vals[k] = np.mean([O.objective_and_grads(params, spec, x, O.draw_eps(spec, k, B, rng), "IWAE", k,
                                                 with_grads=False)[0] for _ in range(40)])
    assert vals[1] < vals[5] < vals[50]


def test_closed_form_densities():
    from scipy import stats
    rng = np.random.default_rng(5)
    x, loc, sc = rng.normal(size=50), rng.normal(size=50), rng.uniform(0.1, 3, 50)
    lp, _ = O.normal_log_prob(x, loc, sc)
    np.testing.assert_allclose(lp, stats.norm.logpdf(x, loc, sc), rtol=1e-12)
    p = rng.uniform(0.01, 0.99, 50)
    xb = (rng.random(50) < 0.5).astype(np.float64)
    np.testing.assert_allclose(np.log1p(-p) * (1 - xb) + np.log(p) * xb, stats.bernoulli.logpmf(xb, p), rtol=1e-12)


def test_median_indices_midpoint():
    assert O.median_indices(50) == (24, 25)
    assert O.median_indices(5) == (2, 2)
    lw = np.arange(10.0)[:, None] * np.ones((1, 3))
    assert O.L_median_from_weights(lw) == pytest.approx(4.5)


def test_adam_matches_tf_kernel_form():
    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    p0 = np.array([1.0, -2.0, 0.5])
    g = np.array([0.1, -0.3, 0.0])
    p1 = opt.apply(p0.copy(), g)
    alpha = 1e-3 * math.sqrt(1 - 0.999) / (1 - 0.9)
    m = 0.1 * g
    v = 0.001 * g * g
    np.testing.assert_allclose(p1, p0 - m * alpha / (np.sqrt(v) + 1e-4), rtol=1e-12)
    assert opt.t == 1


def test_nll_chunked_lse_equals_whole():
    rng, spec, params = tiny(6, 2)
    B, k = 3, 37
    x = (rng.random((B, spec.x_dim)) < 0.4).astype(np.float64)
    eps = O.draw_eps(spec, k, B, rng)
    whole = O.L_k_per_image(O.forward(params, spec, x, eps)["lw"])
    np.testing.assert_allclose(O.log_px_per_image(params, spec, x, k, eps=eps, chunk=10), whole, rtol=1e-12)


def test_spec_param_counts_match_survey():
    # 425,284 (1L) and 521,084 (2L) parameters
    assert O.ModelSpec([200], [200], [50], [784]).n_params() == 425284
    assert O.ModelSpec([200, 100], [100, 200], [100, 50], [100, 784]).n_params() == 521084


# ------------------------------------------------ evaluation statistics (F:249-F:300, F:466-F:494)
def _stat_model(L, seed=3):
    from oracle import iwae_oracle as O
    arch = {1: ([32], [32], [8], [784]), 2: ([32, 16], [16, 32], [12, 6], [12, 784])}[L]
    spec = O.ModelSpec(*arch)
    rng = np.random.default_rng(seed)
    mean = rng.uniform(0.05, 0.4, 784)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    x = (rng.random((5, 784)) < mean).astype(np.float64)
    return O, spec, params, x, rng


def test_oracle_reconstruction_one_layer_is_the_forward_decoder():
    """L=1: generate_x has no prior layers, so the probabilities are the
    forward pass's p on the same encoder draw; loss = mean_B sum Keras BCE."""
    O, spec, params, x, rng = _stat_model(1)
    eps = O.draw_eps(spec, 1, x.shape[0], rng)
    p, loss = O.reconstruct(params, spec, x, eps, [])
    c = O.forward(params, spec, x, eps, need_bce=True)
    np.testing.assert_allclose(p, c["p"], rtol=1e-12)
    np.testing.assert_allclose(loss, -c["bce_row"].mean(), rtol=1e-12)


def test_oracle_reconstruction_two_layers_redraws_h1_from_the_prior():
    O, spec, params, x, rng = _stat_model(2)
    B = x.shape[0]
    eps = O.draw_eps(spec, 1, B, rng)
    pri = [rng.standard_normal((1, B, spec.n_latent_encoder[0]))]
    p, _ = O.reconstruct(params, spec, x, eps, pri)
    c = O.forward(params, spec, x, eps)
    d0 = O._stoch_forward(params, "dec0", c["h"][1])
    h1 = pri[0] * d0["scale"] + d0["mu"]
    c2 = O.forward(params, spec, x, [(h1 - c["enc"][0]["mu"]) / c["enc"][0]["scale"], eps[1]])
    # forcing the encoder's h1 to the prior draw gives the same decoder input
    np.testing.assert_allclose(c2["h"][0], h1, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(p, c2["p"], rtol=1e-9)


def test_oracle_pca_eigenvalues_sum_to_the_variances():
    """trace(cov) = sum of per-unit population variances; eigenvalues >= 0."""
    O, spec, params, x, rng = _stat_model(2)
    eps = O.draw_eps(spec, 7, x.shape[0], rng)
    var, eig = O.levels_of_units_activity(O.encoder_means(params, spec, x, eps))
    for v, e in zip(var, eig):
        np.testing.assert_allclose(e.sum(), v.sum(), rtol=1e-10)
        assert e.min() > -1e-12
    au, n_au, n_pca = O.active_units([np.array([0.5, 0.001, 0.02])], [np.array([0.0, 0.005, 0.6])])
    assert au == [[1, 0, 1]] and n_au == [2] and n_pca == [1]


def test_oracle_masks_of_ones_change_nothing_and_zero_masks_pin_h():
    O, spec, params, x, rng = _stat_model(2)
    eps = O.draw_eps(spec, 4, x.shape[0], rng)
    ones = [np.ones(d) for d in spec.n_latent_encoder]
    a = O.forward(params, spec, x, eps)["lw"]
    b = O.forward(params, spec, x, eps, masks=ones)["lw"]
    np.testing.assert_array_equal(a, b)
    zero = [np.zeros(d) for d in spec.n_latent_encoder]
    c = O.forward(params, spec, x, eps, masks=zero)
    assert all(np.all(h == 0) for h in c["h"])
