"""GPU parity: the HIP path (through the C ABI / Flexible_Model facade) against
the float64 CPU oracle and the golden fixtures, on identical injected noise and
weights.  Tolerances (north_star): losses and gradients 1e-4 relative; NLL
0.05 nats.  Run as: python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REL = 1e-4          # losses / gradients (north_star)
NLL_TOL = 0.05      # nats
# Post-Adam weights: Adam's first step lr*g/(|g|+eps) amplifies a gradient's
# absolute error by up to lr/eps = 10 for near-zero gradient elements.  The
# tiled GEMMs default to bf16x3 products (a_hi b_hi + a_hi b_lo + a_lo b_hi,
# <= ~2.3e-5 relative per product), so isolated near-zero gradient elements
# carry up to ~5e-6 absolute error: 6e-5 = 6% of lr on the weights.
ADAM_ATOL = 6e-5


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    return torch


def make_model(he, hd, le, ld, x_dim=784, loss="IWAE", k=5, seed=0, **kw):
    from iwae_replication_project_amd import Flexible_Model
    return Flexible_Model(he, hd, le, ld, dataset_bias=None, loss_function=loss, k=k, x_dim=x_dim, seed=seed, **kw)


def flat(ws):
    return np.concatenate([np.asarray(w, np.float64).ravel() for w in ws])


def rel_l2(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-30))


def load_gold(name):
    z = np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)
    L = len(z["he"])
    g = dict(he=list(z["he"]), hd=list(z["hd"]), le=list(z["le"]), ld=list(z["ld"]), x_dim=int(z["x_dim"]),
             B=int(z["B"]), k=int(z["k"]), k1=int(z["k1"]), k2=int(z["k2"]), params=z["params"], x=z["x"],
             eps=[z[f"eps{i}"] for i in range(L)], eps2=[z[f"eps2_{i}"] for i in range(L)], lw=z["lw"],
             logpx=z["logpx"], bce_mean=float(z["bce_mean"]), z=z)
    return g


def weights_from_flat(model, fl):
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    return _split(np.asarray(fl, np.float32), weight_shapes(model.dense))


LOSS_KW = {"VAE": {}, "IWAE": {}, "L_power_p": dict(p=2.5), "L_median": {}, "L_alpha": dict(alpha=0.3),
           "VAE_V1": {}, "CIWAE": dict(beta=0.3), "MIWAE": {}, "PIWAE": {}}


# ------------------------------------------------------------- GEMM unit
@pytest.mark.parametrize("precision,tol", [("f32", 2e-6), ("bf16x3", 3e-5)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 16), (37, 53, 20), (130, 300, 68), (1000, 784, 200), (5, 7, 4)])
def test_debug_gemm_matches_fp32_reference(torch_mod, M, N, K, precision, tol):
    torch = torch_mod
    from iwae_replication_project_amd import _lib
    m = make_model([16], [16], [4], [64], x_dim=64, precision=precision)
    g = torch.Generator().manual_seed(M * 1000 + N)
    lda, ldb, ldc = (K + 3) // 4 * 4, (N + 3) // 4 * 4, (N + 3) // 4 * 4
    A = torch.zeros(M, lda)
    B = torch.zeros(K, ldb)
    A[:, :K] = torch.randn(M, K, generator=g)
    B[:, :N] = torch.randn(K, N, generator=g) + torch.arange(N).float() * 0.01   # asymmetric
    Ad, Bd = A.cuda(), B.cuda()
    Cd = torch.zeros(M, ldc, device="cuda")
    torch.cuda.synchronize()
    m._call(m._lib.iwae_debug_gemm(m._h, _lib.fptr(Ad), lda, _lib.fptr(Bd), ldb, _lib.fptr(Cd), ldc, M, N, K))
    m._stream.synchronize()
    ref = (A[:, :K].double() @ B[:, :N].double())
    err = (Cd[:, :N].cpu().double() - ref).abs().max().item()
    scale = (A[:, :K].abs().double() @ B[:, :N].abs().double()).max().item()
    # f32: exact fmaf chain; bf16x3: (2^-16 + 2^-17) relative per product, worst case
    assert err <= tol * scale, (err, scale)


# ---------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("name", ["g1L", "g2L", "g2L784"])
def test_log_weights_match_golden(name):
    g = load_gold(name)
    m = make_model(g["he"], g["hd"], g["le"], g["ld"], x_dim=g["x_dim"])
    m.set_weights(weights_from_flat(m, g["params"]))
    lw = m.get_log_weights(g["x"], g["k"], eps=g["eps"]).cpu().numpy()
    ref = g["lw"]
    assert np.max(np.abs(lw - ref)) <= REL * np.max(np.abs(ref)), np.max(np.abs(lw - ref))


@pytest.mark.parametrize("loss", list(LOSS_KW))
@pytest.mark.parametrize("name", ["g1L", "g2L", "g2L784"])
def test_bound_and_gradients_match_golden(name, loss):
    g = load_gold(name)
    kw = dict(LOSS_KW[loss])
    if loss in ("MIWAE", "PIWAE"):
        kw.update(k1=g["k1"], k2=g["k2"])
    m = make_model(g["he"], g["hd"], g["le"], g["ld"], x_dim=g["x_dim"], loss=loss, k=g["k"], **kw)
    m.set_weights(weights_from_flat(m, g["params"]))
    eps = g["eps"] + (g["eps2"] if loss == "CIWAE" else [])
    J = float(g["z"][f"{loss}.J"])
    # forward-only bound (get_L, get_L_k, ... F:354-F:460)
    if loss not in ("PIWAE",):
        lc = m._lc()
        val = m._bound(lc, g["x"], eps, 2 if loss == "CIWAE" else 1)
        assert abs(val - J) <= REL * abs(J), (val, J)
    # train step: returned loss == -J, gradient of the loss
    from iwae_replication_project_amd import Adam
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    out = m.train_step(g["x"], eps=eps)[loss]
    assert abs(out + J) <= REL * abs(J), (out, -J)
    key = f"{loss}.grad_loss"
    if key in g["z"]:
        gref = g["z"][key].astype(np.float64)
        gg = flat(m.get_gradients())
        assert rel_l2(gg, gref) <= REL, rel_l2(gg, gref)
        # per-element: within REL of the largest element of each parameter tensor
        o = 0
        for w in weights_from_flat(m, gref):
            n = w.size
            a, b = gg[o:o + n], gref[o:o + n]
            assert np.max(np.abs(a - b)) <= 5 * REL * max(np.max(np.abs(b)), 1e-8), (o, np.max(np.abs(a - b)))
            o += n


@pytest.mark.parametrize("name", ["g1L", "g2L", "g2L784"])
def test_nll_and_e_log_px_match_golden(name):
    g = load_gold(name)
    m = make_model(g["he"], g["hd"], g["le"], g["ld"], x_dim=g["x_dim"])
    m.set_weights(weights_from_flat(m, g["params"]))
    lp = m.log_px(g["x"], g["k"], eps=g["eps"]).cpu().numpy()
    assert np.max(np.abs(lp - g["logpx"])) <= 1e-3
    eq = m.get_E_qhIx_log_pxIh(g["x"], g["k"], eps=g["eps"])
    assert abs(eq - g["bce_mean"]) <= REL * abs(g["bce_mean"])


# --------------------------------------------- full-size config C2 vs oracle
def test_c2_full_size_iwae_train_step_matches_oracle():
    """2L 784-200-200-100-100-50, k=50, batch 20 (BASELINE config 2): loss,
    gradients and post-Adam weights against the float64 oracle."""
    from oracle import iwae_oracle as O
    he, hd, le, ld = [200, 100], [100, 200], [100, 50], [100, 784]
    B, k = 20, 50
    rng = np.random.default_rng(11)
    mean = rng.uniform(0.01, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    x = (rng.random((B, 784)) < mean).astype(np.float64)
    eps = [e.astype(np.float32).astype(np.float64) for e in O.draw_eps(spec, k, B, rng)]
    from iwae_replication_project_amd import Adam
    m = make_model(he, hd, le, ld, loss="IWAE", k=k)
    m.set_weights(weights_from_flat(m, O.flatten_params(spec, params)))
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    loss = m.train_step(x.astype(np.float32), eps=[e.astype(np.float32) for e in eps])["IWAE"]
    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    ref_loss, ref_new, ref_g = O.train_step(params, spec, x, eps, "IWAE", k, opt)
    assert abs(loss - ref_loss) <= REL * abs(ref_loss)
    assert rel_l2(flat(m.get_gradients()), ref_g) <= REL
    # Adam's first step lr*g/(|g|+eps) amplifies gradient rounding by up to lr/eps = 10
    # for near-zero gradients: allow 2% of lr on the updated weights
    np.testing.assert_allclose(flat(m.get_weights()), O.flatten_params(spec, ref_new), atol=ADAM_ATOL)


@pytest.mark.parametrize("path", ["fused", "engine"])
@pytest.mark.parametrize("loss", ["IWAE", "VAE", "CIWAE", "PIWAE", "VAE_V1", "L_alpha", "L_median", "MIWAE",
                                  "L_power_p"])
@pytest.mark.parametrize("arch", [([64], [64], [16], [784]), ([64, 32], [32, 64], [32, 16], [32, 784]),
                                  ([48, 32, 24], [24, 32, 48], [20, 12, 8], [12, 20, 784])])
def test_fused_and_layerwise_paths_agree(arch, loss, path):
    """The fused row-block kernels / the bf16x3 row-chain engine and the
    layer-wise GEMM kernels compute the same train step (same Philox noise):
    loss, gradients and updated weights.  (The engine runs every loss but
    VAE_V1 / L_alpha / PIWAE; those take the fused kernels under "engine".)"""
    he, hd, le, ld = arch
    rng = np.random.default_rng(19)
    x = (rng.random((9, 784)) < 0.2).astype(np.float32)
    kw = dict(k1=3, k2=2) if loss in ("PIWAE", "MIWAE") else {}
    if loss == "L_power_p":
        kw["p"] = 2.0
    outs = []
    for path in ("layerwise", path):
        from iwae_replication_project_amd import Adam
        m = make_model(he, hd, le, ld, loss=loss, k=6, seed=77, kernel_path=path, alpha=0.4, beta=0.3, **kw)
        m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        l1 = m.train_step(x)[loss]
        g1 = flat(m.get_gradients())
        l2 = m.train_step(x)[loss]
        outs.append((l1, l2, g1, flat(m.get_weights())))
    (a1, a2, ga, wa), (b1, b2, gb, wb) = outs
    # two independent approximations, each within REL of the exact value: |a - b| <= 2 REL
    assert abs(a1 - b1) <= 2 * REL * abs(a1) and abs(a2 - b2) <= 2 * REL * abs(a2)
    assert rel_l2(gb, ga) <= 2 * REL
    np.testing.assert_allclose(wb, wa, atol=2 * ADAM_ATOL)      # see the Adam note above


@pytest.mark.parametrize("d0", [130, 260])
def test_engine_wide_first_latent_agrees_with_layerwise(d0):
    """A first latent wider than 128 (the image-row Gaussian backward splits
    d0 / 4 column quads over the workgroup): engine and layer-wise steps agree."""
    rng = np.random.default_rng(23)
    x = (rng.random((5, 784)) < 0.2).astype(np.float32)
    outs = []
    for path in ("layerwise", "engine"):
        from iwae_replication_project_amd import Adam
        m = make_model([64, 32], [32, 64], [d0, 16], [d0, 784], loss="IWAE", k=7, seed=5, kernel_path=path)
        m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        l1 = m.train_step(x)["IWAE"]
        outs.append((l1, flat(m.get_gradients())))
    (a1, ga), (b1, gb) = outs
    assert abs(a1 - b1) <= 2 * REL * abs(a1)
    assert rel_l2(gb, ga) <= 2 * REL


def test_fused_and_layerwise_paths_agree_at_large_batch():
    """configs[1]/[4] architecture at 10,000 sample rows (B=200, k=50): the
    large-batch kernel choices of the fused step (128x128 output-layer dX
    tiles, more weight-gradient slabs) against the layer-wise step."""
    he, hd, le, ld = [200, 100], [100, 200], [100, 50], [100, 784]
    rng = np.random.default_rng(23)
    x = (rng.random((200, 784)) < 0.15).astype(np.float32)
    outs = []
    for path in ("layerwise", "fused"):
        from iwae_replication_project_amd import Adam
        m = make_model(he, hd, le, ld, loss="IWAE", k=50, seed=78, kernel_path=path)
        m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        l1 = m.train_step(x)["IWAE"]
        outs.append((l1, flat(m.get_gradients()), flat(m.get_weights())))
    (a1, ga, wa), (b1, gb, wb) = outs
    assert abs(a1 - b1) <= 2 * REL * abs(a1)
    assert rel_l2(gb, ga) <= 2 * REL
    np.testing.assert_allclose(wb, wa, atol=2 * ADAM_ATOL)


# ----------------------------------------------- multi-step training parity
def test_five_adam_steps_track_oracle():
    from oracle import iwae_oracle as O
    he, hd, le, ld = [64], [64], [16], [784]
    B, k = 8, 5
    rng = np.random.default_rng(12)
    mean = rng.uniform(0.02, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    from iwae_replication_project_amd import Adam
    m = make_model(he, hd, le, ld, loss="IWAE", k=k)
    m.set_weights(weights_from_flat(m, O.flatten_params(spec, params)))
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    for step in range(5):
        x = (rng.random((B, 784)) < mean).astype(np.float64)
        eps = [e.astype(np.float32).astype(np.float64) for e in O.draw_eps(spec, k, B, rng)]
        loss = m.train_step(x.astype(np.float32), eps=[e.astype(np.float32) for e in eps])["IWAE"]
        ref_loss, params, _ = O.train_step(params, spec, x, eps, "IWAE", k, opt)
        assert abs(loss - ref_loss) <= REL * abs(ref_loss), (step, loss, ref_loss)
    np.testing.assert_allclose(flat(m.get_weights()), O.flatten_params(spec, params), atol=1e-5)
    _, _, t = m.get_optimizer_state()
    assert t == 5


# -------------------------------------------------- device-noise (Philox) path
def test_philox_path_graphs_equal_eager_and_is_reproducible():
    he, hd, le, ld = [200, 100], [100, 200], [100, 50], [100, 784]
    rng = np.random.default_rng(13)
    x = (rng.random((20, 784)) < 0.15).astype(np.float32)
    runs = []
    for graphs in (True, False):
        m = make_model(he, hd, le, ld, loss="IWAE", k=50, seed=42, use_graphs=graphs)
        from iwae_replication_project_amd import Adam
        m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        losses = [m.train_step(x)["IWAE"] for _ in range(4)]
        runs.append((losses, flat(m.get_weights())))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    assert len(set(runs[0][0])) == 4       # fresh noise every step


def test_graph_replays_follow_the_callers_batch():
    """The captured train step reads each call's x where the caller keeps it
    (its input-layer launch is re-pointed per replay): different device
    batches at different addresses give the same losses and weights as eager."""
    import torch
    he, hd, le, ld = [200, 100], [100, 200], [100, 50], [100, 784]
    rng = np.random.default_rng(31)
    xs = (rng.random((5 * 20, 784)) < 0.2).astype(np.float32)
    runs = []
    for graphs in (True, False):
        m = make_model(he, hd, le, ld, loss="IWAE", k=50, seed=7, use_graphs=graphs)
        from iwae_replication_project_amd import Adam
        m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        X = torch.from_numpy(xs).to(m.device)
        order = [0, 3, 1, 3, 4, 2]
        losses = [m.train_step(X[i * 20:(i + 1) * 20])["IWAE"] for i in order]
        runs.append((losses, flat(m.get_weights())))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize("loss", ["IWAE", "PIWAE"])
def test_gradient_snr_harness_matches_per_draw_gradients(loss):
    """get_gradient_snr (device moment accumulation over R Philox draws) equals
    the SNR computed on the host from the same R draws' gradients, one
    forward_backward + get_gradients at a time (same seed, same stream)."""
    he, hd, le, ld = [64, 32], [32, 64], [32, 16], [32, 784]
    rng = np.random.default_rng(41)
    x = (rng.random((6, 784)) < 0.2).astype(np.float32)
    kw = dict(k1=4, k2=2) if loss == "PIWAE" else {}
    k = 8
    R = 40
    a = make_model(he, hd, le, ld, loss=loss, k=k, seed=5, **kw)
    snr, info = a.get_gradient_snr(x, R=R, seed=123)
    b = make_model(he, hd, le, ld, loss=loss, k=k, seed=5, **kw)
    b.set_weights(a.get_weights())
    b._call(b._lib.iwae_set_seed(b._h, 123))
    xd = b._x(x)
    lc = b._lc()
    gs = []
    for _ in range(R):
        b._forward_backward(lc, xd, xd.shape[0], None, 0)
        gs.append(flat(b.get_gradients()))
    G = np.stack(gs)
    mean = G.mean(0)
    sd = np.sqrt(np.maximum((G * G).mean(0) - mean * mean, 0.0))
    ref = np.where(sd > 0, np.abs(mean) / np.where(sd > 0, sd, 1.0), np.inf)
    got = flat(snr)
    fin = np.isfinite(ref) & (sd > 1e-6 * np.abs(mean).max())
    assert info["R"] == R and np.isfinite(got[fin]).all()
    np.testing.assert_allclose(got[fin], ref[fin], rtol=2e-3, atol=1e-4)


def test_philox_noise_statistics_match_oracle_vae_bound():
    """The VAE bound mean_{s,b} lw depends on the whole noise distribution:
    estimate it with device Philox noise and with numpy noise in the oracle
    (k=4000, 6 images) and require agreement within 5 standard errors."""
    from oracle import iwae_oracle as O
    he, hd, le, ld = [64, 32], [32, 64], [32, 16], [32, 784]
    rng = np.random.default_rng(18)
    mean = rng.uniform(0.02, 0.3, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    m = make_model(he, hd, le, ld, seed=21)
    m.set_weights(weights_from_flat(m, O.flatten_params(spec, params)))
    x = (rng.random((6, 784)) < mean).astype(np.float32)
    k = 4000
    gpu = m.get_L(x, k)
    lw = O.forward(params, spec, x.astype(np.float64), O.draw_eps(spec, k, 6, rng))["lw"]
    se = lw.std() / math.sqrt(lw.size)
    assert abs(gpu - lw.mean()) <= 5 * se + 1e-4 * abs(lw.mean()), (gpu, lw.mean(), se)


def _concentrated_model(seed, he=(64,), le=(16,)):
    """A model whose log-weights barely depend on the noise: encoder heads zero
    (q = N(0, (1+1e-6)^2) ~ prior) and decoder output kernel scaled by 1e-3, so
    every k-sample estimate of log p(x) agrees to ~1e-3 nats.  This isolates
    the NLL machinery (sampling, LSE over k, chunk merging) from Monte-Carlo
    spread, which for an untrained model is tens of nats."""
    from oracle import iwae_oracle as O
    he, le = list(he), list(le)
    hd, ld = list(reversed(he)), [*le[:-1][::-1], 784] if len(le) > 1 else [784]
    spec = O.ModelSpec(he, hd, le, ld)
    rng = np.random.default_rng(seed)
    mean = rng.uniform(0.02, 0.3, 784)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    for n in params:
        if n.startswith("enc") and (n.endswith("lmu") or n.endswith("lstd")):
            params[n] = [np.zeros_like(params[n][0]), np.zeros_like(params[n][1])]
        if n.startswith("dec") and (n.endswith("lmu") or n.endswith("lstd")):
            params[n] = [np.zeros_like(params[n][0]), np.zeros_like(params[n][1])]
    params["out.l3"][0] = params["out.l3"][0] * 1e-3
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    m = make_model(he, hd, le, ld, seed=seed)
    m.set_weights(weights_from_flat(m, O.flatten_params(spec, params)))
    x = (rng.random((6, 784)) < mean).astype(np.float32)
    return O, spec, params, m, x, rng


@pytest.mark.parametrize("layers", [((64,), (16,)), ((64, 32), (32, 16))])
def test_nll_k5000_matches_oracle_within_0p05_nats(layers):
    """k=5000 NLL from device Philox noise vs the float64 oracle with its own
    numpy noise (north_star: 0.05 nats)."""
    O, spec, params, m, x, rng = _concentrated_model(3, *layers)
    nll_gpu = m.get_NLL(x, k=5000)
    ref = -np.mean(O.log_px_per_image(params, spec, x.astype(np.float64), 5000, rng=rng, chunk=1000))
    assert abs(nll_gpu - ref) <= NLL_TOL, (nll_gpu, ref)
    assert abs(nll_gpu - ref) <= 5e-3, (nll_gpu, ref)


@pytest.mark.parametrize("arch", [([64], [64], [16], [784]), ([40], [40], [6], [784]),
                                  ([64, 32], [32, 64], [32, 16], [32, 784]),
                                  ([48, 32, 24], [24, 32, 48], [20, 12, 8], [12, 20, 784]),
                                  ([200, 100], [100, 200], [100, 50], [100, 784])])
@pytest.mark.parametrize("pixels", ["binary", "fractional"])
def test_fused_nll_kernel_matches_layerwise_path(arch, pixels):
    """The fused k-sample kernel (activations in LDS, sampling and prior density
    in the MFMA epilogue, product-of-probabilities Bernoulli sum) and the
    layer-wise GEMM path give the same per-image log p(x) on the same Philox
    noise; fractional pixels take the two-log Bernoulli form."""
    he, hd, le, ld = arch
    rng = np.random.default_rng(23)
    x = rng.random((5, 784)).astype(np.float32)
    if pixels == "binary":
        x = (x < 0.25).astype(np.float32)
    out = {}
    for path in ("layerwise", "fused"):
        m = make_model(he, hd, le, ld, seed=41, kernel_path=path)
        if path == "layerwise":
            w0 = m.get_weights()
        else:
            m.set_weights(w0)
        out[path] = m.log_px(x, 700).cpu().numpy().astype(np.float64)
    a, b = out["layerwise"], out["fused"]
    assert np.all(np.isfinite(b))
    np.testing.assert_allclose(b, a, rtol=2e-5, atol=2e-3)


@pytest.mark.parametrize("arch", [([200, 100], [100, 200], [100, 50], [100, 784]),    # configs[1..4]
                                  ([200], [200], [50], [784])])                          # configs[0]
@pytest.mark.parametrize("pixels", ["binary", "fractional"])
@pytest.mark.parametrize("k", [700, 5000, 100])
def test_weight_ring_nll_kernel_matches_register_streaming_kernel(arch, pixels, k):
    """The weight-ring NLL kernel (nring_kernel: activations of 16 rows per wave
    in registers, weights shared by 128 rows through an LDS-DMA ring) against
    mega_fwd_kernel on the same Philox noise and weights: same products in the
    same order, so per-image log p(x) agree to float rounding.  k=700 puts
    image boundaries inside workgroups and a ragged last workgroup; k=100
    (< 128 samples per image) runs mega_fwd_kernel on both sides (counter)."""
    he, hd, le, ld = arch
    rng = np.random.default_rng(29)
    x = rng.random((5, 784)).astype(np.float32)
    if pixels == "binary":
        x = (x < 0.25).astype(np.float32)
    out = {}
    for ring in (0, 1):
        m = make_model(he, hd, le, ld, seed=43)
        if ring == 0:
            w0 = m.get_weights()
        else:
            m.set_weights(w0)
        m.set_tuning("nring", ring)
        n0 = m._lib.iwae_debug_count(m._h, 3)
        out[ring] = m.log_px(x, k).cpu().numpy().astype(np.float64)
        launches = m._lib.iwae_debug_count(m._h, 3) - n0
        assert (launches > 0) == (ring == 1 and k >= 128), (ring, k, launches)
    assert np.all(np.isfinite(out[1]))
    np.testing.assert_allclose(out[1], out[0], rtol=1e-5, atol=2e-4)


def test_nll_chunking_and_sample_split_are_consistent():
    O, spec, params, m, x, rng = _concentrated_model(4, (64, 32), (32, 16))
    a = m.log_px(x, 3000, chunk=6).cpu().numpy()
    b = m.log_px(x, 3000, chunk=2).cpu().numpy()
    assert np.all(np.isfinite(a)) and np.all(np.isfinite(b))
    np.testing.assert_allclose(a, b, atol=2e-3)
    # sample-sharded partials merged like two ranks: M = max m, S = sum s exp(m - M)
    import torch
    from iwae_replication_project_amd import _lib
    parts = []
    for kl in (1200, 1800):
        xd = m._x(x)
        mm = torch.empty(6, device=m.device)
        ss = torch.empty(6, device=m.device)
        m._call(m._lib.iwae_nll_partials(m._h, _lib.fptr(xd), 6, kl, 0, _lib.fptr(mm), _lib.fptr(ss)))
        m._stream.synchronize()
        parts.append((mm.cpu().double(), ss.cpu().double()))
    M = torch.maximum(parts[0][0], parts[1][0])
    S = sum(s * torch.exp(mm - M) for mm, s in parts)
    merged = (M + torch.log(S) - math.log(3000)).numpy()
    np.testing.assert_allclose(merged, a, atol=2e-3)


def test_nll_full_model_is_a_bound_upper_than_elbo():
    """Untrained 2L model (heavy-tailed weights): L_5000 >= L_VAE on average
    (PDF p5 eq. 3) and every per-image estimate is finite."""
    he, hd, le, ld = [200, 100], [100, 200], [100, 50], [100, 784]
    rng = np.random.default_rng(15)
    x = (rng.random((7, 784)) < 0.15).astype(np.float32)
    m = make_model(he, hd, le, ld, seed=9)
    lp = m.log_px(x, 5000).cpu().numpy()
    assert np.all(np.isfinite(lp))
    assert float(lp.mean()) > m.get_L(x, 1000)


# --------------------------------------------------------- data parallel (1 rank)
def test_data_parallel_single_rank_equals_train_step():
    from iwae_replication_project_amd import Adam, distributed
    he, hd, le, ld = [64, 32], [32, 64], [32, 16], [32, 784]
    rng = np.random.default_rng(16)
    x = (rng.random((12, 784)) < 0.2).astype(np.float32)
    from oracle import iwae_oracle as O
    spec = O.ModelSpec(he, hd, le, ld)
    eps = [e.astype(np.float32) for e in O.draw_eps(spec, 5, 12, rng)]
    ms = []
    for dp in (False, True):
        m = make_model(he, hd, le, ld, loss="IWAE", k=5, seed=1)
        m.compile(Adam(learning_rate=1e-3))
        if dp:
            distributed.enable_data_parallel(m)
        ms.append((m.train_step(x, eps=eps)["IWAE"], flat(m.get_weights())))
    assert ms[0][0] == ms[1][0]
    np.testing.assert_array_equal(ms[0][1], ms[1][1])


def test_unknown_loss_raises_value_error():
    with pytest.raises(ValueError):
        make_model([16], [16], [4], [784], loss="NOT_A_LOSS")


def test_fit_runs_epochs_and_decreases_loss():
    he, hd, le, ld = [64], [64], [16], [784]
    rng = np.random.default_rng(17)
    mean = rng.uniform(0.02, 0.4, 784)
    x = (rng.random((400, 784)) < mean).astype(np.float32)
    from iwae_replication_project_amd import Adam
    m = make_model(he, hd, le, ld, loss="IWAE", k=5, seed=2)
    m.compile(Adam(learning_rate=3e-3, epsilon=1e-4))
    hist = m.fit(x, epochs=4, batch_size=100, seed=0)["IWAE"]
    assert len(hist) == 4 and hist[-1] < hist[0]
