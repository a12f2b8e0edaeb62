"""GPU edge cases of the train step against the float64 oracle: ragged batch
sizes around the kernels' row-block / few-row / tile boundaries, k = 1 (the
LSE over one sample, F:369), batch-size changes between captured-graph
replays, and the argument errors the C ABI reports.  Same tolerances as
test_gpu_parity.py (north_star: 1e-4 relative on losses and gradients)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-4
ADAM_ATOL = 6e-5        # see test_gpu_parity.py: Adam's first step amplifies near-zero gradient errors
ARCH2 = ([200, 100], [100, 200], [100, 50], [100, 784])     # BASELINE configs[1] architecture


def _flat(ws):
    return np.concatenate([np.asarray(w, np.float64).ravel() for w in ws])


def _rel_l2(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-30))


def _model(arch, loss, k, **kw):
    from iwae_replication_project_amd import Adam, Flexible_Model
    he, hd, le, ld = arch
    m = Flexible_Model(he, hd, le, ld, dataset_bias=None, loss_function=loss, k=k, seed=3, **kw)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    return m


def _oracle_case(arch, B, k, seed):
    from oracle import iwae_oracle as O
    he, hd, le, ld = arch
    rng = np.random.default_rng(seed)
    mean = rng.uniform(0.01, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    x = (rng.random((B, 784)) < mean).astype(np.float64)
    eps = [e.astype(np.float32).astype(np.float64) for e in O.draw_eps(spec, k, B, rng)]
    return O, spec, params, x, eps


# B: 1 image; 15/17 around the 16-row blocks; 32/33 around the few-row input-layer
# path (<= 32 images); k=1 and odd k put the sample rows off every tile boundary
# (200, 50): 10,000 sample rows, where the output layer's GEMMs switch to bf16x3 products
@pytest.mark.parametrize("B,k", [(1, 1), (1, 50), (15, 3), (17, 7), (32, 50), (33, 50), (65, 13), (200, 50)])
def test_ragged_batches_match_oracle(B, k):
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    O, spec, params, x, eps = _oracle_case(ARCH2, B, k, 100 + 7 * B + k)
    m = _model(ARCH2, "IWAE", k)
    m.set_weights(_split(O.flatten_params(spec, params).astype(np.float32), weight_shapes(m.dense)))
    loss = m.train_step(x.astype(np.float32), eps=[e.astype(np.float32) for e in eps])["IWAE"]
    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    ref_loss, ref_new, ref_g = O.train_step(params, spec, x, eps, "IWAE", k, opt)
    assert abs(loss - ref_loss) <= REL * abs(ref_loss), (loss, ref_loss)
    g = _flat(m.get_gradients())
    assert _rel_l2(g, ref_g) <= REL
    # the device Adam step is exactly Adam (E:36-E:40) applied to the device gradient; the
    # weights then follow the oracle's within 10x the gradient error (lr/eps = 10 bounds
    # d(update)/dg at step 1: near-zero gradient elements amplify their rounding)
    w0 = O.flatten_params(spec, params)
    np.testing.assert_allclose(_flat(m.get_weights()), O.Adam(1e-3, 0.9, 0.999, 1e-4).apply(w0, g), atol=2e-6)
    np.testing.assert_allclose(_flat(m.get_weights()), O.flatten_params(spec, ref_new),
                               atol=max(ADAM_ATOL, 10 * np.abs(g - ref_g).max()))


def test_k1_iwae_equals_vae():
    """IWAE with k = 1 is the VAE bound (F:369 vs F:331): same noise, same loss and gradient."""
    rng = np.random.default_rng(5)
    x = (rng.random((9, 784)) < 0.2).astype(np.float32)
    eps = [rng.standard_normal((1, 9, d)).astype(np.float32) for d in ARCH2[2]]
    out = []
    for loss in ("IWAE", "VAE"):
        m = _model(ARCH2, loss, 1)
        out.append((m.train_step(x, eps=eps)[loss], _flat(m.get_gradients())))
    (a, ga), (b, gb) = out
    assert abs(a - b) <= REL * abs(a)
    assert _rel_l2(ga, gb) <= REL


def test_batch_size_changes_between_graph_replays():
    """Captured graphs are per batch shape: alternating batch sizes (few-row
    path, its boundary and the tiled path) give bit-identical losses and
    weights with and without graphs."""
    import torch
    rng = np.random.default_rng(41)
    xs = (rng.random((120, 784)) < 0.2).astype(np.float32)
    sizes = [20, 7, 33, 20, 64, 7, 20]
    runs = []
    for graphs in (True, False):
        m = _model(ARCH2, "IWAE", 50, use_graphs=graphs)
        X = torch.from_numpy(xs).to(m.device)
        losses, o = [], 0
        for b in sizes:
            losses.append(m.train_step(X[o:o + b])["IWAE"])
            o = (o + b) % 50
        runs.append((losses, _flat(m.get_weights())))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


def test_invalid_arguments_raise():
    """An empty batch and p = 0 are rejected by the C ABI (IWAE_EINVAL, raised as
    ValueError, the F:242 analogue); wrong eps counts and shapes by the facade."""
    m = _model(ARCH2, "IWAE", 5)
    with pytest.raises(ValueError):
        m.train_step(np.zeros((0, 784), np.float32))
    x = np.zeros((4, 784), np.float32)
    with pytest.raises(ValueError):
        m.train_step(x, eps=[np.zeros((5, 4, 100), np.float32)])          # one eps buffer for two layers
    with pytest.raises(ValueError):
        _model(ARCH2, "L_power_p", 5, p=0.0).train_step(x)
    with pytest.raises(ValueError):
        m.train_step(x, eps=[np.zeros((5, 3, 100), np.float32), np.zeros((5, 3, 50), np.float32)])   # wrong B


@pytest.mark.parametrize("path", ["auto", "layerwise"])
@pytest.mark.parametrize("B", [1, 3, 4])
def test_nll_k5000_single_and_few_images_match_oracle(B, path):
    """k=5000 log p(x) per image (get_NLL F:463-F:464 -> get_log_weights
    F:327-F:351) on the configs[1]/[2] architecture 784-200-200-100-100-50,
    Glorot weights with real encoder heads, the oracle's own noise injected:
    within the north_star's 0.05 nats per image.  path "auto" runs the kernel
    the NLL benchmark times -- the weight-ring kernel nring_kernel (bf16x3
    products, reading the injected [k][B][d] noise) -- checked by its own
    launch counter (3: ring chunks), not only the fused-kernel counter (1);
    "layerwise" the tiled-GEMM path."""
    O, spec, params, x, eps = _oracle_case(ARCH2, B, 5000, 500 + B)
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    m = _model(ARCH2, "IWAE", 5, kernel_path=path)
    m.set_weights(_split(O.flatten_params(spec, params).astype(np.float32), weight_shapes(m.dense)))
    n0, r0 = m._lib.iwae_debug_count(m._h, 1), m._lib.iwae_debug_count(m._h, 3)
    lp = m.log_px(x.astype(np.float32), 5000, eps=[e.astype(np.float32) for e in eps]).cpu().numpy()
    fused_launches = m._lib.iwae_debug_count(m._h, 1) - n0
    ring_chunks = m._lib.iwae_debug_count(m._h, 3) - r0
    assert (fused_launches > 0) == (path == "auto"), fused_launches
    assert (ring_chunks > 0) == (path == "auto"), ring_chunks
    assert ring_chunks == (fused_launches if path == "auto" else 0)      # every fused chunk on the ring kernel
    ref = O.log_px_per_image(params, spec, x, 5000, eps=eps, chunk=1000)
    assert lp.shape == (B,)
    assert np.max(np.abs(lp - ref)) <= 0.05, (lp, ref)


@pytest.mark.parametrize("path", ["auto", "fused"])
def test_graph_replays_equal_eager_over_steps_at_10k_rows(path):
    """B=200, k=50 (10,000 sample rows): five Philox train steps replayed from a
    captured graph equal the eager steps bit for bit -- for the train engine
    (auto) and for the fused row-block path, whose output layer switches to
    bf16x3 products at >= 8192 rows with its split copy refreshed inside the
    graph after every Adam step."""
    import torch
    rng = np.random.default_rng(43)
    xs = (rng.random((400, 784)) < 0.25).astype(np.float32)
    runs = []
    for graphs in (True, False):
        m = _model(ARCH2, "IWAE", 50, use_graphs=graphs, kernel_path=path)
        X = torch.from_numpy(xs).to(m.device)
        losses = [m.train_step(X[(i % 2) * 200:(i % 2) * 200 + 200])["IWAE"] for i in range(5)]
        runs.append((losses, _flat(m.get_weights())))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


def test_nll_k5000_ring_chunks_straddling_workgroups_match_oracle():
    """The bench-timed NLL kernel (nring_kernel) over chunks whose 128-row
    workgroups straddle images and whose samples split into two sample chunks
    (knobs: 3 images per chunk, 8192 rows -> 2730 + 2270 samples per image;
    the 4th image in a second image chunk), the oracle's noise injected:
    within 0.05 nats of the float64 oracle (F:463 -> F:327-F:351), and equal to
    the same call with one chunk per image within 1e-3 nats."""
    O, spec, params, x, eps = _oracle_case(ARCH2, 4, 5000, 901)
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    e32 = [e.astype(np.float32) for e in eps]
    m = _model(ARCH2, "IWAE", 5)
    m.set_weights(_split(O.flatten_params(spec, params).astype(np.float32), weight_shapes(m.dense)))
    lp_one = m.log_px(x.astype(np.float32), 5000, eps=e32).cpu().numpy()
    m.set_tuning("nll_imgs", 3)
    m.set_tuning("nll_rows", 8192)
    r0, n0 = m._lib.iwae_debug_count(m._h, 3), m._lib.iwae_debug_count(m._h, 1)
    lp = m.log_px(x.astype(np.float32), 5000, eps=e32).cpu().numpy()
    ring = m._lib.iwae_debug_count(m._h, 3) - r0
    fused = m._lib.iwae_debug_count(m._h, 1) - n0
    assert ring == fused == 4, (ring, fused)          # image chunks [0,3) and [3,4), two sample chunks each
    ref = O.log_px_per_image(params, spec, x, 5000, eps=eps, chunk=1000)
    assert np.max(np.abs(lp - ref)) <= 0.05, (lp, ref)
    assert np.max(np.abs(lp - lp_one)) <= 1e-3, (lp, lp_one)


@pytest.mark.parametrize("big", [60, 100, 512])
def test_alternating_split_and_single_split_output_jobs_leave_no_stale_rows(big):
    """the engine's forward splits the 784-wide Bernoulli layer over
    two jobs (columns 0 / 1 of the per-row sums) at <= 2048 sample rows; the
    single-split job (B=100) and the ring train forward (B=512) must clear
    column 1, or a large step after a small one adds stale partial sums to
    log p(x|h).  big -> 20 -> big on one handle equals big on a fresh handle,
    bit for bit (injected noise, forward_backward)."""
    rng = np.random.default_rng(77 + big)
    k = 50

    def case(B):
        x = (rng.random((B, 784)) < 0.2).astype(np.float32)
        eps = [rng.standard_normal((k, B, d)).astype(np.float32) for d in (100, 50)]
        return x, eps

    (xb, eb), (xs, es) = case(big), case(20)
    import torch
    from iwae_replication_project_amd.flexible_iwae import loss_config

    def fb(m, x, eps):
        lc = loss_config("IWAE", k)
        xd = m._x(x)
        arr, n, keep = m._eps(eps, x.shape[0], k)
        m._forward_backward(lc, xd, x.shape[0], arr, n)
        m._stream.synchronize()
        return float(m._loss_buf.item()), _flat(m.get_gradients())

    a = _model(ARCH2, "IWAE", k)
    b = _model(ARCH2, "IWAE", k)
    b.set_weights(a.get_weights())
    fb(a, xb, eb)
    fb(a, xs, es)
    la, ga = fb(a, xb, eb)
    lb, gb = fb(b, xb, eb)
    torch.cuda.synchronize()
    assert la == lb, (la, lb)
    assert np.array_equal(ga, gb)


@pytest.mark.parametrize("B,n", [(20, 11), (20, 40), (7, 3), (64, 9), (512, 3)])
def test_train_steps_equal_single_step_calls(B, n):
    """fit's batch loop as one call (iwae_train_steps: graphs of up to 32
    captured steps, each re-pointed at its own batch) equals n train_step
    calls -- captured one step per graph, and eager -- bit for bit: per-step
    losses, the final weights and Adam state (same seed, same Philox stream).
    Shapes: the bench's B=20 (11 steps: one graph; 40 = 32 + 8: two graphs of
    different length), a ragged 7, 64 images (image-row jobs; the input GEMM
    reads the caller's x) and the large-batch leg's 512 (ring kernels)."""
    import torch
    rng = np.random.default_rng(11 + B + n)
    xs = (rng.random((n * B + 5, 784)) < 0.25).astype(np.float32)
    runs = []
    for mode in ("steps", "calls", "eager"):
        m = _model(ARCH2, "IWAE", 50, use_graphs=mode != "eager")
        X = torch.from_numpy(xs).to(m.device)
        if mode == "steps":
            # twice over the same batches: the second call replays the graphs it captured
            l1 = m.train_steps(X[:n * B], B)
            l2 = m.train_steps(X[5:5 + n * B], B)          # shifted batches: every input launch re-pointed
            losses = list(l1) + list(l2)
        else:
            losses = [m.train_step(X[i * B:(i + 1) * B])["IWAE"] for i in range(n)]
            losses += [m.train_step(X[5 + i * B:5 + (i + 1) * B])["IWAE"] for i in range(n)]
        mm, vv, st = m.get_optimizer_state()
        runs.append((np.asarray(losses, np.float32), _flat(m.get_weights()), mm, st))
    for r in runs[1:]:
        np.testing.assert_array_equal(runs[0][0], r[0])
        np.testing.assert_array_equal(runs[0][1], r[1])
        np.testing.assert_array_equal(runs[0][2], r[2])
        assert runs[0][3] == r[3] == 2 * n


@pytest.mark.parametrize("B,n", [(20, 20), (20, 45), (512, 3)])
def test_prepared_train_steps_capture_nothing_more_and_equal_unprepared(B, n):
    """iwae_train_steps_prepare captures the graphs of a later train_steps call
    (one per chunk length: 45 = 32 + 13 gives two) without running anything:
    weights, Adam step and an evaluation on injected noise are those of an
    unprepared model; the call then captures nothing (capture counter, id 7)
    and its losses, weights and Adam state equal the unprepared run bit for
    bit.  bench.py relies on this to time steady-state replays only."""
    import torch
    rng = np.random.default_rng(31 + B + n)
    xs = (rng.random((n * B, 784)) < 0.25).astype(np.float32)
    xe = xs[:4]
    eps = [rng.standard_normal((5, 4, d)).astype(np.float32) for d in ARCH2[2]]
    runs = []
    for prep in (False, True):
        m = _model(ARCH2, "IWAE", 50)
        X = torch.from_numpy(xs).to(m.device)
        w0 = _flat(m.get_weights())
        if prep:
            c0 = m.graph_captures()
            m.prepare_train_steps(X, B)
            lens = ({32} if n >= 32 else set()) | ({n % 32} if n % 32 else set())
            assert m.graph_captures() - c0 == len(lens), (lens, m.graph_captures() - c0)
            np.testing.assert_array_equal(_flat(m.get_weights()), w0)
            assert m.get_optimizer_state()[2] == 0
        lw = m.get_log_weights(xe, 5, eps=eps).cpu().numpy()
        c1 = m.graph_captures()
        losses = m.train_steps(X, B)
        if prep:
            assert m.graph_captures() == c1
        mm, vv, st = m.get_optimizer_state()
        runs.append((lw, np.asarray(losses, np.float32), _flat(m.get_weights()), mm, st))
    for a, b in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(a, b)
    assert runs[0][4] == n


@pytest.mark.parametrize("B", [64, 512])
def test_input_gemm_on_the_callers_x_equals_the_staged_copy(B):
    """Above the few-row launches' 32 images the engine step's input Dense is
    a split-K GEMM.  It reads the caller's x with a virtual ones column at
    x_dim (the bias row of W_aug), and its column-0 workgroups fill the padded
    x_in that the later launches read (ring-forward pixels, the input layer's
    weight gradient).  Knob x_direct 0 stages x into x_in with a copy first:
    both give the same losses, weights and Adam state bit for bit, over graph
    replays with a moving batch and eagerly."""
    import torch
    rng = np.random.default_rng(5 + B)
    xs = (rng.random((3 * B + 3, 784)) < 0.3).astype(np.float32)
    runs = []
    for direct in (1, 0):
        for graphs in (True, False):
            m = _model(ARCH2, "IWAE", 50, use_graphs=graphs, tuning={"x_direct": direct})
            X = torch.from_numpy(xs).to(m.device)
            losses = [m.train_step(X[i * B + i:(i + 1) * B + i])["IWAE"] for i in range(3)]
            mm, vv, st = m.get_optimizer_state()
            runs.append((np.asarray(losses, np.float32), _flat(m.get_weights()), mm, vv))
    for r in runs[1:]:
        for u, v in zip(runs[0], r):
            np.testing.assert_array_equal(u, v)


def test_train_steps_losses_copy_node_repointed_and_null():
    """A multi-step graph's last node copies its losses to the caller's array,
    re-pointed per call (hipGraphExecMemcpyNodeSetParams1D).  Calls with no
    loss array (NULL: the copy goes to a sink), with one array and with
    another array replay the same graphs (45 steps: 32 + 13) and leave the
    same weights as a model whose every call passed one array; each array
    receives exactly its call's losses."""
    import ctypes
    import torch
    from iwae_replication_project_amd import _lib
    rng = np.random.default_rng(77)
    B, n = 20, 45
    xs = (rng.random((3 * n * B, 784)) < 0.3).astype(np.float32)
    res = []
    for mode in ("arrays", "mixed"):
        m = _model(ARCH2, "IWAE", 50)
        X = torch.from_numpy(xs).to(m.device)
        outs = []
        for c in range(3):
            xc = X[c * n * B:(c + 1) * n * B]
            if mode == "mixed" and c == 0:
                m._call(m._lib.iwae_train_steps(m._h, m._lc(), _lib.fptr(xc), B, n,
                                                ctypes.cast(None, _lib.FP)))
                m._stream.synchronize()
                outs.append(None)
            else:
                outs.append(np.asarray(m.train_steps(xc, B), np.float32))
        res.append((outs, _flat(m.get_weights())))
    (a_outs, a_w), (b_outs, b_w) = res
    np.testing.assert_array_equal(a_w, b_w)
    for c in (1, 2):
        np.testing.assert_array_equal(a_outs[c], b_outs[c])
    assert np.isfinite(a_outs[0]).all() and not np.array_equal(a_outs[1], a_outs[2])
