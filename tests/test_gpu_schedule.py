"""The reference's LR-stage training driver (E:73-E:97, data.train_schedule)
on the real model, and the per-stream noise counters it relies on.

* Injected noise: train_schedule's stages (E:76: lr_i = 1e-4 round(10^(1 -
  (i-1)/7), 1)) drive the device Adam; the whole trajectory (losses, weights,
  Adam step) tracks the float64 oracle's Keras Adam with each stage's
  learning rate (E:36-E:40).
* Graph-replayed Philox steps: the learning rate pushed between stages reaches
  the captured step (lr lives in device state, not in the graph): each
  stage's update equals Adam at that stage's rate applied to the gradient the
  device used (iwae_get_grads), from the previous weights and moments.
* Noise streams: re-selecting the current stream (what sharded_nll does on
  every call under data parallelism) does not restart its counter, so the
  next step draws fresh noise; switching away and back continues the stream.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-4


def _flat(ws):
    return np.concatenate([np.asarray(w, np.float64).ravel() for w in ws])


def test_lr_stages_track_oracle_adam_with_injected_noise():
    from oracle import iwae_oracle as O
    from iwae_replication_project_amd import Adam, Flexible_Model
    from iwae_replication_project_amd import data as D
    from iwae_replication_project_amd.flexible_iwae import _split, weight_shapes
    he, hd, le, ld = [64, 32], [32, 64], [32, 16], [32, 784]
    B, k, stages = 16, 8, 3
    rng = np.random.default_rng(81)
    mean = rng.uniform(0.02, 0.4, 784)
    spec = O.ModelSpec(he, hd, le, ld)
    params = O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(mean))
    params = {n: [w.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)]
              for n, (w, b) in params.items()}
    x = (rng.random((B, 784)) < mean).astype(np.float64)
    epss = [[e.astype(np.float32).astype(np.float64) for e in O.draw_eps(spec, k, B, rng)] for _ in range(2 * stages)]

    m = Flexible_Model(he, hd, le, ld, dataset_bias=mean, loss_function="IWAE", k=k, seed=1, use_graphs=True)
    m.set_weights(_split(O.flatten_params(spec, params).astype(np.float32), weight_shapes(m.dense)))
    m.compile(Adam(learning_rate=0.5, epsilon=1e-4))        # the driver sets each stage's rate itself
    feed = iter(epss)
    losses = []

    def fit(xs, epochs=1, batch_size=100, verbose=0):        # E:82 with the test's injected noise
        for _ in range(epochs):
            losses.append(m.train_step(xs, eps=[e.astype(np.float32) for e in next(feed)])["IWAE"])
    m.fit = fit
    seen = []
    D.train_schedule(m, x.astype(np.float32), stages=stages, batch_size=B, passes=lambda i: 2 if i == 2 else 1,
                     on_stage=lambda i, tot, res: seen.append((i, tot, m.optimizer.learning_rate)))
    assert [s[:2] for s in seen] == [(1, 1), (2, 3), (3, 4)]
    np.testing.assert_allclose([s[2] for s in seen], [D.stage_learning_rate(i) for i in (1, 2, 3)], rtol=1e-12)
    np.testing.assert_allclose([s[2] for s in seen], [1e-3, 7.2e-4, 5.2e-4], rtol=1e-12)

    opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
    ref = []
    step_lr = [D.stage_learning_rate(1), D.stage_learning_rate(2), D.stage_learning_rate(2),
               D.stage_learning_rate(3)]
    for s, lr in enumerate(step_lr):
        opt.lr = lr
        l, params, _ = O.train_step(params, spec, x, epss[s], "IWAE", k, opt)
        ref.append(l)
    assert len(losses) == 4
    np.testing.assert_allclose(losses, ref, rtol=REL)
    np.testing.assert_allclose(_flat(m.get_weights()), O.flatten_params(spec, params), atol=2e-5)
    assert m.get_optimizer_state()[2] == 4


def test_lr_stages_reach_graph_replayed_steps():
    from oracle import iwae_oracle as O
    from iwae_replication_project_amd import Adam, Flexible_Model
    from iwae_replication_project_amd import data as D
    rng = np.random.default_rng(82)
    x = (rng.random((20, 784)) < 0.15).astype(np.float32)
    m = Flexible_Model([200, 100], [100, 200], [100, 50], [100, 784], dataset_bias=None, loss_function="IWAE",
                       k=50, seed=3, use_graphs=True)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    for _ in range(2):                      # capture the step's graph before the schedule starts
        m.train_step(x)
    checked = []

    def on_stage(i, tot, res):
        checked.append(i)

    prev = {}

    def fit(xs, epochs=1, batch_size=100, verbose=0):
        for _ in range(epochs):
            w0 = _flat(m.get_weights())
            m0, v0, t0 = m.get_optimizer_state()
            m.train_step(xs)                    # Philox noise: graph replay
            g = _flat(m.get_gradients())
            w1 = _flat(m.get_weights())
            opt = O.Adam(m.optimizer.learning_rate, 0.9, 0.999, 1e-4)
            opt.m, opt.v, opt.t = m0.astype(np.float64), v0.astype(np.float64), int(t0)
            np.testing.assert_allclose(w1, opt.apply(w0, g), atol=2e-6)
            prev[m.optimizer.learning_rate] = prev.get(m.optimizer.learning_rate, 0) + 1
    m.fit = fit
    D.train_schedule(m, x, stages=3, batch_size=20, passes=lambda i: 1, on_stage=on_stage)
    assert checked == [1, 2, 3]
    assert sorted(prev) == sorted(D.stage_learning_rate(i) for i in (1, 2, 3))


def test_reselecting_the_noise_stream_keeps_drawing_fresh_noise():
    from iwae_replication_project_amd import Flexible_Model
    rng = np.random.default_rng(83)
    x = (rng.random((10, 784)) < 0.15).astype(np.float32)

    def fb(m):
        xd = m._x(x)
        m._forward_backward(m._lc(), xd, xd.shape[0], None, 0)
        m._stream.synchronize()
        return float(m._loss_buf.item())

    m = Flexible_Model([64], [64], [16], [784], dataset_bias=None, loss_function="IWAE", k=5, seed=7)
    m.set_noise_stream(1)
    la = fb(m)
    m.log_px(x[:2], 100)                   # an evaluation in between (draws noise too)
    m.set_noise_stream(1)                  # what sharded_nll does under data parallelism: a no-op now
    lb = fb(m)
    assert la != lb
    m.set_noise_stream(2)
    lc2 = fb(m)
    m.set_noise_stream(1)                  # back to stream 1: continues, never replays
    lc1 = fb(m)
    assert len({la, lb, lc2, lc1}) == 4
    # per-stream reproducibility: a fresh model with the same seed replays stream 1 from its start
    f = Flexible_Model([64], [64], [16], [784], dataset_bias=None, loss_function="IWAE", k=5, seed=7)
    f.set_weights(m.get_weights())
    f.set_noise_stream(1)
    assert fb(f) == la
    f.set_noise_stream(3)
    f.set_seed(7)                          # restarts every stream (stream 3 stays selected)
    f.set_noise_stream(2)
    assert fb(f) == lc2
