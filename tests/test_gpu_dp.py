"""Multi-rank paths through the HIP library, two processes sharing one GPU
(gloo carries the collectives here; the multi-GPU bench uses RCCL):

* data-parallel train step: replicas built from DIFFERENT seeds start from
  rank 0's weights and Adam state (broadcast) and end bitwise identical; with
  unequal shards (4 + 3 images) the step equals one full-batch step on the
  same injected noise (each rank's loss is its local batch mean, F:369, so
  the gradients are merged as sum_r B_r g_r / sum_r B_r);
* device noise differs per rank (F:59 / F:68 draw iid samples): the ranks'
  local losses on the same batch differ;
* sample-sharded k-sample NLL: each rank's partials come from its own noise
  stream; a single process reproducing the two streams gets the same merged
  estimate, and it differs from the duplicated-noise merge;
* the library-owned RCCL communicator (iwae_dp_init with a unique id) at one
  rank: the graph-captured forward_backward -> ncclAllReduce -> Adam step."""
import math
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ARCH = ([64, 32], [32, 64], [32, 16], [32, 784])
B, K = 7, 6


def _data():
    rng = np.random.default_rng(21)
    mean = rng.uniform(0.02, 0.4, 784)
    x = (rng.random((B, 784)) < mean).astype(np.float32)
    eps = [rng.standard_normal((K, B, d)).astype(np.float32) for d in ARCH[2]]
    return mean, x, eps


def _model(mean, seed=5, **kw):
    from iwae_replication_project_amd import Adam, Flexible_Model
    m = Flexible_Model(*ARCH, dataset_bias=mean, loss_function="IWAE", k=K, seed=seed, **kw)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    return m


def _flat(ws):
    return np.concatenate([np.asarray(w).ravel() for w in ws])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(fn, world=2, timeout=150):
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(fn, r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=timeout) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    return out


def _rank_main(fn, rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:          # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------ rank bodies
def _dp_injected(rank, world):
    from iwae_replication_project_amd import distributed as D
    mean, x, eps = _data()
    m = _model(mean, seed=100 + rank)           # different initial weights per rank
    D.enable_data_parallel(m)
    w_start = _flat(m.get_weights())
    lo, hi = D.shard_range(B, rank, world)      # 4 + 3 images: unequal shards
    m.train_step(x[lo:hi], eps=[e[:, lo:hi] for e in eps])
    mm, vv, t = m.get_optimizer_state()
    return w_start, _flat(m.get_weights()), mm, vv, t


def _dp_philox(rank, world):
    from iwae_replication_project_amd import distributed as D
    mean, x, _ = _data()
    m = _model(mean, seed=200 + rank)
    D.enable_data_parallel(m)
    losses = [m.train_step(x)["IWAE"] for _ in range(3)]     # same batch on both ranks
    return losses, _flat(m.get_weights())


def _nll_sample(rank, world):
    from iwae_replication_project_amd import distributed as D
    mean, x, _ = _data()
    m = _model(mean, seed=9)
    nll, lp = D.sharded_nll(m, x, k=1000, mode="sample")
    return nll, lp.cpu().numpy()


# ------------------------------------------------------------------ tests
def test_dp_unequal_shards_different_seeds_equal_full_batch_step():
    out = _launch(_dp_injected)
    mean, x, eps = _data()
    m = _model(mean, seed=100)                  # rank 0's initial weights
    w0 = _flat(m.get_weights())
    m.train_step(x, eps=eps)
    ref = _flat(m.get_weights())
    rm, rv, rt = m.get_optimizer_state()
    for r in (0, 1):
        w_start, w_end, mm, vv, t = out[r]
        np.testing.assert_array_equal(w_start, w0)          # broadcast from rank 0
        assert np.abs(w_end - w0).max() > 1e-4               # the step moved the weights
        np.testing.assert_allclose(w_end, ref, atol=6e-5)
        # Adam's m = (1 - b1) g: the merged gradient sums the rows in another grouping
        assert np.linalg.norm(mm - rm) <= 1e-4 * np.linalg.norm(rm), np.linalg.norm(mm - rm)
        assert t == rt == 1
    np.testing.assert_array_equal(out[0][1], out[1][1])     # replicas bitwise identical
    np.testing.assert_array_equal(out[0][2], out[1][2])
    np.testing.assert_array_equal(out[0][3], out[1][3])


def test_dp_philox_noise_is_independent_per_rank_and_replicas_stay_identical():
    out = _launch(_dp_philox)
    (l0, w0), (l1, w1) = out[0], out[1]
    assert all(a != b for a, b in zip(l0, l1))      # same batch, same weights, different noise
    np.testing.assert_array_equal(w0, w1)


def test_sample_sharded_nll_uses_disjoint_noise_streams():
    out = _launch(_nll_sample)
    import torch
    mean, x, _ = _data()
    m = _model(mean, seed=9)
    parts = {}
    for stream in (0, 1):
        m.set_noise_stream(stream)
        mm, ss = m.log_px_partials(x, 500)
        parts[stream] = (mm.double().cpu(), ss.double().cpu())

    def merge(a, b):
        M = torch.maximum(a[0], b[0])
        S = a[1] * torch.exp(a[0] - M) + b[1] * torch.exp(b[0] - M)
        return (M + torch.log(S) - math.log(1000)).numpy()

    ref = merge(parts[0], parts[1])
    dup = merge(parts[0], parts[0])
    for r in (0, 1):
        np.testing.assert_allclose(out[r][1], ref, rtol=0, atol=1e-4)
    assert np.abs(ref - dup).max() > 1e-3                  # the streams really differ
    assert not np.allclose(parts[0][0].numpy(), parts[1][0].numpy())


def test_library_rccl_communicator_single_rank_step():
    """iwae_dp_init with an RCCL unique id at world size 1: the train step is
    forward_backward -> ncclAllReduce(n + 4 floats) -> Adam with scale
    1 / B_global, captured in a hipGraph; it matches the plain step."""
    from iwae_replication_project_amd import distributed as D
    mean, x, eps = _data()
    runs = []
    for dp in (False, True):
        m = _model(mean, seed=5)
        if dp:
            d = D.enable_data_parallel(m, comm="library")
            assert d.comm == "library"
        losses = [m.train_step(x)["IWAE"] for _ in range(3)]              # Philox, graphs
        losses.append(m.train_step(x, eps=eps)["IWAE"])                   # eager, injected
        runs.append((losses, _flat(m.get_weights()), _flat(m.get_gradients())))
    (la, wa, ga), (lb, wb, gb) = runs
    np.testing.assert_allclose(lb, la, rtol=1e-6)
    np.testing.assert_allclose(wb, wa, atol=1e-6)
    # B * g / B against g: rounding only, compounded over the three earlier
    # steps' weight differences (north_star: 1e-4 relative)
    assert np.linalg.norm(gb - ga) <= 1e-4 * np.linalg.norm(ga), np.linalg.norm(gb - ga)


def test_library_rccl_train_steps_equal_single_step_calls():
    """With the library communicator, train_steps captures the data-parallel
    step (gradient pass, in-graph ncclAllReduce buckets, Adam) as multi-step
    graphs (45 steps: graphs of 32 and 13); losses, weights and Adam state equal
    45 train_step calls (one graph each) bit for bit, and the prepared call
    captures nothing.  World size 1: this pool's boxes have one GPU."""
    import torch
    from iwae_replication_project_amd import distributed as D
    mean, _, _ = _data()
    rng = np.random.default_rng(77)
    n = 45
    xs = (rng.random((n * B, 784)) < mean).astype(np.float32)
    runs = []
    for mode in ("steps", "calls"):
        m = _model(mean, seed=5)
        D.enable_data_parallel(m, comm="library")
        X = torch.from_numpy(xs).to(m.device)
        if mode == "steps":
            m.prepare_train_steps(X, B)
            c0 = m.graph_captures()
            losses = list(m.train_steps(X, B))
            assert m.graph_captures() == c0
        else:
            losses = [m.train_step(X[i * B:(i + 1) * B])["IWAE"] for i in range(n)]
        mm, vv, st = m.get_optimizer_state()
        runs.append((np.asarray(losses, np.float32), _flat(m.get_weights()), mm, vv, st))
    for a, b in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(a, b)
    assert runs[0][4] == n


def _dp_train_steps(rank, world):
    import torch
    from iwae_replication_project_amd import distributed as D
    mean, _, _ = _data()
    rng = np.random.default_rng(78)
    n = 6
    xs = (rng.random((n * 2 * B, 784)) < mean).astype(np.float32)
    out = []
    for mode in ("steps", "calls"):
        m = _model(mean, seed=300 + rank)
        D.enable_data_parallel(m)
        # this rank's half of every global batch of 2B images
        xl = np.concatenate([xs[(2 * i + rank) * B:(2 * i + rank + 1) * B] for i in range(n)])
        X = torch.from_numpy(xl).to(m.device)
        if mode == "steps":
            losses = list(m.train_steps(X, B))
        else:
            losses = [m.train_step(X[i * B:(i + 1) * B])["IWAE"] for i in range(n)]
        mm, vv, st = m.get_optimizer_state()
        out.append((np.asarray(losses, np.float32), _flat(m.get_weights()), mm, vv, st))
    return out


def test_dp_train_steps_equal_per_step_dp_calls():
    """Two ranks (gloo, torch-reduced gradient buffer): fit's loop through
    train_steps equals per-step data-parallel train_step calls bit for bit on
    every rank, and the replicas stay identical."""
    out = _launch(_dp_train_steps)
    for r in (0, 1):
        steps, calls = out[r]
        for a, b in zip(steps, calls):
            np.testing.assert_array_equal(a, b)
        assert steps[4] == 6
    np.testing.assert_array_equal(out[0][0][1], out[1][0][1])


def _snr(rank, world):
    mean, x, _ = _data()
    from iwae_replication_project_amd import Flexible_Model
    m = Flexible_Model(*ARCH, dataset_bias=mean, loss_function="CIWAE", k=K, beta=0.5, seed=5)
    snr, info = m.get_gradient_snr(x, R=24, seed=123)
    return _flat(snr), info["R"]


def test_gradient_snr_split_over_two_ranks_equals_two_streams():
    """get_gradient_snr under 2 ranks (configs[3]'s harness, CIWAE: two draws
    per estimate): each rank draws R/2 estimates from its own noise stream and
    the moments are summed; a single process running both streams in turn
    gets the same SNR."""
    out = _launch(_snr)
    mean, x, _ = _data()
    from iwae_replication_project_amd import Flexible_Model
    b = Flexible_Model(*ARCH, dataset_bias=mean, loss_function="CIWAE", k=K, beta=0.5, seed=5)
    b.set_seed(123)
    xd = b._x(x)
    lc = b._lc()
    gs = []
    for stream in (0, 1):
        b.set_noise_stream(stream)
        for _ in range(12):
            b._forward_backward(lc, xd, xd.shape[0], None, 0)
            gs.append(_flat(b.get_gradients()).astype(np.float64))
    G = np.stack(gs)
    mu = G.mean(0)
    sd = np.sqrt(np.maximum((G * G).mean(0) - mu * mu, 0.0))
    ref = np.where(sd > 0, np.abs(mu) / np.where(sd > 0, sd, 1.0), np.inf)
    # SNR <= 100: larger ratios come from f32 moment cancellation on the device
    fin = np.isfinite(ref) & (sd > 1e-6 * np.abs(mu).max()) & (ref < 100)
    for r in (0, 1):
        got, R = out[r]
        assert R == 24
        np.testing.assert_allclose(got[fin], ref[fin], rtol=2e-3, atol=1e-4)
    np.testing.assert_array_equal(out[0][0], out[1][0])
