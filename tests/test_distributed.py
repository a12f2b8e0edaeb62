"""Multi-process (world_size 2, gloo on CPU) tests of the sharding logic used
by the multi-GPU paths: image sharding, the cross-rank log-sum-exp merge of
NLL partials, and gradient averaging for data parallelism.  Compute inside the
ranks comes from the oracle (test infrastructure); what is under test is
iwae_replication_project_amd.distributed."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:          # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


def _model():
    from oracle import iwae_oracle as O
    rng = np.random.default_rng(0)
    spec = O.ModelSpec([16, 8], [8, 16], [8, 4], [8, 32], x_dim=32)
    params = O.glorot_init(spec, rng, out_bias=rng.normal(size=32) * 0.3)
    x = (rng.random((7, 32)) < 0.3).astype(np.float64)
    eps = O.draw_eps(spec, 40, 7, rng)
    return O, spec, params, x, eps


def nll_sample_shard(rank, world):
    """Each rank evaluates its k-range of every image; merge partials."""
    from iwae_replication_project_amd import distributed as D
    O, spec, params, x, eps = _model()
    k = eps[0].shape[0]
    lo, hi = D.shard_range(k, rank, world)
    lw = O.forward(params, spec, x, [e[lo:hi] for e in eps])["lw"]
    m = torch.tensor(lw.max(0))
    s = torch.tensor(np.exp(lw - lw.max(0)).sum(0))
    M, S = D.merge_lse_partials(m, s)
    merged = (M + torch.log(S) - math.log(k)).numpy()
    return merged.tolist()


def nll_image_shard(rank, world):
    from iwae_replication_project_amd import distributed as D
    O, spec, params, x, eps = _model()
    lo, hi = D.shard_range(x.shape[0], rank, world)
    lp = O.L_k_per_image(O.forward(params, spec, x[lo:hi], [e[:, lo:hi] for e in eps])["lw"])
    tot = torch.tensor([lp.sum(), float(hi - lo)], dtype=torch.float64)
    dist.all_reduce(tot)
    return float(-(tot[0] / tot[1]))


def dp_grads(rank, world):
    """Per-rank gradient of the batch-mean VAE loss on its shard, averaged
    across ranks == gradient of the full-batch loss (equal shards)."""
    from iwae_replication_project_amd import distributed as D
    O, spec, params, x, eps = _model()
    x, eps = x[:6], [e[:, :6] for e in eps]
    lo, hi = D.shard_range(6, rank, world)
    _, g = O.objective_and_grads(params, spec, x[lo:hi], [e[:, lo:hi] for e in eps], "VAE", eps[0].shape[0])
    t = torch.tensor(O.flatten_params(spec, g))
    D.allreduce_mean_(t)
    return t.numpy().tolist()


def test_shard_range_partitions_everything():
    from iwae_replication_project_amd.distributed import shard_range
    for n in (0, 1, 7, 10000, 10001):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1


def test_sample_sharded_nll_merge_equals_single_process():
    out = spawn(nll_sample_shard)
    O, spec, params, x, eps = _model()
    ref = O.L_k_per_image(O.forward(params, spec, x, eps)["lw"])
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        np.testing.assert_allclose(out[r], ref, rtol=1e-10)


def test_image_sharded_nll_equals_single_process():
    out = spawn(nll_image_shard)
    O, spec, params, x, eps = _model()
    ref = -np.mean(O.L_k_per_image(O.forward(params, spec, x, eps)["lw"]))
    assert out[0] == pytest.approx(ref, rel=1e-12) and out[1] == pytest.approx(ref, rel=1e-12)


def test_data_parallel_gradient_average_equals_full_batch():
    out = spawn(dp_grads)
    O, spec, params, x, eps = _model()
    _, g = O.objective_and_grads(params, spec, x[:6], [e[:, :6] for e in eps], "VAE", eps[0].shape[0])
    ref = O.flatten_params(spec, g)
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        np.testing.assert_allclose(out[r], ref, rtol=1e-10, atol=1e-13)


def dp_grads_unequal(rank, world):
    """Unequal shards (4 + 3 images): the weighted merge sum_r B_r g_r / sum_r B_r
    (what the library's data-parallel step computes from one all-reduce of the
    gradient buffer plus its batch-size tail) equals the full-batch gradient."""
    from iwae_replication_project_amd import distributed as D
    O, spec, params, x, eps = _model()
    lo, hi = D.shard_range(7, rank, world)
    _, g = O.objective_and_grads(params, spec, x[lo:hi], [e[:, lo:hi] for e in eps], "IWAE", eps[0].shape[0])
    t = torch.tensor(np.concatenate([O.flatten_params(spec, g), [0.0]]))
    return D.weighted_grad_merge_(t, hi - lo).numpy().tolist()


def test_data_parallel_weighted_merge_unequal_shards_equals_full_batch():
    out = spawn(dp_grads_unequal)
    O, spec, params, x, eps = _model()
    _, g = O.objective_and_grads(params, spec, x, eps, "IWAE", eps[0].shape[0])
    ref = O.flatten_params(spec, g)
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        np.testing.assert_allclose(out[r], ref, rtol=1e-10, atol=1e-13)
    # the unweighted 1/world average is wrong for unequal shards
    lo = []
    for r in (0, 1):
        a, b = (0, 4) if r == 0 else (4, 7)
        _, gr = O.objective_and_grads(params, spec, x[a:b], [e[:, a:b] for e in eps], "IWAE", eps[0].shape[0])
        lo.append(O.flatten_params(spec, gr))
    assert np.abs((lo[0] + lo[1]) / 2 - ref).max() > 1e-6
