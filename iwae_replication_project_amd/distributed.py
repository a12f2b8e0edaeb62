"""Multi-GPU paths: one process per GPU, torch.distributed over RCCL/xGMI.

* Training: data parallel.  Every rank runs the
  full train step on its own batch shard with its own noise stream (the
  Philox key is derived from (seed, rank), so the iid draws of F:59 / F:68 hold
  across ranks).  Parameters, Adam moments and the Adam step are broadcast
  from rank 0 when data parallelism is enabled, so replicas built from
  different seeds start identical.  Each rank's loss is its local batch mean
  (F:369); forward_backward writes B_local * g plus B_local into the gradient
  buffer's tail, so ONE sum all-reduce of n + 4 floats yields sum_r B_r g_r
  and B_global, and Adam steps with the exact global batch-mean gradient
  (unequal shards included).  Two ways to reduce:
    - "library": the HIP library owns an RCCL communicator (iwae_dp_init with
      a unique id rank 0 draws and torch.distributed broadcasts); the train
      step is forward_backward -> ncclAllReduce -> Adam on the library's
      stream, captured in one hipGraph;
    - "torch": the library fills a torch-owned gradient buffer, torch's
      all_reduce sums it, the library applies Adam (any backend, e.g. gloo).
  The reference has no distributed code at all.
* k=5000 NLL (config C3): sharded by test image (no data-path collective, one
  scalar all-reduce for the mean) or by sample chunk (each rank draws
  k/world independent samples of every image from its own noise stream;
  per-image log-sum-exp partials (m, s) are all-gathered and merged:
  M = max m, S = sum s*exp(m-M), log p(x) = M + log S - log k).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(n, rank, world_size):
    """Contiguous balanced split of n items: the [lo, hi) of this rank."""
    base, rem = divmod(n, world_size)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def allreduce_mean_(t, group=None):
    """In-place mean over ranks (sum all-reduce then 1/world)."""
    _, w = world(group)
    if w > 1:
        dist.all_reduce(t, group=group)
        t.div_(w)
    return t


def weighted_grad_merge_(t, n_local, group=None):
    """The data-parallel gradient merge on a flat buffer t = [g_local..., pad]:
    t[:-1] *= n_local, t[-1] = n_local, sum all-reduce, then divide by the
    reduced total.  Gives sum_r n_r g_r / sum_r n_r = the gradient of the
    global batch mean for any shard sizes (F:369's mean over the batch)."""
    t[:-1].mul_(float(n_local))
    t[-1] = float(n_local)
    _, w = world(group)
    if w > 1:
        dist.all_reduce(t, group=group)
    t[:-1].div_(t[-1])
    return t[:-1]


def merge_lse_partials(m, s, group=None):
    """Merge per-rank log-sum-exp partials of the same images.
    m, s: [N] tensors (max and sum of exp(lw - m)).  Returns merged (M, S)."""
    _, w = world(group)
    if w == 1:
        return m, s
    ms = torch.stack([m, s])
    bufs = [torch.empty_like(ms) for _ in range(w)]
    dist.all_gather(bufs, ms, group=group)
    allm = torch.stack([b[0] for b in bufs])
    alls = torch.stack([b[1] for b in bufs])
    M = allm.max(dim=0).values
    S = (alls * torch.exp(allm - M)).sum(dim=0)
    return M, S


def broadcast_model_state(model, group=None, src=0):
    """Parameters, Adam moments and step from rank `src` to every rank (one-time,
    host-staged; the library path uses iwae_dp_broadcast_state instead)."""
    rank, w = world(group)
    if w == 1:
        return
    dev = model.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    flat = np.concatenate([np.asarray(a, np.float32).ravel() for a in model.get_weights()])
    m, v, step = model.get_optimizer_state()
    buf = torch.from_numpy(np.concatenate([flat, m, v, np.array([float(step)], np.float32)])).to(dev)
    dist.broadcast(buf, src=src, group=group)
    b = buf.cpu().numpy()
    n = flat.size
    from .flexible_iwae import _split, weight_shapes
    model.set_weights(_split(b[:n].copy(), weight_shapes(model.dense)))
    model.set_optimizer_state(b[n:2 * n], b[2 * n:3 * n], int(round(float(b[3 * n]))))


class DataParallel:
    """Data-parallel train step of one rank (see the module docstring)."""

    def __init__(self, model, group=None, comm="auto"):
        self.group = group
        self.rank, self.world = world(group)
        if comm == "auto":
            comm = "library" if (self.world > 1 and dist.get_backend(group) == "nccl") else "torch"
        if comm not in ("library", "torch"):
            raise ValueError("comm must be 'auto', 'library' or 'torch'")
        self.comm = comm
        lib, h = model._lib, model._h
        if comm == "library":
            if group is not None and group is not dist.group.WORLD:
                raise ValueError("the library communicator spans the default process group only")
            uid = torch.zeros(128, dtype=torch.uint8)
            if self.rank == 0:
                raw = (ctypes.c_ubyte * 128)()
                model._call(lib.iwae_dp_unique_id(ctypes.cast(raw, ctypes.c_void_p)))
                uid = torch.tensor(list(bytes(raw)), dtype=torch.uint8)
            if self.world > 1:
                dev = model.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
                uid = uid.to(dev)
                dist.broadcast(uid, src=0, group=group)
                uid = uid.cpu()
            raw = (ctypes.c_ubyte * 128)(*uid.tolist())
            model._call(lib.iwae_dp_init(h, self.rank, self.world, ctypes.cast(raw, ctypes.c_void_p)))
            model._call(lib.iwae_dp_broadcast_state(h))
            self.grad = None
        else:
            broadcast_model_state(model, group)
            model._call(lib.iwae_dp_init(h, self.rank, self.world, None))
            g = _lib.FP()
            n = ctypes.c_longlong(0)
            model._call(lib.iwae_grad_buffer(h, ctypes.byref(g), ctypes.byref(n)))
            self.n = int(n.value)
            with torch.cuda.stream(model._stream):
                # n gradient floats + the batch-size tail (4 floats keep the float4 layout)
                self.grad = torch.zeros(self.n + 4, device=model.device)
            model._call(lib.iwae_bind_grad_buffer(h, _lib.fptr(self.grad), self.n + 4))

    def step(self, model, lc, xd, B, arr, n):
        if self.comm == "library":
            model._call(model._lib.iwae_train_step(model._h, lc, _lib.fptr(xd), B, arr, n,
                                                   _lib.fptr(model._loss_buf)))
            return
        model._forward_backward(lc, xd, B, arr, n)     # grad = B_local * g, tail = B_local
        if self.world > 1:
            with torch.cuda.stream(model._stream):
                dist.all_reduce(self.grad, group=self.group)
        # scale 1 / sum_r B_r, read on the device (one rank: the plain local mean)
        model._apply_adam(0.0 if self.world > 1 else 1.0)


def enable_data_parallel(model, group=None, comm="auto"):
    model._dp = DataParallel(model, group, comm)
    return model._dp


def sharded_nll(model, x, k=5000, mode="image", group=None):
    """Test NLL over all images of x (every rank passes the same x).  Each rank
    draws from its own noise stream (rank).  Returns (mean NLL over all images,
    this rank's per-image log p(x))."""
    rank, w = world(group)
    if w > 1:
        model.set_noise_stream(rank)
    xd = model._x(x)
    N = xd.shape[0]
    if mode == "image":
        lo, hi = shard_range(N, rank, w)
        lp = model.log_px(xd[lo:hi], k) if hi > lo else torch.zeros(0, device=model.device)
        tot = torch.stack([lp.sum(), torch.tensor(float(hi - lo), device=model.device)])
        if w > 1:
            dist.all_reduce(tot, group=group)
        return float(-(tot[0] / tot[1]).item()), lp
    if mode == "sample":
        lo, hi = shard_range(k, rank, w)
        kl = hi - lo
        m, s = model.log_px_partials(xd, kl)
        M, S = merge_lse_partials(m, s, group)
        lp = M + torch.log(S) - math.log(k)
        return float(-lp.mean().item()), lp
    raise ValueError("mode must be 'image' or 'sample'")
