"""Multi-GPU paths: one process per GPU, torch.distributed over RCCL/xGMI.

* Training: data parallel.  Every rank runs the
  full train step on its own batch shard, the flat gradient buffer (2.08 MB
  fp32 for the 2-layer model) is summed with one RCCL all-reduce, and every
  rank applies the identical Adam update scaled by 1/world (the loss is a batch
  mean, F:369).  The reference has no distributed code at all.
* k=5000 NLL (config C3): sharded by test image (no data-path collective, one
  scalar all-reduce for the mean) or by sample chunk (each rank draws
  k/world samples of every image; per-image log-sum-exp partials (m, s) are
  all-gathered and merged: M = max m, S = sum s*exp(m-M),
  log p(x) = M + log S - log k).
"""
from __future__ import annotations

import math

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


class DataParallel:
    """Binds a torch-owned gradient buffer to the handle so RCCL can reduce it
    in place; step = forward_backward -> all_reduce(sum) -> Adam(grad/world)."""

    def __init__(self, model, group=None):
        self.group = group
        g = _lib.FP()
        n = __import__("ctypes").c_longlong(0)
        model._call(model._lib.iwae_grad_buffer(model._h, __import__("ctypes").byref(g),
                                                __import__("ctypes").byref(n)))
        with torch.cuda.stream(model._stream):
            self.grad = torch.zeros(int(n.value), device=model.device)
        model._call(model._lib.iwae_bind_grad_buffer(model._h, _lib.fptr(self.grad), int(n.value)))
        self.rank, self.world = world(group)

    def step(self, model, lc, xd, B, arr, n):
        model._forward_backward(lc, xd, B, arr, n)
        if self.world > 1:
            with torch.cuda.stream(model._stream):
                dist.all_reduce(self.grad, group=self.group)
        model._apply_adam(1.0 / self.world)


def enable_data_parallel(model, group=None):
    model._dp = DataParallel(model, group)
    return model._dp


def sharded_nll(model, x, k=5000, mode="image", group=None):
    """Test NLL over all images of x (every rank passes the same x).
    Returns (mean NLL over all images, this rank's per-image log p(x))."""
    rank, w = world(group)
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
        with torch.cuda.stream(model._stream):
            m = torch.empty(N, device=model.device)
            s = torch.empty(N, device=model.device)
        model._call(model._lib.iwae_nll_partials(model._h, _lib.fptr(xd), N, int(kl), 0, _lib.fptr(m),
                                                 _lib.fptr(s)))
        model._stream.synchronize()
        M, S = merge_lse_partials(m, s, group)
        lp = M + torch.log(S) - math.log(k)
        return float(-lp.mean().item()), lp
    raise ValueError("mode must be 'image' or 'sample'")
