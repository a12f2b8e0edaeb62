"""Host-side data plumbing around the hot path:
local-file dataset loaders, stochastic binarisation, the output-bias
initialiser, and the reference's learning-rate-stage training driver.

Nothing here is on the GPU path; it feeds ``Flexible_Model`` the same arrays
the reference builds from TF datasets (F:147-F:175, E:20-E:31), but only from
files already on disk -- there is no network.
"""
from __future__ import annotations

import gzip
import os

import numpy as np

from .flexible_iwae import output_bias


def _open(path):
    return gzip.open(path, "rb") if str(path).endswith(".gz") else open(path, "rb")


def load_mnist_idx(path):
    """MNIST images from an IDX file (train-images-idx3-ubyte[.gz]) as float32
    [N, 784] in [0, 1] -- the array keras.datasets.mnist.load_data() gives the
    reference before /255 (F:160, F:171)."""
    with _open(path) as f:
        data = f.read()
    magic, n, rows, cols = (int.from_bytes(data[i:i + 4], "big") for i in range(0, 16, 4))
    if magic != 2051:
        raise ValueError(f"{path}: not an IDX3 image file (magic {magic})")
    x = np.frombuffer(data, dtype=np.uint8, count=n * rows * cols, offset=16)
    return (x.reshape(n, rows * cols).astype(np.float32) / 255.0)


def load_binarized_mnist(path):
    """Fixed-binarisation MNIST (E:25 loads it with tfds as binarized_mnist):
    the Larochelle .amat text format (one image of 784 0/1 values per line) or
    a .npy / .npz array of shape [N, 784] (or [N, 28, 28(, 1)])."""
    p = str(path)
    if p.endswith(".amat") or p.endswith(".amat.gz"):
        with _open(p) as f:
            rows = [np.array(line.split(), dtype=np.float32) for line in f.read().decode().splitlines()
                    if line.strip()]
        x = np.stack(rows)
    elif p.endswith(".npz"):
        with np.load(p, allow_pickle=False) as z:
            x = z[z.files[0]]
    else:
        x = np.load(p, allow_pickle=False)
    x = np.asarray(x, dtype=np.float32).reshape(len(x), -1)
    if x.shape[1] != 784:
        raise ValueError(f"{p}: expected 784 pixels per image, got {x.shape[1]}")
    return x


def load_omniglot_chardata(path, split="data"):
    """OMNIGLOT from chardata.mat (F:164: d["data"].transpose().reshape(-1,
    784)); ``split`` is "data" (train) or "testdata".  scipy.io.loadmat parses
    the MATLAB container without executing anything from the file."""
    import scipy.io as sio
    d = sio.loadmat(path)
    return np.asarray(d[split], dtype=np.float32).transpose().reshape((-1, 28 * 28))


def stochastic_binarize(x, rng):
    """Dynamic binarisation (the "MNIST" stochastic setting, PDF p7 s3.1):
    pixel ~ Bernoulli(grey level), redrawn each time it is called."""
    return (rng.random(x.shape, dtype=np.float32) < x).astype(np.float32)


def bias_from_train(x_train):
    """Decoder output bias from training pixel means (F:170-F:175)."""
    return output_bias(np.asarray(x_train, np.float64).reshape(len(x_train), -1).mean(axis=0))


def stage_learning_rate(i):
    """E:76: learning rate of stage i = 1..8 (1e-3 down to 1e-4)."""
    return 1e-4 * round(10.0 ** (1 - (i - 1) / 7.0), 1)


def stage_passes(i):
    """E:77: 3**(i-1) passes over the training data in stage i."""
    return 3 ** (i - 1)


def train_schedule(model, x_train, stages=8, batch_size=100, x_test=None, k_test=None, on_stage=None,
                   save_prefix=None, stochastic_rng=None, passes=stage_passes, verbose=0):
    """The reference's training driver (E:73-E:97): for stage i = 1..stages set
    the Adam learning rate (E:76), run passes(i) epochs of fit (E:82), then
    optionally evaluate get_training_statistics(x_test, k_test) (E:87),
    call on_stage(i, total_passes, res) and save the weights (E:95) and the
    statistics so far (E:96-E:97: the reference pickles (res1s, res2s); here
    they are JSON, `<save_prefix>.res2.json`).  With stochastic_rng the
    training set is re-binarised every epoch.  Returns the list of per-stage
    statistics ((res1, res2) pairs, or None without x_test)."""
    if model.optimizer is None:
        model.compile()
    results = []
    total = 0
    for i in range(1, stages + 1):
        model.optimizer.learning_rate = stage_learning_rate(i)
        model._push_adam()
        n = passes(i)
        for _ in range(n):
            xs = stochastic_binarize(x_train, stochastic_rng) if stochastic_rng is not None else x_train
            model.fit(xs, epochs=1, batch_size=batch_size, verbose=verbose)
        total += n
        res = None
        if x_test is not None:
            res = model.get_training_statistics(x_test, k_test or model.k)
        results.append(res)
        if on_stage is not None:
            on_stage(i, total, res)
        if save_prefix is not None:
            model.save_weights(f"{save_prefix}-epoch_{i}.npz")
            if x_test is not None:
                save_results(f"{save_prefix}.res2.json", results)
    return results


def default_prefix(model):
    """The reference's file stem (E:95): <loss>-<L>L-k_<k>."""
    return f"{model.loss_function}-{len(model.n_latent_encoder)}L-k_{model.k}"


def _plain(v):
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


def save_results(path, results):
    """(res1s, res2s) of the stages so far as JSON (E:96-E:97 without pickle)."""
    import json
    res1s = [r[0] for r in results if r is not None]
    res2s = [r[1] for r in results if r is not None]
    with open(path, "w") as f:
        json.dump({"res1s": _plain(res1s), "res2s": _plain(res2s)}, f)


def load_results(path):
    import json
    with open(path) as f:
        d = json.load(f)
    return d["res1s"], d["res2s"]
