"""Drop-in ``Flexible_Model`` for the IWAE train-step / NLL hot path.

Mirrors the public surface of the reference class
``flexible_IWAE.Flexible_Model`` (/root/reference/flexible_IWAE.py, "F:"):
same constructor knobs (F:178-F:180), same method names, argument meaning and
return values -- but every number is computed by the HIP library
(libiwae_hip.so, gfx950) through the C ABI of include/iwae.h.  PyTorch is used
only for device memory, the HIP stream and torch.distributed; there is no CPU
fallback (the constructor raises without a GPU or without the library).

Differences a user of the reference should know about (all deliberate):
  * ``train_step`` returns ``{loss_function: float}``; ``fit`` runs the
    Keras-style epoch/batch loop over a device-resident copy of the data.
  * ``dataset_bias`` may be a 784-vector of training pixel means (the quantity
    F:170-F:175 derives from the downloaded dataset) or ``None``; dataset
    names need the mean stored locally (no network): ``$IWAE_DATA_DIR/
    {mnist,omniglot}_train_mean.npy``.
  * Every evaluation entry point accepts an optional ``eps=`` list of
    ``[k, B, d_i]`` noise arrays (the reference's sample-major layout) so runs
    can be reproduced exactly; by default noise is drawn on device (Philox).
  * ``loss_function`` additionally accepts "MIWAE" and "PIWAE" (k = k1*k2,
    IWAE_replication.pdf p7); an unknown name raises ValueError where the
    reference hits UnboundLocalError (F:242).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _lib

LOSSES = tuple(_lib.LOSS_IDS)


# ----------------------------------------------------------------- helpers
def architecture(n_hidden_encoder, n_hidden_decoder, n_latent_encoder, n_latent_decoder, x_dim=784):
    """Validate the constructor knobs and return the Dense layers in Keras
    ``trainable_weights`` order as (name, fan_in, fan_out) (F:22-F:96)."""
    he, hd = [int(v) for v in n_hidden_encoder], [int(v) for v in n_hidden_decoder]
    le, ld = [int(v) for v in n_latent_encoder], [int(v) for v in n_latent_decoder]
    L = len(he)
    if L < 1 or L > _lib.MAX_LAYERS:
        raise ValueError(f"need 1..{_lib.MAX_LAYERS} stochastic layers")
    if len(le) != L or len(hd) != L or len(ld) != L:
        raise ValueError("n_hidden_encoder, n_hidden_decoder, n_latent_encoder and n_latent_decoder "
                         "must have one entry per stochastic layer (F:206-F:209)")
    if min(he + hd + le) <= 0:
        raise ValueError("layer sizes must be positive")
    for i in range(L - 1):
        if ld[i] != le[L - 2 - i]:
            raise ValueError(f"n_latent_decoder[{i}]={ld[i]} must equal n_latent_encoder[{L-2-i}]={le[L-2-i]} "
                             "(decoder layer i models h_{L-1-i}, F:139-F:140)")
    dense = []
    for i in range(L):
        fin = x_dim if i == 0 else le[i - 1]
        dense += [(f"enc{i}.l1", fin, he[i]), (f"enc{i}.l2", he[i], he[i]),
                  (f"enc{i}.lmu", he[i], le[i]), (f"enc{i}.lstd", he[i], le[i])]
    for i in range(L - 1):
        fin = le[L - 1 - i]
        dense += [(f"dec{i}.l1", fin, hd[i]), (f"dec{i}.l2", hd[i], hd[i]),
                  (f"dec{i}.lmu", hd[i], ld[i]), (f"dec{i}.lstd", hd[i], ld[i])]
    dense += [("out.l1", le[0], hd[-1]), ("out.l2", hd[-1], hd[-1]), ("out.l3", hd[-1], x_dim)]
    return dense


def weight_shapes(dense):
    out = []
    for _, fin, fout in dense:
        out += [(fin, fout), (fout,)]
    return out


def output_bias(train_mean):
    """F:170-F:175: -log(1/clip(mean, .001, .999) - 1)."""
    m = np.clip(np.asarray(train_mean, dtype=np.float64).reshape(-1), 0.001, 0.999)
    return -np.log(1.0 / m - 1.0)


def resolve_dataset_bias(dataset_bias, x_dim=784):
    """Decoder output-bias initialiser (Decoder.get_bias, F:147-F:175)."""
    if dataset_bias is None:
        return np.zeros(x_dim)
    if isinstance(dataset_bias, str):
        name = dataset_bias.lower()
        if "mnist" in name:           # covers F:148 (binarized_mnist) and F:157 (mnist)
            key = "mnist"
        elif "omniglot" in name:      # F:162
            key = "omniglot"
        else:                         # F:167
            raise Exception("Trying to set the initialisation for the bias, "
                            "but the dataset is not recognized")
        d = os.environ.get("IWAE_DATA_DIR")
        path = os.path.join(d, f"{key}_train_mean.npy") if d else None
        if not path or not os.path.exists(path):
            raise FileNotFoundError(
                f"dataset_bias={dataset_bias!r} needs the training pixel means offline: put "
                f"{key}_train_mean.npy (784 values in [0,1]) in $IWAE_DATA_DIR, or pass the mean "
                "vector itself (or None) as dataset_bias")
        return output_bias(np.load(path, allow_pickle=False))
    arr = np.asarray(dataset_bias, dtype=np.float64).reshape(-1)
    if arr.size != x_dim:
        raise ValueError(f"dataset_bias vector must have {x_dim} entries")
    return output_bias(arr)


def glorot_weights(dense, rng, out_bias):
    """Keras defaults: glorot_uniform kernels, zero biases (PDF p8 s3.4)."""
    ws = []
    for name, fin, fout in dense:
        lim = math.sqrt(6.0 / (fin + fout))
        ws.append(rng.uniform(-lim, lim, size=(fin, fout)).astype(np.float32))
        b = np.zeros(fout, np.float32)
        if name == "out.l3":
            b = np.asarray(out_bias, np.float32).reshape(fout)
        ws.append(b)
    return ws


def loss_config(loss_function, k, p=1.0, alpha=1.0, beta=0.5, k1=None, k2=None):
    if loss_function not in _lib.LOSS_IDS:
        raise ValueError(f"unknown loss_function {loss_function!r}; expected one of {LOSSES}")
    if loss_function in ("MIWAE", "PIWAE"):
        if k1 is None or k2 is None:
            raise ValueError(f"{loss_function} needs k1 and k2 (k = k1*k2)")
        k = int(k1) * int(k2)
    return _lib.IwaeLossConfig(_lib.LOSS_IDS[loss_function], int(k), float(p), float(alpha), float(beta),
                               int(k1 or 0), int(k2 or 0))


# --------------------------------------------------------------- optimizer
class Adam:
    """Keras ``tf.keras.optimizers.Adam`` knobs used by E:36-E:40 (defaults are
    Keras' own).  Setting ``learning_rate`` (E:76) updates every compiled model."""

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self._lr = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self._models = []

    @property
    def learning_rate(self):
        return self._lr

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr = float(v)
        for m in self._models:
            m._push_adam()

    lr = learning_rate


# ------------------------------------------------------------------ model
class Flexible_Model:
    """HIP-backed ``Flexible_Model`` (F:177-F:545)."""

    def __init__(self, n_hidden_encoder, n_hidden_decoder, n_latent_encoder, n_latent_decoder,
                 dataset_bias="Binarized_MNIST", loss_function="VAE", k=50, p=1, alpha=1, beta=0.5,
                 *, k1=None, k2=None, x_dim=784, device=None, seed=None, use_graphs=True,
                 kernel_path="auto", precision="bf16x3", tuning=None, **kwargs):
        self.dense = architecture(n_hidden_encoder, n_hidden_decoder, n_latent_encoder, n_latent_decoder, x_dim)
        loss_config(loss_function, k, p, alpha, beta, k1, k2)   # validate early
        if not torch.cuda.is_available():
            raise RuntimeError("Flexible_Model runs on the HIP library only and needs a ROCm GPU "
                               "(no CPU fallback)")
        self._lib = _lib.load()
        self.n_hidden_encoder = list(n_hidden_encoder)
        self.n_hidden_decoder = list(n_hidden_decoder)
        self.n_latent_encoder = list(n_latent_encoder)
        self.n_latent_decoder = list(n_latent_decoder)
        self.n_stochastic_encoder = len(n_hidden_encoder)      # F:210
        self.n_stochastic_decoder = len(n_hidden_decoder)      # F:211
        self.dataset_bias = dataset_bias
        self.loss_function = loss_function
        self.k, self.p, self.alpha, self.beta = k, p, alpha, beta
        self.k1, self.k2 = k1, k2
        self.x_dim = x_dim
        self.epoch = 0                                          # F:218
        self.optimizer = None
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
        self._dp = None
        cfg = _lib.IwaeConfig()
        L = len(self.n_hidden_encoder)
        cfg.n_stochastic = L
        cfg.x_dim = x_dim
        for i in range(L):
            cfg.n_hidden_encoder[i] = self.n_hidden_encoder[i]
            cfg.n_latent_encoder[i] = self.n_latent_encoder[i]
            cfg.n_hidden_decoder[i] = self.n_hidden_decoder[i]
            cfg.n_latent_decoder[i] = self.n_latent_decoder[i]
        h = self._lib.iwae_create(cfg, self.device.index)
        if not h:
            raise RuntimeError(f"iwae_create failed: {self._lib.iwae_create_error().decode()}")
        self._h = h
        self._stream = torch.cuda.Stream(device=self.device)
        self._call(self._lib.iwae_set_stream(h, ctypes_stream(self._stream)))
        self._nparams = int(self._lib.iwae_num_params(h))
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self._call(self._lib.iwae_set_seed(h, int(seed) & ((1 << 64) - 1)))
        self._call(self._lib.iwae_set_graphs(h, 1 if use_graphs else 0))
        paths = {"auto": 0, "layerwise": 1, "fused": 2, "engine": 3}
        if kernel_path not in paths:
            raise ValueError(f"kernel_path must be one of {tuple(paths)}")
        self._call(self._lib.iwae_set_path(h, paths[kernel_path]))
        precisions = {"f32": 0, "bf16x3": 1}
        if precision not in precisions:
            raise ValueError(f"precision must be one of {tuple(precisions)}")
        self._call(self._lib.iwae_set_precision(h, precisions[precision]))
        for name, value in (tuning or {}).items():
            self.set_tuning(name, value)
        rng = np.random.default_rng(int(seed) & ((1 << 63) - 1))
        self.set_weights(glorot_weights(self.dense, rng, resolve_dataset_bias(dataset_bias, x_dim)))
        self._loss_buf = torch.zeros(1, device=self.device)
        self._scratch = torch.zeros(1, device=self.device)

    # ------------------------------------------------------------- plumbing
    def set_seed(self, seed):
        """Re-key the device Philox stream and restart its counter (reproducible
        draws from here on).  The reference has no seed."""
        self._call(self._lib.iwae_set_seed(self._h, int(seed) & ((1 << 64) - 1)))

    def set_noise_stream(self, stream):
        """Select the noise stream (one per rank: Philox key derived from (seed,
        stream); stream 0 is the seed's own).  Each stream continues from its
        own counter position (re-selecting the current stream is a no-op);
        ``set_seed`` restarts them all."""
        self._call(self._lib.iwae_set_noise_stream(self._h, int(stream) & ((1 << 64) - 1)))

    def set_tuning(self, name, value):
        """Kernel-variant / tuning knob of the library (include/iwae.h enum
        iwae_knob, e.g. ``set_tuning("upd", 0)``): for A/B measurements and the
        variant-agreement tests; the defaults are the measured-fastest paths."""
        if name not in _lib.KNOBS:
            raise ValueError(f"unknown tuning knob {name!r}; expected one of {tuple(_lib.KNOBS)}")
        self._call(self._lib.iwae_set_tuning(self._h, _lib.KNOBS[name], int(value)))

    def _call(self, rc):
        _lib.check(self._lib, self._h, rc)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                self._lib.iwae_destroy(h)
            except Exception:
                pass
            self._h = None

    def _x(self, x):
        t = torch.as_tensor(x)
        if t.dim() < 2:
            raise ValueError("x must be [B, 28, 28, 1] or [B, 784]")
        t = t.reshape(t.shape[0], int(np.prod(t.shape[1:])))     # explicit width: an empty batch stays [0, 784]
        if t.shape[1] != self.x_dim:                      # F:57 assert(x.shape[1] == 28*28)
            raise ValueError(f"x must flatten to {self.x_dim} pixels, got {t.shape[1]}")
        with torch.cuda.stream(self._stream):
            return t.to(device=self.device, dtype=torch.float32, non_blocking=True).contiguous()

    def _eps(self, eps, B, k, n_draws=1):
        if eps is None:
            return None, 0, []
        eps = list(eps)
        L = len(self.n_latent_encoder)
        if len(eps) != n_draws * L:
            raise ValueError(f"expected {n_draws * L} eps arrays, got {len(eps)}")
        ts = []
        with torch.cuda.stream(self._stream):
            for i, e in enumerate(eps):
                t = torch.as_tensor(e).to(device=self.device, dtype=torch.float32, non_blocking=True).contiguous()
                d = self.n_latent_encoder[i % L]
                if tuple(t.shape) != (k, B, d):
                    raise ValueError(f"eps[{i}] must be [k={k}, B={B}, d={d}], got {tuple(t.shape)}")
                ts.append(t)
        arr, n = _lib.fptr_array(ts)
        return arr, n, ts

    def _scalar(self, fn, *args):
        with torch.cuda.stream(self._stream):
            out = torch.empty(1, device=self.device)
        self._call(fn(self._h, *args, _lib.fptr(out)))
        self._stream.synchronize()
        return float(out.item())

    def _lc(self, loss_function=None, k=None, p=None, alpha=None, beta=None, k1=None, k2=None):
        return loss_config(loss_function or self.loss_function, self.k if k is None else k,
                           self.p if p is None else p, self.alpha if alpha is None else alpha,
                           self.beta if beta is None else beta,
                           self.k1 if k1 is None else k1, self.k2 if k2 is None else k2)

    # ------------------------------------------------------------- weights
    @property
    def trainable_weights(self):
        return self.get_weights()

    def get_weights(self):
        flat = np.empty(self._nparams, np.float32)
        self._call(self._lib.iwae_get_params(self._h, flat.ctypes.data_as(_lib.FP), flat.size))
        return _split(flat, weight_shapes(self.dense))

    def set_weights(self, weights):
        flat = _join(weights, weight_shapes(self.dense))
        self._call(self._lib.iwae_set_params(self._h, flat.ctypes.data_as(_lib.FP), flat.size))

    def get_gradients(self):
        """Gradient of the loss from the last train step / forward_backward."""
        flat = np.empty(self._nparams, np.float32)
        self._call(self._lib.iwae_get_grads(self._h, flat.ctypes.data_as(_lib.FP), flat.size))
        return _split(flat, weight_shapes(self.dense))

    def get_optimizer_state(self):
        m = np.empty(self._nparams, np.float32)
        v = np.empty(self._nparams, np.float32)
        import ctypes
        step = ctypes.c_longlong(0)
        self._call(self._lib.iwae_get_adam_state(self._h, m.ctypes.data_as(_lib.FP), v.ctypes.data_as(_lib.FP),
                                                 m.size, ctypes.byref(step)))
        return m, v, int(step.value)

    def set_optimizer_state(self, m, v, step):
        m = np.ascontiguousarray(m, np.float32)
        v = np.ascontiguousarray(v, np.float32)
        self._call(self._lib.iwae_set_adam_state(self._h, m.ctypes.data_as(_lib.FP), v.ctypes.data_as(_lib.FP),
                                                 m.size, int(step)))

    def save_weights(self, path):
        """Weights + Adam state as .npz (the reference uses TF checkpoints, E:95)."""
        m, v, step = self.get_optimizer_state()
        ws = self.get_weights()
        np.savez(path, *ws, adam_m=m, adam_v=v, adam_step=np.int64(step), epoch=np.int64(self.epoch))

    def load_weights(self, path):
        with np.load(path, allow_pickle=False) as z:
            n = len(weight_shapes(self.dense))
            self.set_weights([z[f"arr_{i}"] for i in range(n)])
            if "adam_m" in z:
                self.set_optimizer_state(z["adam_m"], z["adam_v"], int(z["adam_step"]))
            if "epoch" in z:
                self.epoch = int(z["epoch"])

    # ------------------------------------------------------------- training
    def compile(self, optimizer=None, **kwargs):
        self.optimizer = optimizer if optimizer is not None else Adam()
        if self not in self.optimizer._models:
            self.optimizer._models.append(self)
        self._push_adam()

    def _push_adam(self):
        o = self.optimizer
        self._call(self._lib.iwae_set_adam(self._h, o.learning_rate, o.beta_1, o.beta_2, o.epsilon))

    def train_step(self, x, eps=None, sync=True):
        """F:221-F:247: one optimisation step; returns {loss_function: loss}."""
        if self.optimizer is None:
            self.compile()
        xd = self._x(x)
        B = xd.shape[0]
        lc = self._lc()
        arr, n, keep = self._eps(eps, B, lc.k, 2 if self.loss_function == "CIWAE" else 1)
        if self._dp is not None:
            self._dp.step(self, lc, xd, B, arr, n)
        else:
            self._call(self._lib.iwae_train_step(self._h, lc, _lib.fptr(xd), B, arr, n, _lib.fptr(self._loss_buf)))
        self.epoch += 1                                                   # F:245
        if not sync:
            return {self.loss_function: self._loss_buf}
        self._stream.synchronize()
        loss = float(self._loss_buf.item())
        self._call(self._lib.iwae_status(self._h))      # an in-launch wait that gave up raises
        return {self.loss_function: loss}

    def train_steps(self, x, batch_size, sync=True):
        """len(x) // batch_size consecutive train steps (F:221-F:247 each) on the
        batches x[i*batch_size:(i+1)*batch_size] with device noise: fit's inner
        loop (E:82) as one library call (iwae_train_steps: up to 32 steps per
        captured graph).  Returns the per-step losses (device tensor if
        sync=False)."""
        if self.optimizer is None:
            self.compile()
        xd = self._x(x)
        B = int(batch_size)
        if B <= 0:
            raise ValueError("batch_size must be positive")
        n = xd.shape[0] // B
        with torch.cuda.stream(self._stream):
            losses = torch.empty(n, device=self.device)
        if n == 0:
            return losses if not sync else losses.cpu().numpy()
        if self._dp is not None and self._dp.comm != "library":
            for i in range(n):
                self._dp.step(self, self._lc(), xd[i * B:(i + 1) * B], B, None, 0)
                with torch.cuda.stream(self._stream):
                    losses[i] = self._loss_buf[0]
        else:
            self._call(self._lib.iwae_train_steps(self._h, self._lc(), _lib.fptr(xd), B, n, _lib.fptr(losses)))
        self.epoch += n                                                   # F:245, per step
        if not sync:
            return losses
        self._stream.synchronize()
        out = losses.cpu().numpy()
        self._call(self._lib.iwae_status(self._h))      # an in-launch wait that gave up raises
        return out

    def prepare_train_steps(self, x, batch_size):
        """Capture every graph train_steps(x, batch_size) will replay, without
        running a step (iwae_train_steps_prepare): a timed loop then measures
        replays only.  Parameters, Adam state and noise are untouched."""
        if self.optimizer is None:
            self.compile()
        xd = self._x(x)
        B = int(batch_size)
        if B <= 0:
            raise ValueError("batch_size must be positive")
        n = xd.shape[0] // B
        if n and not (self._dp is not None and self._dp.comm != "library"):
            self._call(self._lib.iwae_train_steps_prepare(self._h, self._lc(), _lib.fptr(xd), B, n))

    def graph_captures(self):
        """Train-step graphs captured so far (iwae_debug_count id 7)."""
        return int(self._lib.iwae_debug_count(self._h, 7))

    def check_kernel_status(self):
        """Synchronize and raise if a kernel reported a failure: an in-launch
        wait of the combined image-row backward + update launch that gave up
        (iwae_status; give-ups counted by iwae_debug_count id 8)."""
        self._call(self._lib.iwae_synchronize(self._h))
        n = int(self._lib.iwae_debug_count(self._h, 8))
        if n:
            raise _lib.IwaeError(f"{n} in-launch wait(s) gave up")

    def fit(self, x, epochs=1, batch_size=100, shuffle=True, verbose=0, seed=None):
        """Keras-style loop (E:82): per epoch shuffle, batches of batch_size
        (last partial batch included), one train step each (the whole batches
        through train_steps, the partial one through train_step)."""
        xd = self._x(x)
        N = xd.shape[0]
        g = torch.Generator(device="cpu")
        if seed is not None:
            g.manual_seed(int(seed))
        hist = []
        for ep in range(int(epochs)):
            perm = torch.randperm(N, generator=g) if shuffle else torch.arange(N)
            with torch.cuda.stream(self._stream):
                xs = xd[perm.to(self.device)] if shuffle else xd
                losses = torch.zeros((N + batch_size - 1) // batch_size, device=self.device)
            nfull = N // batch_size
            if nfull:
                full = self.train_steps(xs[:nfull * batch_size], batch_size, sync=False)
                with torch.cuda.stream(self._stream):
                    losses[:nfull] = full
            if N % batch_size:
                out = self.train_step(xs[nfull * batch_size:], sync=False)[self.loss_function]
                with torch.cuda.stream(self._stream):
                    losses[nfull] = out[0]
            self._stream.synchronize()
            hist.append(float(losses.mean().item()))
            if verbose:
                print(f"epoch {ep + 1}/{epochs} - {self.loss_function}: {hist[-1]:.4f}")
        return {self.loss_function: hist}

    # ----------------------------------------------------------- evaluation
    def get_log_weights(self, x, n_samples, eps=None):
        """F:327-F:351: log w, returned sample-major [n_samples, B] like the reference."""
        xd = self._x(x)
        B = xd.shape[0]
        arr, n, keep = self._eps(eps, B, n_samples)
        with torch.cuda.stream(self._stream):
            lw = torch.empty(B, n_samples, device=self.device)
        self._call(self._lib.iwae_log_weights(self._h, _lib.fptr(xd), B, int(n_samples), arr, n, _lib.fptr(lw)))
        with torch.cuda.stream(self._stream):
            out = lw.t().contiguous()
        self._stream.synchronize()
        return out

    @staticmethod
    def L_k_from_weights(log_weights):
        """F:363-F:370 on a [k, B] tensor."""
        lw = torch.as_tensor(log_weights)
        m = lw.max(dim=0).values
        return torch.mean(torch.log(torch.mean(torch.exp(lw - m), dim=0)) + m)

    @staticmethod
    def L_from_weights(log_weights):
        """F:429-F:430."""
        return torch.mean(torch.as_tensor(log_weights))

    def _bound(self, lc, x, eps, n_draws=1):
        xd = self._x(x)
        B = xd.shape[0]
        arr, n, keep = self._eps(eps, B, lc.k, n_draws)
        return self._scalar(self._lib.iwae_bound, lc, _lib.fptr(xd), B, arr, n)

    def get_L_k(self, x, k, eps=None):
        """F:354-F:361."""
        return self._bound(self._lc("IWAE", k=k), x, eps)

    def get_L(self, x, k=5000, eps=None):
        """F:419-F:427."""
        return self._bound(self._lc("VAE", k=k), x, eps)

    def get_L_median(self, x, k, eps=None):
        """F:373-F:379."""
        return self._bound(self._lc("L_median", k=k), x, eps)

    def get_L_CIWAE(self, x, n_samples, beta, eps=None):
        """F:382-F:383 (two independent draws: eps = draw1 + draw2)."""
        return self._bound(self._lc("CIWAE", k=n_samples, beta=beta), x, eps, 2)

    def get_L_alpha(self, x, n_samples, alpha, eps=None):
        """F:386-F:402."""
        return self._bound(self._lc("L_alpha", k=n_samples, alpha=alpha), x, eps)

    def get_L_power_p(self, x, k, p, eps=None):
        """F:405-F:409."""
        return self._bound(self._lc("L_power_p", k=k, p=p), x, eps)

    def get_L_V1(self, x, n_samples, eps=None):
        """F:434-F:460."""
        return self._bound(self._lc("VAE_V1", k=n_samples), x, eps)

    def get_L_MIWAE(self, x, k1, k2, eps=None):
        """MIWAE(k1, k2) (IWAE_replication.pdf p7)."""
        return self._bound(self._lc("MIWAE", k1=k1, k2=k2), x, eps)

    def get_E_qhIx_log_pxIh(self, x, n_samples, eps=None):
        """F:304-F:325 (Keras binary cross-entropy form)."""
        xd = self._x(x)
        B = xd.shape[0]
        arr, n, keep = self._eps(eps, B, n_samples)
        return self._scalar(self._lib.iwae_e_log_px, _lib.fptr(xd), B, int(n_samples), arr, n)

    def get_Dkl_qhIx_ph(self, x, k):
        """F:414-F:415."""
        return self.get_E_qhIx_log_pxIh(x, k) - self.get_L(x, k)

    def get_Dkl_qhIx_phIx(self, x, k):
        """F:411-F:412."""
        return -1 * (self.get_L(x, k) + self.get_NLL(x))

    def log_px(self, x, k=5000, eps=None, chunk=0):
        """Per-image k-sample log p(x) estimate (device tensor [N])."""
        xd = self._x(x)
        N = xd.shape[0]
        with torch.cuda.stream(self._stream):
            out = torch.empty(N, device=self.device)
        if eps is not None:
            arr, n, keep = self._eps(eps, N, k)
            self._call(self._lib.iwae_nll_eps(self._h, _lib.fptr(xd), N, int(k), arr, n, _lib.fptr(out)))
        else:
            self._call(self._lib.iwae_nll(self._h, _lib.fptr(xd), N, int(k), int(chunk), _lib.fptr(out)))
        self._stream.synchronize()
        return out

    def log_px_partials(self, x, k_local, chunk=0):
        """Per-image log-sum-exp partials over k_local device-noise samples of
        this handle's noise stream: (m, s) with m = max_s lw, s = sum_s exp(lw - m)
        (the sample-sharded NLL's per-rank contribution)."""
        xd = self._x(x)
        N = xd.shape[0]
        with torch.cuda.stream(self._stream):
            m = torch.empty(N, device=self.device)
            s = torch.empty(N, device=self.device)
        self._call(self._lib.iwae_nll_partials(self._h, _lib.fptr(xd), N, int(k_local), int(chunk), _lib.fptr(m),
                                               _lib.fptr(s)))
        self._stream.synchronize()
        return m, s

    def get_NLL(self, x, k=5000, eps=None):
        """F:463-F:464: -L_k with k = 5000 by default."""
        return float(-self.log_px(x, k, eps).mean().item())

    # ------------------------------------------------ evaluation statistics
    def _reconstruct(self, x, eps, want_probs):
        xd = self._x(x)
        B = xd.shape[0]
        L = len(self.n_latent_encoder)
        arr, n, keep = None, 0, []
        if eps is not None:
            eps = list(eps)
            if len(eps) != 2 * L - 1:
                raise ValueError(f"expected {2 * L - 1} eps arrays (encoder, then prior), got {len(eps)}")
            dims = list(self.n_latent_encoder) + [self.n_latent_encoder[L - 2 - j] for j in range(L - 1)]
            with torch.cuda.stream(self._stream):
                for e, d in zip(eps, dims):
                    t = torch.as_tensor(e).to(device=self.device, dtype=torch.float32).contiguous()
                    if tuple(t.shape) != (1, B, d):
                        raise ValueError(f"eps arrays must be [1, B={B}, d={d}], got {tuple(t.shape)}")
                    keep.append(t)
            arr, n = _lib.fptr_array(keep)
        with torch.cuda.stream(self._stream):
            ld = (self.x_dim + 3) // 4 * 4
            probs = torch.empty(B, ld, device=self.device) if want_probs else None
            loss = torch.empty(1, device=self.device)
        self._call(self._lib.iwae_reconstruct(self._h, _lib.fptr(xd), B, arr, n, _lib.fptr(probs),
                                              ld if want_probs else 0, _lib.fptr(loss)))
        self._stream.synchronize()
        return (probs[:, :self.x_dim] if want_probs else None), float(loss.item())

    def reconstructed_x_probs(self, x, eps=None):
        """F:249-F:254: pixel probabilities [1, B, 784] of x reconstructed from
        one q(h|x) draw of h_L through the decoder's prior layers (generate_x,
        F:107-F:119).  ``eps``: L encoder arrays [1,B,d_i], then the L-1 prior
        draws in generation order ([1,B,d_{L-2-j}])."""
        probs, _ = self._reconstruct(x, eps, True)
        return probs.unsqueeze(0)

    def get_reconstruction_loss(self, x, eps=None):
        """F:256-F:262: mean over the batch of the Keras BCE of x against the
        reconstructed probabilities, summed over pixels."""
        return self._reconstruct(x, eps, False)[1]

    def encoder_means(self, x, n_samples, eps=None):
        """Device [N, d_i] per layer: the mean over n_samples draws of q(h|x)
        of h_i (the accumulation of F:268-F:276).  ``eps``: [n, N, d_i]."""
        xd = self._x(x)
        N = xd.shape[0]
        arr, n, keep = self._eps(eps, N, n_samples)
        with torch.cuda.stream(self._stream):
            outs = [torch.empty(N, d, device=self.device) for d in self.n_latent_encoder]
        oarr, no = _lib.fptr_array(outs)
        self._call(self._lib.iwae_encoder_means(self._h, _lib.fptr(xd), N, int(n_samples), arr, n, oarr, no))
        self._stream.synchronize()
        return outs

    def get_levels_of_units_activity(self, x, n_samples, eps=None):
        """F:264-F:281: per stochastic layer, the variance over the batch of
        E_q[h_i] and the PCA eigenvalues of those means (host float64 on the
        [N, d_i] means the device produced)."""
        means = [m.double().cpu().numpy() for m in self.encoder_means(x, n_samples, eps)]
        variances = [m.var(0) for m in means]
        return variances, [self.get_eigenvalues_PCA(m) for m in means]

    @staticmethod
    def get_eigenvalues_PCA(data):
        """F:284-F:291: ascending eigenvalues of the empirical covariance
        (divisor N) of data [N, D]."""
        d = np.asarray(data, dtype=np.float64)
        z = d - d.mean(0)
        return np.linalg.eigvalsh(z.T @ z / d.shape[0])

    @staticmethod
    def get_active_units(variances, eigen_values, threshold=0.01):
        """F:294-F:300: 0/1 activity per unit, active counts by variance and
        by PCA eigenvalue."""
        active_units = [[1 if v > threshold else 0 for v in var] for var in variances]
        number_active_units = [int(sum(a)) for a in active_units]
        number_active_units_PCA = [int(sum(1 for e in eig if e > threshold)) for eig in eigen_values]
        return active_units, number_active_units, number_active_units_PCA

    def log_px_masked(self, x, masks, k=5000, eps=None):
        """Per-image k-sample log p(x) with every sampled h_i multiplied by
        masks[i] (0/1, length d_i) before log q and the later layers."""
        xd = self._x(x)
        N = xd.shape[0]
        L = len(self.n_latent_encoder)
        if len(masks) != L:
            raise ValueError(f"expected {L} masks, got {len(masks)}")
        with torch.cuda.stream(self._stream):
            mts = []
            for m, d in zip(masks, self.n_latent_encoder):
                t = torch.as_tensor(np.asarray(m, dtype=np.float32)).to(self.device).contiguous()
                if tuple(t.shape) != (d,):
                    raise ValueError(f"mask must have {d} entries, got {tuple(t.shape)}")
                mts.append(t)
            out = torch.empty(N, device=self.device)
        marr, nm = _lib.fptr_array(mts)
        arr, n, keep = self._eps(eps, N, k)
        self._call(self._lib.iwae_nll_masked(self._h, _lib.fptr(xd), N, int(k), arr, n, marr, nm, _lib.fptr(out)))
        self._stream.synchronize()
        return out

    def get_NLL_without_inactive_units(self, x, threshold=0.01, n_samples=5000, eps=None, eps_activity=None):
        """F:466-F:494: the activity of the units is measured on x with
        n_samples draws, inactive units are zeroed in every sample, and the
        n_samples-sample estimate is returned as -L_k (an NLL)."""
        variances, eigen_values = self.get_levels_of_units_activity(x, n_samples, eps_activity)
        active_units, _, _ = self.get_active_units(variances, eigen_values, threshold)
        return float(-self.log_px_masked(x, active_units, n_samples, eps).mean().item())

    def get_training_statistics(self, x, k, batch_size=10, batched=True, chunk_images=2000):
        """F:496-F:526: (res, res2) with the reference's keys.  res: batch
        means of VAE, IWAE, NLL (k=5000), E_q log p(x|h), both KL terms,
        reconstruction_loss, and LL_pruned (on the first batch); res2: active
        units (1000 draws over all of x), their counts, PCA counts, variances.

        batched=False runs the reference's loop literally: per batch of
        batch_size images (F:512) one launch series per statistic -- for 10k
        images, 2,000 k=5000 NLL calls of 10 images each (F:515, F:518).
        batched=True (default) evaluates each statistic over many batches per
        call (chunk_images, a multiple of batch_size; the k=5000 NLLs over all
        images at once, chunked by the library) and keeps the per-batch
        reduction: every statistic is a mean over images (equal batches), so
        the mean of the batch means is the chunk-size-weighted mean of the
        chunk means.  Each statistic still gets its own independent draw (the
        reference's separate get_L / get_NLL calls), per image."""
        xd = self._x(x)
        N = xd.shape[0]
        if batch_size <= 0 or N == 0 or N % batch_size != 0:
            # F:500 tf.reshape(x, (-1, batch_size, 28, 28, 1)) raises on a ragged tail
            raise ValueError(f"get_training_statistics: {N} images do not split into batches of {batch_size}")
        nb = N // batch_size
        res = dict(VAE=0.0, IWAE=0.0, NLL=0.0)
        res["E_q(h|x)[log(p(x|h))]"] = 0.0
        res["D_kl(q(h|x),p(h))"] = 0.0
        res["D_kl(q(h|x),p(h|x))"] = 0.0
        res["reconstruction_loss"] = 0.0
        if batched:
            step = max(batch_size, (int(chunk_images) // batch_size) * batch_size)
            for lo in range(0, N, step):
                b = xd[lo:lo + step]
                w = b.shape[0] / N                 # (its batches) / nb
                vae = self.get_L(b, k)
                res["VAE"] += vae * w
                res["IWAE"] += self.get_L_k(b, k) * w
                eq = self.get_E_qhIx_log_pxIh(b, k)
                res["E_q(h|x)[log(p(x|h))]"] += eq * w
                res["D_kl(q(h|x),p(h))"] += (eq - self.get_L(b, k)) * w
                res["D_kl(q(h|x),p(h|x))"] += -1 * self.get_L(b, k) * w
                res["reconstruction_loss"] += self.get_reconstruction_loss(b) * w
            nll1 = self.get_NLL(xd)                 # F:515, every batch in one launch series
            nll2 = self.get_NLL(xd)                 # F:518's second, independent estimate
            res["NLL"] = nll1
            res["D_kl(q(h|x),p(h|x))"] += -1 * nll2          # -(get_L + get_NLL), F:412
        else:
            for i in range(nb):
                b = xd[i * batch_size:(i + 1) * batch_size]
                vae = self.get_L(b, k)
                res["VAE"] += vae / nb
                res["IWAE"] += self.get_L_k(b, k) / nb
                res["NLL"] += self.get_NLL(b) / nb
                eq = self.get_E_qhIx_log_pxIh(b, k)
                res["E_q(h|x)[log(p(x|h))]"] += eq / nb
                res["D_kl(q(h|x),p(h))"] += (eq - self.get_L(b, k)) / nb
                res["D_kl(q(h|x),p(h|x))"] += -1 * (self.get_L(b, k) + self.get_NLL(b)) / nb
                res["reconstruction_loss"] += self.get_reconstruction_loss(b) / nb
        res2 = {}
        variances, eigen_values = self.get_levels_of_units_activity(xd, 1000)
        res2["active_units"], res2["number_of_active_units"], res2["number_of_PCA_active_units"] = \
            self.get_active_units(variances, eigen_values)
        res2["variances"] = variances
        res["LL_pruned"] = self.get_NLL_without_inactive_units(xd[:batch_size])
        return res, res2

    # ------------------------------------------------------------ data parallel
    def get_gradient_snr(self, x, k=None, R=1000, loss_function=None, p=None, alpha=None, beta=None, k1=None,
                         k2=None, seed=None, group=None):
        """Per-parameter gradient signal-to-noise ratio |E g| / std(g) over R
        independent noise draws at fixed weights (the
        estimator SNR of Rainforth et al. 2018, PDF p7).  Each draw is one
        device forward+backward (Philox noise, no Adam step); the moments
        sum g and sum g^2 accumulate on the device (iwae_grad_moments).  Under
        torch.distributed the R draws are split over the ranks (noise stream
        seed + rank) and the moments summed with one all-reduce each.
        Returns (list of SNR arrays in Keras weight order, {'R': R})."""
        from . import distributed as D
        rank, w = D.world(group)
        xd = self._x(x)
        B = xd.shape[0]
        lc = self._lc(loss_function, k, p, alpha, beta, k1, k2)
        if seed is not None:
            self._call(self._lib.iwae_set_seed(self._h, int(seed) & ((1 << 64) - 1)))
        if w > 1:
            self.set_noise_stream(rank)       # per-rank independent draws (also with the default seed)
        import ctypes
        g = _lib.FP()
        n = ctypes.c_longlong(0)
        self._call(self._lib.iwae_grad_buffer(self._h, ctypes.byref(g), ctypes.byref(n)))
        with torch.cuda.stream(self._stream):
            s1 = torch.zeros(int(n.value), device=self.device)
            s2 = torch.zeros(int(n.value), device=self.device)
        lo, hi = D.shard_range(int(R), rank, w)
        for _ in range(hi - lo):
            self._call(self._lib.iwae_forward_backward(self._h, lc, _lib.fptr(xd), B, None, 0,
                                                       _lib.fptr(self._loss_buf)))
            self._call(self._lib.iwae_grad_moments(self._h, _lib.fptr(s1), _lib.fptr(s2)))
        if w > 1:
            with torch.cuda.stream(self._stream):
                torch.distributed.all_reduce(s1, group=group)
                torch.distributed.all_reduce(s2, group=group)
        self._stream.synchronize()
        m1 = np.empty(self._nparams, np.float32)
        m2 = np.empty(self._nparams, np.float32)
        self._call(self._lib.iwae_export_internal(self._h, _lib.fptr(s1), m1.ctypes.data_as(_lib.FP), m1.size))
        self._call(self._lib.iwae_export_internal(self._h, _lib.fptr(s2), m2.ctypes.data_as(_lib.FP), m2.size))
        mean = m1.astype(np.float64) / R
        var = np.maximum(m2.astype(np.float64) / R - mean * mean, 0.0)
        with np.errstate(divide="ignore", invalid="ignore"):
            snr = np.where(var > 0, np.abs(mean) / np.sqrt(var), np.inf)
        return _split(snr, weight_shapes(self.dense)), {"R": int(R)}

    def _forward_backward(self, lc, xd, B, arr, n):
        self._call(self._lib.iwae_forward_backward(self._h, lc, _lib.fptr(xd), B, arr, n,
                                                   _lib.fptr(self._loss_buf)))

    def _apply_adam(self, scale):
        self._call(self._lib.iwae_apply_adam(self._h, float(scale)))


# ------------------------------------------------------------------ utils
def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(int(s.cuda_stream))


def _split(flat, shapes):
    out, o = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(flat[o:o + n].reshape(s).copy())
        o += n
    assert o == flat.size
    return out


def _join(weights, shapes):
    if len(weights) != len(shapes):
        raise ValueError(f"expected {len(shapes)} weight arrays, got {len(weights)}")
    parts = []
    for w, s in zip(weights, shapes):
        a = np.asarray(w, np.float32)
        if a.shape != tuple(s):
            raise ValueError(f"weight of shape {a.shape} where {tuple(s)} is expected")
        parts.append(a.ravel())
    return np.ascontiguousarray(np.concatenate(parts), np.float32)
