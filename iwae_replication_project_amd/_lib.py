"""ctypes binding of libiwae_hip.so (the C ABI declared in include/iwae.h).

The product path has exactly one backend: the HIP library.  If it is missing
or cannot be loaded, :func:`load` raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_longlong, c_ulonglong, c_void_p, c_char_p

MAX_LAYERS = 8
LIB_NAME = "libiwae_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

# loss ids (include/iwae.h enum iwae_loss_id)
# include/iwae.h enum iwae_knob (iwae_set_tuning)
KNOBS = {
    "engine": 1, "tc_img": 2, "tc_imgbwd": 3, "tc_fold0": 4, "tc_xcd": 5, "tc_bound": 6, "tc_rt": 7,
    "upd": 8, "upd_rows": 9, "upd_slabs": 11, "upd_slab_wg": 12, "dw_target": 13,
    "smallm_rows": 14, "out_x3_rows": 15, "mg_waves": 16, "nll_rows": 17, "wide_rows": 18, "dw_wide": 19, "ld_align": 20,
    "nring": 21, "nring_train": 22, "nring_train_rows": 23, "nring_bwd": 24, "wide_rt": 25, "upd_waves": 26,
    "nll_imgs": 27, "dw_wg": 28, "piwae_one": 29, "dw_alpha": 30,
    "img_rows_fwd": 31, "img_rows_bwd": 32, "x_direct": 33, "tcu": 34, "upd_apply": 35, "tcu_wait_test": 41, "tcu_wt": 42,
}
LOSS_IDS = {
    "VAE": 0, "IWAE": 1, "VAE_V1": 2, "L_alpha": 3, "L_power_p": 4,
    "L_median": 5, "CIWAE": 6, "MIWAE": 7, "PIWAE": 8,
}


class IwaeConfig(ctypes.Structure):
    _fields_ = [
        ("n_stochastic", c_int),
        ("x_dim", c_int),
        ("n_hidden_encoder", c_int * MAX_LAYERS),
        ("n_latent_encoder", c_int * MAX_LAYERS),
        ("n_hidden_decoder", c_int * MAX_LAYERS),
        ("n_latent_decoder", c_int * MAX_LAYERS),
    ]


class IwaeLossConfig(ctypes.Structure):
    _fields_ = [
        ("loss", c_int), ("k", c_int), ("p", c_float), ("alpha", c_float),
        ("beta", c_float), ("k1", c_int), ("k2", c_int),
    ]


FP = POINTER(c_float)
FPP = POINTER(FP)
H = c_void_p

# name -> (restype, argtypes); the exported surface of include/iwae.h
SIGNATURES = {
    "iwae_create": (H, [POINTER(IwaeConfig), c_int]),
    "iwae_create_error": (c_char_p, []),
    "iwae_destroy": (None, [H]),
    "iwae_last_error": (c_char_p, [H]),
    "iwae_set_stream": (c_int, [H, c_void_p]),
    "iwae_synchronize": (c_int, [H]),
    "iwae_status": (c_int, [H]),
    "iwae_set_seed": (c_int, [H, c_ulonglong]),
    "iwae_set_noise_stream": (c_int, [H, c_ulonglong]),
    "iwae_set_graphs": (c_int, [H, c_int]),
    "iwae_set_path": (c_int, [H, c_int]),
    "iwae_set_precision": (c_int, [H, c_int]),
    "iwae_set_tuning": (c_int, [H, c_int, c_longlong]),
    "iwae_num_params": (c_longlong, [H]),
    "iwae_set_params": (c_int, [H, FP, c_longlong]),
    "iwae_get_params": (c_int, [H, FP, c_longlong]),
    "iwae_get_grads": (c_int, [H, FP, c_longlong]),
    "iwae_set_adam": (c_int, [H, c_float, c_float, c_float, c_float]),
    "iwae_get_adam_state": (c_int, [H, FP, FP, c_longlong, POINTER(c_longlong)]),
    "iwae_set_adam_state": (c_int, [H, FP, FP, c_longlong, c_longlong]),
    "iwae_train_step": (c_int, [H, POINTER(IwaeLossConfig), FP, c_int, FPP, c_int, FP]),
    "iwae_train_steps": (c_int, [H, POINTER(IwaeLossConfig), FP, c_int, c_int, FP]),
    "iwae_train_steps_prepare": (c_int, [H, POINTER(IwaeLossConfig), FP, c_int, c_int]),
    "iwae_forward_backward": (c_int, [H, POINTER(IwaeLossConfig), FP, c_int, FPP, c_int, FP]),
    "iwae_grad_buffer": (c_int, [H, POINTER(FP), POINTER(c_longlong)]),
    "iwae_bind_grad_buffer": (c_int, [H, FP, c_longlong]),
    "iwae_apply_adam": (c_int, [H, c_float]),
    "iwae_dp_unique_id": (c_int, [c_void_p]),
    "iwae_dp_init": (c_int, [H, c_int, c_int, c_void_p]),
    "iwae_dp_broadcast_state": (c_int, [H]),
    "iwae_dp_world": (c_int, [H, POINTER(c_int), POINTER(c_int)]),
    "iwae_grad_moments": (c_int, [H, FP, FP]),
    "iwae_export_internal": (c_int, [H, FP, FP, c_longlong]),
    "iwae_log_weights": (c_int, [H, FP, c_int, c_int, FPP, c_int, FP]),
    "iwae_bound": (c_int, [H, POINTER(IwaeLossConfig), FP, c_int, FPP, c_int, FP]),
    "iwae_e_log_px": (c_int, [H, FP, c_int, c_int, FPP, c_int, FP]),
    "iwae_nll": (c_int, [H, FP, c_int, c_int, c_int, FP]),
    "iwae_nll_partials": (c_int, [H, FP, c_int, c_int, c_int, FP, FP]),
    "iwae_nll_eps": (c_int, [H, FP, c_int, c_int, FPP, c_int, FP]),
    "iwae_encoder_means": (c_int, [H, FP, c_int, c_int, FPP, c_int, FPP, c_int]),
    "iwae_reconstruct": (c_int, [H, FP, c_int, FPP, c_int, FP, c_int, FP]),
    "iwae_nll_masked": (c_int, [H, FP, c_int, c_int, FPP, c_int, FPP, c_int, FP]),
    "iwae_debug_gemm": (c_int, [H, FP, c_int, FP, c_int, FP, c_int, c_int, c_int, c_int]),
    "iwae_workspace_bytes": (c_double, [H]),
    "iwae_debug_count": (c_longlong, [H, c_int]),
    "iwae_profile_gemm": (c_int, [H, c_int, c_int]),
    "iwae_profile_read": (c_int, [H, POINTER(c_double), POINTER(c_double), POINTER(c_longlong)]),
    "iwae_profile_replay": (c_int, [H, c_int, POINTER(c_double), POINTER(c_double)]),
}

_lib = None


class IwaeError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load and type the HIP library.  Raises if it is absent: the product
    path has no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("IWAE_HIP_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise ImportError(
            f"{LIB_NAME} not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(lib, h, rc):
    if rc != 0:
        msg = lib.iwae_last_error(h)
        msg = msg.decode() if msg else "unknown error"
        if rc == -1:
            raise ValueError(msg)
        raise IwaeError(f"libiwae_hip error {rc}: {msg}")


def fptr(t) -> "ctypes.POINTER(c_float)":
    """float* from a torch tensor (device or host) or None."""
    if t is None:
        return None
    return ctypes.cast(ctypes.c_void_p(t.data_ptr()), FP)


def fptr_array(tensors):
    if not tensors:
        return None, 0
    # an array of float* is accepted where float** is declared and keeps itself alive
    arr = (FP * len(tensors))(*[fptr(t) for t in tensors])
    return arr, len(tensors)
