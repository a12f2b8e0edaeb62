"""MI355X-native IWAE train-step / k-sample NLL hot path (drop-in for
CharlesArnal/IWAE_replication_project's ``Flexible_Model``).

Compute: libiwae_hip.so (hand-written HIP for gfx950) behind the C ABI in
include/iwae.h.  This package is the host-side mirror of the reference's
Python API; see DESIGN.md.
"""
from .flexible_iwae import (Adam, Flexible_Model, LOSSES, architecture, glorot_weights,  # noqa: F401
                            loss_config, output_bias, resolve_dataset_bias, weight_shapes)
from . import data  # noqa: F401,E402  (local-file loaders, LR-stage driver)

__all__ = ["Adam", "Flexible_Model", "LOSSES", "architecture", "glorot_weights", "loss_config",
           "output_bias", "resolve_dataset_bias", "weight_shapes"]
