"""beforeholiday_amd -- an MI355X-native (gfx950 / CDNA4) mixed-precision and distributed
training library with the public API of NVIDIA Apex / SkyHeroesS/beforeholiday.

Layout (reference package ``apex`` -> this package):

* ``amp``, ``fp16_utils``                        mixed precision runtime
* ``optimizers``, ``multi_tensor_apply``         fused multi-tensor optimizers (HIP kernels)
* ``normalization``, ``fused_dense``, ``mlp``    fused layers (HIP kernels, MFMA GEMMs)
* ``parallel``                                   DDP / Reducer / SyncBatchNorm / LARC over RCCL
* ``transformer``                                Megatron-style TP/SP/PP
* ``contrib``                                    xentropy, focal loss, MHA, ZeRO optimizers, ...
* ``ops``                                        op-level entry points (amp_C, syncbn, ...)
* ``models``                                     ResNet-50 / BERT / GPT reference workloads
* ``utils``                                      logging, timers, profiling helpers

GPU tensors always run the native extension ``beforeholiday_amd._C`` (built in-tree with
``python -m beforeholiday_amd._build``); CPU tensors run PyTorch reference implementations.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

import logging as _logging

from . import _native  # noqa: F401

# library root logger (reference: apex/__init__.py:27-39); handlers / rank-aware format in utils.logging
_library_root_logger = _logging.getLogger(__name__)
from ._native import available as native_available  # noqa: F401

_SUBMODULES = [
    "ops", "multi_tensor_apply", "optimizers", "amp", "fp16_utils", "normalization", "parallel",
    "fused_dense", "mlp", "transformer", "contrib", "RNN", "models", "utils", "testing",
]


def __getattr__(name):
    if name in _SUBMODULES:
        mod = importlib.import_module(f".{name}", __name__)
        globals()[name] = mod
        return mod
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


def install_apex_aliases():
    """Opt-in: make ``import apex`` / ``import amp_C`` resolve to this package, so code written
    against the reference runs unchanged (``apex.amp``, ``apex.optimizers.FusedLAMB``, ...)."""
    import sys

    sys.modules.setdefault("apex", sys.modules[__name__])
    for sub in _SUBMODULES:
        try:
            sys.modules.setdefault(f"apex.{sub}", importlib.import_module(f".{sub}", __name__))
        except ImportError:
            pass
    from .ops import amp_C, apex_C, distributed_adam_cuda, distributed_lamb_cuda, fused_adam_cuda

    sys.modules.setdefault("amp_C", amp_C)
    sys.modules.setdefault("apex_C", apex_C)
    # python modules with CPU reference paths around the native submodules
    sys.modules.setdefault("fused_adam_cuda", fused_adam_cuda)
    sys.modules.setdefault("distributed_adam_cuda", distributed_adam_cuda)
    sys.modules.setdefault("distributed_lamb_cuda", distributed_lamb_cuda)
    # the reference's other top-level extension modules map onto submodules of the native _C
    if _native.available():
        for ext in ("syncbn", "fused_layer_norm_cuda", "fused_dense_cuda", "mlp_cuda", "fused_weight_gradient_mlp_cuda",
                    "scaled_upper_triang_masked_softmax_cuda", "scaled_masked_softmax_cuda", "scaled_softmax_cuda",
                    "generic_scaled_masked_softmax_cuda", "xentropy_cuda", "focal_loss_cuda", "fused_index_mul_2d",
                    "fast_multihead_attn", "transducer_joint_cuda", "transducer_loss_cuda"):
            try:
                sys.modules.setdefault(ext, _native.submodule(ext))
            except (AttributeError, ImportError):
                pass
