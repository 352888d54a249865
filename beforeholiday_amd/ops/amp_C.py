"""``amp_C``: multi-tensor-apply ops with the reference's module name and call ABI.

GPU tensor lists run the gfx950 kernels of ``beforeholiday_amd._C.amp_C``; CPU lists run the
PyTorch reference in ``ops._ref.multi_tensor``. The device is taken from ``noop_flag`` (every op
receives it), exactly like the reference kernels which require it on the tensors' device.
"""
from __future__ import annotations

from .._native import submodule
from ._ref import multi_tensor as _ref

__all__ = [
    "multi_tensor_scale", "multi_tensor_sgd", "multi_tensor_axpby", "multi_tensor_l2norm",
    "multi_tensor_l2norm_mp", "multi_tensor_l2norm_scale", "multi_tensor_norm_out",
    "multi_tensor_lamb_stage1_cuda", "multi_tensor_lamb_stage2_cuda", "multi_tensor_adam",
    "multi_tensor_adam_capturable", "multi_tensor_adagrad", "multi_tensor_novograd",
    "multi_tensor_lamb", "multi_tensor_lamb_mp", "multi_tensor_lars",
]


def _make(name):
    ref = getattr(_ref, name)

    def op(chunk_size, noop_flag, tensor_lists, *args, **kwargs):
        if noop_flag.is_cuda:
            return getattr(submodule("amp_C"), name)(chunk_size, noop_flag, tensor_lists, *args, **kwargs)
        return ref(chunk_size, noop_flag, tensor_lists, *args, **kwargs)

    op.__name__ = name
    op.__qualname__ = name
    op.__doc__ = f"amp_C.{name} (reference ABI: csrc/amp_C_frontend.cpp). GPU: native HIP; CPU: torch reference."
    return op


for _n in __all__:
    globals()[_n] = _make(_n)
del _n

_scale_float = multi_tensor_scale  # noqa: F821


def multi_tensor_scale(chunk_size, noop_flag, tensor_lists, scale):  # noqa: F811
    """out = in * scale. ``scale`` may be a 1-element GPU tensor: it is then read on the device
    (no host synchronisation), e.g. a gradient-clipping coefficient."""
    import torch
    if isinstance(scale, torch.Tensor):
        if noop_flag.is_cuda:
            return submodule("amp_C").multi_tensor_scale_tensor(chunk_size, noop_flag, tensor_lists,
                                                                scale.reshape(1).float())
        scale = float(scale)
    return _scale_float(chunk_size, noop_flag, tensor_lists, scale)
