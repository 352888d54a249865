"""``apex_C``: flatten / unflatten (reference: csrc/flatten_unflatten.cpp). Native C++ (ATen) on
every device; the torch._utils helpers when the extension is not built (CPU-only installs)."""
from .._native import available, submodule


def flatten(tensors):
    if available():
        return submodule("apex_C").flatten(list(tensors))
    from torch._utils import _flatten_dense_tensors
    return _flatten_dense_tensors(tensors)


def unflatten(flat, tensors):
    if available():
        return submodule("apex_C").unflatten(flat, list(tensors))
    from torch._utils import _unflatten_dense_tensors
    return _unflatten_dense_tensors(flat, tensors)
