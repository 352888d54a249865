"""torch.Tensor method cast lists (reference: apex/amp/lists/tensor_overrides.py:14-67)."""
import torch

from . import torch_overrides

MODULE = torch.Tensor


def _filter(names):
    return [n for n in names if hasattr(MODULE, n)]


FP16_FUNCS = _filter(["__matmul__"])
BFLOAT16_FUNCS = _filter(["__matmul__"])
FP32_FUNCS = _filter(["__ipow__", "__pow__", "__rpow__", "cpu"])
CASTS = _filter(["__add__", "__div__", "__eq__", "__ge__", "__gt__", "__iadd__", "__idiv__", "__imul__",
                 "__isub__", "__itruediv__", "__le__", "__lt__", "__mul__", "__ne__", "__radd__", "__rdiv__",
                 "__rmul__", "__rsub__", "__rtruediv__", "__sub__", "__truediv__"])
SEQUENCE_CASTS = []

for _name in ["FP16_FUNCS", "BFLOAT16_FUNCS", "FP32_FUNCS", "CASTS", "SEQUENCE_CASTS"]:
    _lst = globals()[_name]
    for _fn in getattr(torch_overrides, _name):
        if hasattr(MODULE, _fn) and _fn not in _lst:
            _lst.append(_fn)
