"""torch.* cast lists (reference: apex/amp/lists/torch_overrides.py:7-136).

The bmm family is on the low-precision list unconditionally: the reference keys it on
``torch.version.cuda`` and therefore never casts it on ROCm; on MI355X batched GEMMs
are exactly what the MFMA units are for.
"""
import torch

MODULE = torch

FP16_FUNCS = ["conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
              "conv_tbc", "prelu", "addmm", "addmv", "addr", "matmul", "mm", "mv", "addbmm", "baddbmm", "bmm",
              "einsum", "chain_matmul"]
BFLOAT16_FUNCS = [f for f in FP16_FUNCS if f != "prelu"]
FP32_FUNCS = ["acos", "asin", "cosh", "erfinv", "exp", "expm1", "log", "log10", "log2", "log1p", "reciprocal",
              "rsqrt", "sinh", "tan", "pow", "cumprod", "cumsum", "dist", "norm", "prod", "std", "sum", "var",
              "renorm", "softmax", "log_softmax", "layer_norm", "group_norm", "batch_norm", "cdist"]
CASTS = ["addcdiv", "addcmul", "atan2", "cross", "bilinear", "dot", "add", "div", "mul", "eq", "equal", "ge",
         "gt", "le", "lt", "ne", "sub", "where"]
SEQUENCE_CASTS = ["cat", "stack"]
