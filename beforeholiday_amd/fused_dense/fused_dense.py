"""Fused dense layers (reference: apex/fused_dense/fused_dense.py:6-111).

``FusedDense``: y = x W^T + b with the bias folded into the GEMM epilogue and the bias gradient
reduced by one HIP pass. ``FusedDenseGeluDense``: dense -> GELU -> dense with the pre-activation kept
for the (correct) dGELU backward fused with the first bias-gradient reduction.
"""
import torch
from torch import nn

from .. import amp
from ..ops import fused_dense as _ops


class FusedDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias):
        ctx.save_for_backward(input, weight)
        return _ops.linear_bias_forward(input, weight, bias)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        return tuple(_ops.linear_bias_backward(input, weight, grad_output))


class DenseNoBiasFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight):
        ctx.save_for_backward(input, weight)
        return torch.matmul(input, weight.t())

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        dy = grad_output.reshape(-1, grad_output.size(-1))
        return grad_output.matmul(weight), dy.t().mm(input.reshape(-1, input.size(-1)))


class FusedDenseGeluDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, weight2, bias2):
        gelu_in, gelu_out, output = _ops.linear_gelu_linear_forward(input, weight, bias, weight2, bias2)
        ctx.save_for_backward(input, weight, weight2, gelu_in, gelu_out)
        shape = list(input.shape[:-1]) + [weight2.size(0)]
        return output.view(shape)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight, weight2, gelu_in, gelu_out = ctx.saved_tensors
        return tuple(_ops.linear_gelu_linear_backward(input, gelu_in, gelu_out, weight, weight2, grad_output))


fused_dense_function = amp.half_function(FusedDenseFunc.apply)
dense_no_bias_function = amp.half_function(DenseNoBiasFunc.apply)
fused_dense_gelu_dense_function = amp.half_function(FusedDenseGeluDenseFunc.apply)


class FusedDense(nn.Module):
    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.randn(out_features, in_features))
        if bias:
            self.bias = nn.Parameter(torch.randn(out_features))
        else:
            self.register_parameter("bias", None)

    def forward(self, input):
        if self.bias is not None:
            return fused_dense_function(input, self.weight, self.bias)
        return dense_no_bias_function(input, self.weight)


class FusedDenseGeluDense(nn.Module):
    """dense1 -> GELU -> dense2 in one autograd node."""

    def __init__(self, in_features, intermediate_features, out_features, bias=True):
        super().__init__()
        assert bias, "DenseGeluDense module without bias is currently not supported"
        self.in_features = in_features
        self.intermediate_features = intermediate_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.randn(intermediate_features, in_features))
        self.bias = nn.Parameter(torch.randn(intermediate_features))
        self.weight2 = nn.Parameter(torch.randn(out_features, intermediate_features))
        self.bias2 = nn.Parameter(torch.randn(out_features))

    def forward(self, input):
        return fused_dense_gelu_dense_function(input, self.weight, self.bias, self.weight2, self.bias2)
