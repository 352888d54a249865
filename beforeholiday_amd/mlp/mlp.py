"""N-layer MLP in one autograd node (reference: apex/mlp/mlp.py:7-79).

Forward: per layer ONE GEMM with bias + activation in its epilogue -- the MFMA kernel of
kernels/gemm.hip where its static rule picks it (K <= 1024), else hipBLASLt's addmm + one in-place
activation pass (``gemm.linear_act``).
Backward: the last layer's dActivation + bias gradient in one pass; every earlier layer's dActivation
and bias gradient inside the data-gradient GEMM's epilogue (``gemm.linear_dact``); the weight
gradients on MFMA kernels where they apply (``ops.fused_dense.weight_grad``, >= 4096 rows: the
transposed-operand GEMM of kernels/gemm_tn.hip from 1.5M weight elements, the 1x1 weight-gradient kernel
below that), hipBLASLt otherwise.
The activation follows EVERY layer (including the last), like the reference.
"""
import math
from copy import copy

import torch
from torch import nn

from .. import amp
from ..ops import fused_dense as _ops


class MlpFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bias, activation, *args):
        outputs = _ops.mlp_forward(bias, activation, list(args))
        ctx.save_for_backward(*args, *outputs)
        ctx.n_in = len(args)
        ctx.bias = bias
        ctx.activation = activation
        return outputs[-1]

    @staticmethod
    def backward(ctx, grad_o):
        saved = ctx.saved_tensors
        inputs, outputs = list(saved[:ctx.n_in]), list(saved[ctx.n_in:])
        grads = _ops.mlp_backward(ctx.bias, ctx.activation, grad_o.contiguous(), outputs, inputs)
        return (None, None, *grads)


mlp_function = amp.half_function(MlpFunction.apply)


class MLP(torch.nn.Module):
    """MLP(mlp_sizes=[in, h1, ..., out], bias=True, activation='relu'|'sigmoid'|'none')."""

    def __init__(self, mlp_sizes, bias=True, activation="relu"):
        super().__init__()
        self.num_layers = len(mlp_sizes) - 1
        self.mlp_sizes = copy(mlp_sizes)
        self.bias = 1 if bias else 0
        acts = {"none": 0, "relu": 1, "sigmoid": 2}
        if activation not in acts:
            raise TypeError("activation must be relu or none.")
        self.activation = acts[activation]
        self.weights = []
        self.biases = []
        for i in range(self.num_layers):
            w = torch.nn.Parameter(torch.empty(mlp_sizes[i + 1], mlp_sizes[i]))
            self.weights.append(w)
            setattr(self, f"weight_{i}", w)
            if self.bias:
                b = torch.nn.Parameter(torch.empty(mlp_sizes[i + 1]))
                self.biases.append(b)
                setattr(self, f"bias_{i}", b)
        self.reset_parameters()

    def reset_parameters(self):
        for w in self.weights:
            nn.init.normal_(w, 0.0, math.sqrt(2.0 / float(w.size(0) + w.size(1))))
        for b in self.biases:
            nn.init.normal_(b, 0.0, math.sqrt(1.0 / float(b.size(0))))

    def forward(self, input):
        return mlp_function(self.bias, self.activation, input, *self.weights, *self.biases)

    def extra_repr(self):
        return f"MLP sizes: {self.mlp_sizes}, Bias={self.bias}, activation={self.activation}"
