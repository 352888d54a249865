"""out = in1[idx1] * in2 with fused backward and double backward
(reference: apex/contrib/index_mul_2d/index_mul_2d.py:5-145). fp32 / fp16 (and bf16 here)."""
import torch

from ..._native import submodule


def _ops():
    return submodule("fused_index_mul_2d")


def _check(in1, in2, idx1):
    assert in2.size(0) == idx1.size(0)
    if in1.dtype not in (torch.float32, torch.half, torch.bfloat16) or in2.dtype != in1.dtype:
        raise RuntimeError("input1'dtype and input2's dtype must be fp32 or fp16. And input type must be same")
    if in1.dim() != 2 or in2.dim() != 2:
        raise RuntimeError("in1 and in2 must be 2-dimension tensor.")
    if idx1.dim() != 1:
        raise RuntimeError("idx1 must be 1-dimension tensor.")


class IndexMul2d_(torch.autograd.Function):
    @staticmethod
    def forward(ctx, in1: torch.Tensor, in2: torch.Tensor, idx1: torch.Tensor) -> torch.Tensor:
        _check(in1, in2, idx1)
        in1, in2, idx1 = in1.contiguous(), in2.contiguous(), idx1.contiguous().long()
        if in1.is_cuda:
            out = torch.empty_like(in2)
            _ops().forward(out, in1, in2, idx1)
        else:
            out = in1[idx1] * in2
        ctx.for_backwards = (in1, in2, idx1)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        in1, in2, idx1 = ctx.for_backwards
        grad_in1, grad_in2 = index_mul_2d_backward(in1, in2, idx1, grad_out)
        return grad_in1, grad_in2, None


class IndexMul2dBackward_(torch.autograd.Function):
    @staticmethod
    def forward(ctx, in1, in2, idx1, grad_out):
        grad_out = grad_out.contiguous()
        if in1.is_cuda:
            grad_in1 = torch.zeros_like(in1)
            grad_in2 = torch.empty_like(in2)
            _ops().backward(grad_in1, grad_in2, grad_out, in1, in2, idx1)
        else:
            grad_in1 = torch.zeros_like(in1).index_add_(0, idx1, grad_out * in2)
            grad_in2 = grad_out * in1[idx1]
        ctx.for_backwards = (in1, in2, idx1, grad_out)
        return grad_in1, grad_in2

    @staticmethod
    def backward(ctx, grad_grad_in1, grad_grad_in2):
        in1, in2, idx1, grad_out = ctx.for_backwards
        grad_grad_in1 = grad_grad_in1.contiguous()
        grad_grad_in2 = grad_grad_in2.contiguous()
        if in1.is_cuda:
            grad_in1 = torch.zeros_like(in1)
            grad_in2 = torch.empty_like(in2)
            grad_grad_out = torch.empty_like(grad_out)
            _ops().backward_backward(grad_grad_out, grad_in1, grad_in2, grad_out, grad_grad_in1, grad_grad_in2, in1,
                                     in2, idx1)
        else:
            grad_grad_out = grad_grad_in1[idx1] * in2 + grad_grad_in2 * in1[idx1]
            grad_in1 = torch.zeros_like(in1).index_add_(0, idx1, grad_grad_in2 * grad_out)
            grad_in2 = grad_grad_in1[idx1] * grad_out
        return grad_in1, grad_in2, None, grad_grad_out


index_mul_2d = IndexMul2d_.apply
index_mul_2d_backward = IndexMul2dBackward_.apply
