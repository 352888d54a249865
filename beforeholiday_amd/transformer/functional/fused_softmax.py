"""Fused scale + mask + softmax (reference: apex/transformer/functional/fused_softmax.py).

The HIP kernels schedule each row independently (a wave per row up to sk 4096, a workgroup per row
beyond), so ``is_kernel_available`` only requires a 16-bit input, a supported mask type and
16 < sk <= 32768 -- none of the reference's divisibility / batch-per-block constraints, and no
4096 cap for padding masks. The generic variant's backward works.
"""
from __future__ import annotations

import torch

from ..._autocast_utils import _cast_if_autocast_enabled
from ...ops import softmax as _sm
from ..enums import AttnMaskType


class ScaledUpperTriangMaskedSoftmax(torch.autograd.Function):
    """scale -> causal (upper-triangular) mask -> softmax over [attn_batches, sq, sk]."""

    @staticmethod
    def forward(ctx, inputs, scale):
        scale_t = torch.tensor([scale])
        softmax_results = _sm.scaled_upper_triang_masked_softmax_forward(inputs, scale)
        ctx.save_for_backward(softmax_results, scale_t)
        return softmax_results

    @staticmethod
    def backward(ctx, output_grads):
        softmax_results, scale_t = ctx.saved_tensors
        return _sm.scaled_upper_triang_masked_softmax_backward(output_grads, softmax_results, float(scale_t[0])), None


def scaled_upper_triang_masked_softmax(inputs, _, scale):
    b, np_, sq, sk = inputs.size()
    assert sq == sk, "causal mask is only for self attention"
    inputs = inputs.reshape(-1, sq, sk)
    args = _cast_if_autocast_enabled(inputs, scale)
    with torch.amp.autocast("cuda", enabled=False):
        probs = ScaledUpperTriangMaskedSoftmax.apply(*args)
    return probs.view(b, np_, sq, sk)


class ScaledMaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, mask, scale):
        scale_t = torch.tensor([scale])
        softmax_results = _sm.scaled_masked_softmax_forward(inputs, mask, scale)
        ctx.save_for_backward(softmax_results, scale_t)
        return softmax_results

    @staticmethod
    def backward(ctx, output_grads):
        softmax_results, scale_t = ctx.saved_tensors
        return _sm.scaled_masked_softmax_backward(output_grads, softmax_results, float(scale_t[0])), None, None


def scaled_masked_softmax(inputs, mask, scale):
    if mask is not None:
        args = _cast_if_autocast_enabled(inputs, mask, scale)
        with torch.amp.autocast("cuda", enabled=False):
            return ScaledMaskedSoftmax.apply(*args)
    args = _cast_if_autocast_enabled(inputs, scale)
    with torch.amp.autocast("cuda", enabled=False):
        return ScaledSoftmax.apply(*args)


class GenericScaledMaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, mask, scale):
        scale_t = torch.tensor([scale])
        softmax_results = _sm.generic_scaled_masked_softmax_forward(inputs, mask, scale)
        ctx.save_for_backward(softmax_results, scale_t)
        return softmax_results

    @staticmethod
    def backward(ctx, output_grads):
        softmax_results, scale_t = ctx.saved_tensors
        return _sm.generic_scaled_masked_softmax_backward(output_grads, softmax_results, float(scale_t[0])), None, None


def generic_scaled_masked_softmax(inputs, mask, scale):
    args = _cast_if_autocast_enabled(inputs, mask, scale)
    with torch.amp.autocast("cuda", enabled=False):
        return GenericScaledMaskedSoftmax.apply(*args)


class ScaledSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, scale):
        scale_t = torch.tensor([scale])
        softmax_results = _sm.scaled_softmax_forward(inputs, scale)
        ctx.save_for_backward(softmax_results, scale_t)
        return softmax_results

    @staticmethod
    def backward(ctx, output_grads):
        softmax_results, scale_t = ctx.saved_tensors
        return _sm.scaled_softmax_backward(output_grads, softmax_results, float(scale_t[0])), None, None


class FusedScaleMaskSoftmax(torch.nn.Module):
    """scale + mask + softmax, fused when possible, PyTorch otherwise.

    Args: input_in_fp16, input_in_bf16, attn_mask_type (padding/causal), scaled_masked_softmax_fusion,
    mask_func (fallback path), softmax_in_fp32, scale.
    """

    def __init__(self, input_in_fp16, input_in_bf16, attn_mask_type, scaled_masked_softmax_fusion, mask_func,
                 softmax_in_fp32, scale):
        super().__init__()
        self.input_in_fp16 = input_in_fp16
        self.input_in_bf16 = input_in_bf16
        if self.input_in_fp16 and self.input_in_bf16:
            raise RuntimeError("both fp16 and bf16 flags cannot be active at the same time.")
        self.input_in_float16 = self.input_in_fp16 or self.input_in_bf16
        self.attn_mask_type = attn_mask_type
        self.scaled_masked_softmax_fusion = scaled_masked_softmax_fusion
        self.mask_func = mask_func
        self.softmax_in_fp32 = softmax_in_fp32
        self.scale = scale
        if not (self.scale is None or softmax_in_fp32):
            raise RuntimeError("softmax should be in fp32 when scaled")
        if self.scaled_masked_softmax_fusion:
            if self.attn_mask_type == AttnMaskType.causal:
                self.fused_softmax_func = scaled_upper_triang_masked_softmax
            elif self.attn_mask_type == AttnMaskType.padding:
                self.fused_softmax_func = scaled_masked_softmax
            else:
                raise ValueError("Invalid attn_mask_type.")

    def forward(self, input, mask):
        assert input.dim() == 4
        if self.is_kernel_available(mask, *input.size()):
            return self.forward_fused_softmax(input, mask)
        return self.forward_torch_softmax(input, mask)

    def is_kernel_available(self, mask, b, np, sq, sk):
        if not (self.scaled_masked_softmax_fusion and self.input_in_float16):
            return False
        if not (self.attn_mask_type == AttnMaskType.causal or
                (self.attn_mask_type == AttnMaskType.padding and mask is not None)):
            return False
        if self.attn_mask_type == AttnMaskType.causal and sq != sk:
            return False
        return 16 < sk <= 32768

    def forward_fused_softmax(self, input, mask):
        scale = self.scale if self.scale is not None else 1.0
        return self.fused_softmax_func(input, mask, scale)

    def forward_torch_softmax(self, input, mask):
        if self.input_in_float16 and self.softmax_in_fp32:
            input = input.float()
        if self.scale is not None:
            input = input * self.scale
        mask_output = self.mask_func(input, mask) if mask is not None else input
        probs = torch.nn.Softmax(dim=-1)(mask_output)
        if self.input_in_float16 and self.softmax_in_fp32:
            probs = probs.half() if self.input_in_fp16 else probs.bfloat16()
        return probs

    @staticmethod
    def get_batch_per_block(sq, sk, b, np):
        return _sm.get_batch_per_block(sq, sk, b, np)


class GenericFusedScaleMaskSoftmax(FusedScaleMaskSoftmax):
    """Padding-mask softmax for arbitrary sk through the generic kernel."""

    def __init__(self, input_in_fp16, input_in_bf16, scaled_masked_softmax_fusion, mask_func, softmax_in_fp32, scale):
        super().__init__(input_in_fp16, input_in_bf16, AttnMaskType.padding, scaled_masked_softmax_fusion, mask_func,
                         softmax_in_fp32, scale)
        self.scaled_masked_softmax_fusion = generic_scaled_masked_softmax

    def is_kernel_available(self, mask, b, np, sq, sk):
        return bool(self.scaled_masked_softmax_fusion) and self.input_in_float16 and 0 < sk

    def forward_fused_softmax(self, input, mask):
        scale = self.scale if self.scale is not None else 1.0
        return generic_scaled_masked_softmax(input, mask, scale)
