"""Fused softmax cross-entropy with label smoothing (reference:
apex/contrib/xentropy/softmax_xentropy.py). Saves only the per-row log-sum-exp; the backward
recomputes the softmax from the logits."""
import torch

from ...ops import softmax as _sm


class SoftmaxCrossEntropyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing=0.0, padding_idx=0, half_to_float=False):
        losses, max_log_sum_exp = _sm.xentropy_forward(logits, labels, smoothing, half_to_float)
        losses.masked_fill_(labels == padding_idx, 0)
        ctx.save_for_backward(logits, max_log_sum_exp, labels)
        ctx.smoothing = smoothing
        ctx.padding_idx = padding_idx
        return losses

    @staticmethod
    def backward(ctx, grad_loss):
        logits, max_log_sum_exp, labels = ctx.saved_tensors
        grad_loss = grad_loss.contiguous().masked_fill(labels == ctx.padding_idx, 0)
        grad_logits = _sm.xentropy_backward(grad_loss, logits, max_log_sum_exp, labels, ctx.smoothing)
        return grad_logits, None, None, None, None
