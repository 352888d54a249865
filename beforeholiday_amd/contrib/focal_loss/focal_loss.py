"""Fused sigmoid focal loss (reference: apex/contrib/focal_loss/focal_loss.py:4-69).

``loss = sum(FL(x, y)) / num_positives_sum`` over [N, C] logits with per-row labels (-1 background,
-2 ignored row; classes >= ``num_real_classes`` are padding). Forward caches the partial gradient
so backward is a single in-place scale (kernels/contrib.hip).
"""
import torch

from ..._native import submodule


def _ref_forward(x, y, num_pos, num_real_classes, alpha, gamma, smoothing):
    xf = x.float()
    C = x.size(-1)
    rows = xf.reshape(-1, C)
    lab = y.reshape(-1)
    cls = torch.arange(C, device=x.device)
    pos = (lab.unsqueeze(1) == cls.unsqueeze(0)) & (lab.unsqueeze(1) >= 0)
    valid = (lab.unsqueeze(1) != -2) & (cls.unsqueeze(0) < num_real_classes)
    s = smoothing
    p = rows
    sigma = torch.sigmoid(p)
    off_a = torch.nn.functional.softplus(-p)
    base = torch.where(pos, (s - s / 2) * p if s > 0 else torch.zeros_like(p), (1 - s / 2) * p if s > 0 else p)
    off_b = torch.where(pos, ((1 - s + s / 2) if s > 0 else 1.0) - sigma, ((s / 2) if s > 0 else 0.0) - sigma)
    f1 = torch.where(pos, torch.full_like(p, alpha), torch.full_like(p, 1 - alpha))
    f2 = torch.where(pos, 1 - sigma, sigma)
    b = torch.where(pos, -gamma * sigma, gamma * (1 - sigma))
    cf = f1 * f2.pow(gamma)
    t = base + off_a
    loss_el = torch.where(valid, cf * t, torch.zeros_like(p))
    grad = torch.where(valid, cf * (b * t - off_b), torch.zeros_like(p))
    loss = loss_el.sum() / num_pos.float().reshape(())
    return loss, grad.reshape(x.shape).to(x.dtype)


class FocalLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cls_output, cls_targets_at_level, num_positives_sum, num_real_classes, alpha, gamma,
                label_smoothing=0.0):
        if cls_output.is_cuda:
            loss, partial_grad = submodule("focal_loss_cuda").forward(
                cls_output, cls_targets_at_level, num_positives_sum, num_real_classes, alpha, gamma, label_smoothing)
        else:
            loss, partial_grad = _ref_forward(cls_output, cls_targets_at_level, num_positives_sum, num_real_classes,
                                              alpha, gamma, label_smoothing)
        ctx.save_for_backward(partial_grad, num_positives_sum)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        partial_grad, num_positives_sum = ctx.saved_tensors
        if partial_grad.is_cuda:
            grad_input = submodule("focal_loss_cuda").backward(grad_loss, partial_grad, num_positives_sum)
        else:
            grad_input = partial_grad * (grad_loss.float() / num_positives_sum.float()).to(partial_grad.dtype)
        return grad_input, None, None, None, None, None, None


def focal_loss(cls_output: torch.Tensor, cls_targets_at_level: torch.Tensor, num_positive_sum: torch.Tensor,
               num_real_classes: int, alpha: float, gamma: float, label_smoothing: float = 0.0) -> torch.Tensor:
    """Fused focal loss function."""
    return FocalLoss.apply(cls_output, cls_targets_at_level, num_positive_sum, num_real_classes, alpha, gamma,
                           label_smoothing)
