"""Legacy FusedAdam with explicit ``grads`` / ``output_params`` / ``scale`` / ``grad_norms``
(reference: apex/contrib/optimizers/fused_adam.py:6-200, ``fused_adam_cuda``).

Runs the deprecated ``fused_adam_cuda`` kernels (kernels/legacy_optim.hip) with the reference's
update rule: ``step_size = lr*sqrt(1-b2^t)/(1-b1^t)``, ``p -= step_size*(m/denom + wd*p)``,
``denom = sqrt(v + eps)`` (``eps_inside_sqrt``) or ``sqrt(v) + eps``; the reduced-precision
``output_params`` copy is written in the same pass. ``use_mt`` launches one multi-tensor kernel per
group (lists p, m, v, g[, out]).
"""
import torch

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import fused_adam_cuda
from ._legacy import group_lists


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0.0, max_grad_norm=0.0, amsgrad=False, use_mt=False, amp_scale_adjustment=1.0):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self._use_multi_tensor = use_mt
        self._amp_scale_adjustment = amp_scale_adjustment

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        loss = closure() if closure is not None else None
        if hasattr(self, "_amp_stash"):
            grads = self._amp_stash.grads
            output_params = self._amp_stash.output_params
            scale = self._amp_stash.scale * self._amp_scale_adjustment
            grad_norms = self._amp_stash.grad_norms
        n = len(self.param_groups)
        grads_group = group_lists(grads, n)
        out_group = group_lists(output_params, n)
        grad_norms = grad_norms if grad_norms is not None else [None] * n
        for group, g_this, o_this, gnorm in zip(self.param_groups, grads_group, out_group, grad_norms):
            g_this = g_this or [None] * len(group["params"])
            o_this = o_this or [None] * len(group["params"])
            combined = float(scale)
            if group["max_grad_norm"] > 0 and gnorm is not None:
                # the norm is of the scaled gradients
                clip = ((float(gnorm) / scale) + 1e-6) / group["max_grad_norm"]
                if clip > 1:
                    combined = clip * scale
            beta1, beta2 = group["betas"]
            bias_correction = 1 if group["bias_correction"] else 0
            mt_lists, mt_dev, has_out = [[], [], [], [], []], None, False
            for p, g, o in zip(group["params"], g_this, o_this):
                if p.grad is None and g is None:
                    continue
                g = p.grad if g is None else g
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients, please consider SparseAdam instead")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                if self._use_multi_tensor:
                    if mt_dev is not None and p.device != mt_dev:
                        raise RuntimeError("FusedAdam does not support use_mt with tensors on multiple device")
                    mt_dev = p.device
                    for lst, t in zip(mt_lists, (p, st["exp_avg"], st["exp_avg_sq"], g, o)):
                        lst.append(t)
                    has_out = has_out or o is not None
                    continue
                out_p = o if o is not None else torch.empty(0, dtype=torch.float32, device=p.device)
                fused_adam_cuda.adam(p, out_p, st["exp_avg"], st["exp_avg_sq"], g, group["lr"], beta1, beta2,
                                     group["eps"], combined, st["step"], self.eps_mode, bias_correction,
                                     group["weight_decay"])
            if self._use_multi_tensor and mt_lists[0]:
                if has_out and any(o is None for o in mt_lists[4]):
                    raise RuntimeError("FusedAdam use_mt: output_params must be given for all params or none")
                lists = mt_lists if has_out else mt_lists[:4]
                flag = torch.zeros(1, dtype=torch.int, device=mt_dev)
                multi_tensor_applier(fused_adam_cuda.adam_mt, flag, lists, group["lr"], beta1, beta2, group["eps"],
                                     combined, self.state[mt_lists[0][0]]["step"], self.eps_mode, bias_correction,
                                     group["weight_decay"])
        return loss
