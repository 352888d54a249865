"""Legacy FusedAdam with explicit ``grads`` / ``output_params`` / ``scale`` / ``grad_norms``
(reference: apex/contrib/optimizers/fused_adam.py:6-200, ``fused_adam_cuda``).

Runs the capturable multi-tensor Adam kernel: the combined unscale / clip factor is a device scalar
and the reduced-precision output copy is written in the same pass (5th tensor list). The
``eps_inside_sqrt`` variant (update = m / sqrt(v + eps)) is computed with torch ops.
"""
import torch

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C
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
                clip = ((float(gnorm) / scale) + 1e-6) / group["max_grad_norm"]
                if clip > 1:
                    combined = clip * scale
            beta1, beta2 = group["betas"]
            buckets = {}
            for p, g, o in zip(group["params"], g_this, o_this):
                if p.grad is None and g is None:
                    continue
                g = p.grad if g is None else g
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32 if p.dtype != torch.float64 else p.dtype)
                    st["exp_avg_sq"] = torch.zeros_like(st["exp_avg"])
                st["step"] += 1
                key = (g.dtype, p.dtype, None if o is None else o.dtype, st["step"])
                buckets.setdefault(key, [[], [], [], [], []])
                lists = buckets[key]
                lists[0].append(g)
                lists[1].append(p)
                lists[2].append(st["exp_avg"])
                lists[3].append(st["exp_avg_sq"])
                lists[4].append(o)
            for (gdt, pdt, odt, step), lists in buckets.items():
                dev = lists[1][0].device
                if self.eps_mode == 0:
                    self._eps_inside_sqrt(group, lists, step, combined)
                    continue
                use = lists if odt is not None else lists[:4]
                flag = torch.zeros(1, dtype=torch.int, device=dev)
                multi_tensor_applier(amp_C.multi_tensor_adam_capturable, flag, use,
                                     torch.full([1], group["lr"], dtype=torch.float32, device=dev), beta1, beta2,
                                     group["eps"], torch.full([1], step, dtype=torch.int, device=dev), 0,
                                     1 if group["bias_correction"] else 0, group["weight_decay"],
                                     torch.full([1], 1.0 / combined, dtype=torch.float32, device=dev), None)
        return loss

    def _eps_inside_sqrt(self, group, lists, step, combined):
        beta1, beta2 = group["betas"]
        bc1 = 1 - beta1 ** step if group["bias_correction"] else 1.0
        bc2 = 1 - beta2 ** step if group["bias_correction"] else 1.0
        for g, p, m, v, o in zip(*lists):
            gf = g.float() / combined + group["weight_decay"] * p.float()
            m.mul_(beta1).add_(gf, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
            upd = (m / bc1) / torch.sqrt(v / bc2 + group["eps"])
            p.copy_((p.float() - group["lr"] * upd).to(p.dtype))
            if o is not None:
                o.copy_(p.to(o.dtype))
