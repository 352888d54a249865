"""Fused optimizers vs torch.optim / in-test references over 7 steps (reference:
tests/L0/run_optimizers/test_fused_optimizer.py, test_lamb.py)."""
import math

import pytest
import torch

from beforeholiday_amd.optimizers import (FusedAdagrad, FusedAdam, FusedLAMB, FusedLARS, FusedMixedPrecisionLamb,
                                          FusedNovoGrad, FusedSGD)

from conftest import devices


def _params(device, dtype=torch.float32, shapes=((35, 53), (17,), (4, 8, 3, 3), (10001,)), seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).to(dtype).to(device).requires_grad_(True) for s in shapes]


def _clone(ps):
    return [p.detach().clone().requires_grad_(True) for p in ps]


def _run(ref_cls, ref_kw, fused_cls, fused_kw, device, dtype=torch.float32, steps=7, tol=1e-5):
    ps = _params(device, dtype)
    qs = _clone(ps)
    ref = ref_cls([{"params": qs}], **ref_kw)
    fused = fused_cls([{"params": ps}], **fused_kw)
    for s in range(steps):
        g = torch.Generator().manual_seed(100 + s)
        for p, q in zip(ps, qs):
            gr = torch.randn(p.shape, generator=g).to(dtype).to(device)
            p.grad = gr.clone()
            q.grad = gr.clone()
        ref.step()
        fused.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.float(), q.float(), rtol=tol, atol=tol)


class RefLAMB(torch.optim.Optimizer):
    """LAMB reference (same math as tests/L0/run_optimizers/test_lamb.py, global grad-norm clip)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0,
                 adam_w_mode=True, use_nvlamb=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_grad_norm, self.adam_w_mode, self.use_nvlamb = max_grad_norm, adam_w_mode, use_nvlamb

    @torch.no_grad()
    def step(self):
        gn = torch.sqrt(sum((p.grad.float() ** 2).sum() for g in self.param_groups for p in g["params"]))
        clip = gn / self.max_grad_norm if gn > self.max_grad_norm else 1.0
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["m"] = torch.zeros_like(p, dtype=torch.float32)
                    st["v"] = torch.zeros_like(p, dtype=torch.float32)
                st["step"] += 1
                g = p.grad.float() / clip
                pf = p.float()
                if not self.adam_w_mode:
                    g = g + group["weight_decay"] * pf
                st["m"].mul_(b1).add_(g, alpha=1 - b1)
                st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
                mh = st["m"] / (1 - b1 ** st["step"])
                vh = st["v"] / (1 - b2 ** st["step"])
                u = mh / (vh.sqrt() + group["eps"])
                if self.adam_w_mode:
                    u = u + group["weight_decay"] * pf
                ratio = group["lr"]
                if self.use_nvlamb or group["weight_decay"] != 0:
                    pn, un = pf.norm(), u.norm()
                    if pn > 0 and un > 0:
                        ratio = group["lr"] * float(pn / un)
                p.copy_((pf - ratio * u).to(p.dtype))


class RefNovoGrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.95, 0.98), eps=1e-8, weight_decay=0.0, reg_inside_moment=False,
                 norm_type=2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.inside, self.norm_type = reg_inside_moment, norm_type

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                st = self.state[p]
                g = p.grad.float()
                n = g.norm() if self.norm_type == 2 else g.abs().max()
                if not st:
                    st["step"], st["m"], st["v"] = 0, torch.zeros_like(g), n.clone()
                st["step"] += 1
                st["v"] = torch.sqrt(b2 * st["v"] ** 2 + (1 - b2) * n ** 2) if self.norm_type == 2 else b2 * st["v"] + (1 - b2) * n
                bc1 = 1 - b1 ** st["step"]
                bc2 = math.sqrt(1 - b2 ** st["step"])
                denom = st["v"] / bc2 + group["eps"]
                if self.inside:
                    g = g / denom + group["weight_decay"] * p.float()
                    st["m"].mul_(b1).add_(g, alpha=1 - b1)
                    p.sub_(group["lr"] * st["m"] / bc1)
                else:
                    st["m"].mul_(b1).add_(g, alpha=1 - b1)
                    p.sub_(group["lr"] * ((st["m"] / bc1) / denom + group["weight_decay"] * p.float()))


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("adam_w_mode", [True, False])
@pytest.mark.parametrize("wd", [0.0, 0.05])
def test_fused_adam(device, adam_w_mode, wd):
    ref = torch.optim.AdamW if adam_w_mode else torch.optim.Adam
    _run(ref, dict(lr=1e-3, weight_decay=wd, eps=1e-8), FusedAdam,
         dict(lr=1e-3, weight_decay=wd, adam_w_mode=adam_w_mode), device)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_adam_low_precision(device, dtype):
    if device == "cpu":
        pytest.skip("16-bit params are a GPU path")
    # 16-bit params keep fp32 moments (fp16 moments underflow -> inf, see fused_adam.py): compare with
    # torch AdamW on fp32 copies; only the per-step rounding of the stored params differs.
    ps = _params(device, dtype)
    qs = [p.detach().float().clone().requires_grad_(True) for p in ps]
    fused = FusedAdam(ps, lr=1e-3, weight_decay=0.01)
    ref = torch.optim.AdamW(qs, lr=1e-3, weight_decay=0.01)
    for s in range(7):
        for p, q in zip(ps, qs):
            g = torch.randn(q.shape, device=device)
            p.grad, q.grad = g.to(dtype), g.to(dtype).float()
        fused.step()
        ref.step()
        with torch.no_grad():
            for p, q in zip(ps, qs):
                q.copy_(q.to(dtype).float())
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.float(), q, rtol=1e-2, atol=1e-2)
        assert fused.state[p]["exp_avg"].dtype == torch.float32


@pytest.mark.gpu
def test_fused_adam_master_weights_and_capturable():
    ps = _params("cuda", torch.bfloat16)
    qs = [p.detach().float().clone().requires_grad_(True) for p in ps]
    fused = FusedAdam(ps, lr=1e-3, master_weights=True, capturable=True)
    ref = torch.optim.AdamW(qs, lr=1e-3, weight_decay=0.0)
    for s in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(q)
            p.grad, q.grad = g.to(p.dtype), g.to(p.dtype).float()
        fused.step()
        ref.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(fused.state[p]["master_param"], q, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(p.float(), q.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("nesterov,momentum,wd", [(False, 0.0, 0.0), (False, 0.9, 1e-4), (True, 0.9, 1e-4)])
def test_fused_sgd(device, nesterov, momentum, wd):
    _run(torch.optim.SGD, dict(lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=wd), FusedSGD,
         dict(lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=wd), device)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("adam_w_mode,nvlamb,wd", [(True, False, 0.01), (False, False, 0.01), (True, True, 0.0)])
@pytest.mark.parametrize("max_grad_norm", [1.0, 100.0])
def test_fused_lamb(device, adam_w_mode, nvlamb, wd, max_grad_norm):
    _run(RefLAMB, dict(lr=1e-2, weight_decay=wd, max_grad_norm=max_grad_norm, adam_w_mode=adam_w_mode,
                       use_nvlamb=nvlamb), FusedLAMB,
         dict(lr=1e-2, weight_decay=wd, max_grad_norm=max_grad_norm, adam_w_mode=adam_w_mode, use_nvlamb=nvlamb),
         device, tol=2e-5)


@pytest.mark.parametrize("device", devices())
def test_fused_mixed_precision_lamb(device):
    _run(RefLAMB, dict(lr=1e-2, weight_decay=0.01), FusedMixedPrecisionLamb, dict(lr=1e-2, weight_decay=0.01),
         device, tol=2e-5)


@pytest.mark.gpu
def test_fused_mixed_precision_lamb_reduced_precision():
    ps = _params("cuda", torch.bfloat16)
    qs = [p.detach().float().clone().requires_grad_(True) for p in ps]
    fused = FusedMixedPrecisionLamb(ps, lr=1e-2, weight_decay=0.01, reduced_precision_dtype=torch.bfloat16)
    ref = RefLAMB(qs, lr=1e-2, weight_decay=0.01)
    for s in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(q).to(torch.bfloat16)
            p.grad, q.grad = g, g.float()
        fused.step()
        ref.step()
    for p, q, pf in zip(ps, qs, fused.param_groups_full_precision[0]["params"]):
        torch.testing.assert_close(pf, q, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(p.float(), q.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("reg_inside_moment", [False, True])
@pytest.mark.parametrize("norm_type", [2, 0])
def test_fused_novograd(device, reg_inside_moment, norm_type):
    _run(RefNovoGrad, dict(lr=1e-2, weight_decay=0.01, reg_inside_moment=reg_inside_moment, norm_type=norm_type),
         FusedNovoGrad, dict(lr=1e-2, betas=(0.95, 0.98), weight_decay=0.01, reg_inside_moment=reg_inside_moment,
                             norm_type=norm_type), device, tol=1e-4)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adagrad(device, wd):
    _run(torch.optim.Adagrad, dict(lr=1e-2, weight_decay=wd, eps=1e-10), FusedAdagrad,
         dict(lr=1e-2, weight_decay=wd, eps=1e-10), device)


class RefLARS(torch.optim.Optimizer):
    def __init__(self, params, lr, momentum=0.9, weight_decay=1e-4, trust_coefficient=0.001, eps=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay))
        self.tc, self.eps, self.nesterov = trust_coefficient, eps, nesterov

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state[p]
                if "mom" not in st:
                    st["mom"] = torch.zeros_like(p)
                pn, gn = p.norm(), p.grad.norm()
                trust = self.tc * pn / (gn + pn * group["weight_decay"] + self.eps) if (pn > 0 and gn > 0) else 1.0
                lr = group["lr"] * float(trust)
                g = p.grad + group["weight_decay"] * p
                st["mom"] = st["mom"] * group["momentum"] - lr * g
                p.add_(st["mom"] * group["momentum"] - lr * g if self.nesterov else st["mom"])


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("nesterov", [False, True])
def test_fused_lars(device, nesterov):
    _run(RefLARS, dict(lr=0.1, nesterov=nesterov), FusedLARS,
         dict(lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=nesterov), device, tol=1e-5)


@pytest.mark.parametrize("device", devices())
def test_set_grad_none_and_state_dict(device):
    ps = _params(device)
    opt = FusedAdam(ps, lr=1e-3)
    for p in ps:
        p.grad = torch.ones_like(p)
    opt.step()
    sd = opt.state_dict()
    opt2 = FusedAdam(_clone(ps), lr=1e-3)
    opt2.load_state_dict(sd)
    assert opt2.param_groups[0]["step"] == 1
    opt.zero_grad()
    assert all(p.grad is None for p in ps)


def _ab_params(seed):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(8, 6, 3, 3, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    return [torch.randn(33, 17, generator=g).cuda(), torch.randn(5, generator=g).cuda(), w,
            torch.randn(4097, generator=g).cuda()]


@pytest.mark.gpu
@pytest.mark.parametrize("cls,kw", [
    (FusedLAMB, dict(lr=1e-2, weight_decay=0.01, max_grad_norm=1.0)),
    (FusedLAMB, dict(lr=1e-2, weight_decay=0.0, use_nvlamb=True, adam_w_mode=False)),
    (FusedAdam, dict(lr=1e-3, weight_decay=0.01)),
    (FusedAdam, dict(lr=1e-3, weight_decay=0.0, master_weights=True)),
])
def test_native_param_table_matches_list_path(cls, kw):
    """The native ParamTable step (one host call) against the per-step tensor-list path: identical
    kernels, so bit-identical results -- through a parameter that gets its first gradient late, a
    channels_last parameter whose gradient arrives contiguous, a second param group added mid-run and
    a state_dict round trip."""
    dtype = torch.bfloat16 if kw.get("master_weights") else torch.float32
    runs = []
    for native in (True, False):
        ps = [p.to(dtype).requires_grad_(True) for p in _ab_params(0)]
        opt = cls([{"params": ps[:3]}], **kw)
        opt.native_table = native
        extra = None
        for s in range(6):
            g = torch.Generator().manual_seed(50 + s)
            for i, p in enumerate(ps[:3]):
                if i == 1 and s < 2:
                    p.grad = None  # first gradient only at step 2
                    continue
                p.grad = torch.randn(p.shape, generator=g).to(dtype).cuda().contiguous()
            if extra is not None:
                extra.grad = torch.randn(extra.shape, generator=g).to(dtype).cuda()
            opt.step()
            if s == 2:
                extra = ps[3]
                opt.add_param_group({"params": [extra], "lr": 5e-3})
            if s == 3:
                sd = opt.state_dict()
                opt.load_state_dict(sd)
        runs.append([p.detach().float().clone() for p in ps])
    for a, b in zip(*runs):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
