"""contrib FusedLAMB (the deprecated contrib optimizer, reference: apex/contrib/optimizers/fused_lamb.py):
matches the main FusedLAMB on fp32 parameters (same LAMB math, one group, max_grad_norm from defaults),
blends the fp32 and fp16 list norms as sqrt(n32^2 + n16^2), and rejects bf16 as the reference does."""
import pytest
import torch


def _params(dtypes, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i, dt in enumerate(dtypes):
        p = torch.nn.Parameter((torch.randn(17 + 5 * i, 9, generator=g) * 0.3).to(device=device, dtype=dt))
        p.grad = (torch.randn(p.shape, generator=g) * 0.1).to(device=device, dtype=dt)
        out.append(p)
    return out


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_matches_main_fused_lamb_fp32(device):
    from beforeholiday_amd.contrib.optimizers import FusedLAMB as ContribLAMB
    from beforeholiday_amd.optimizers import FusedLAMB

    a = _params([torch.float32] * 3, device)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    for p, q in zip(a, b):
        q.grad = p.grad.clone()
    oa = ContribLAMB(a, lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    ob = FusedLAMB(b, lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    for _ in range(3):
        oa.step()
        ob.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)  # (norm blend: sqrt(n^2) vs n, 1 ulp)
    assert oa.param_groups[0]["step"] == 3


@pytest.mark.gpu
def test_mixed_fp16_fp32_norm_blend_and_bf16_rejected():
    from beforeholiday_amd.contrib.optimizers import FusedLAMB as ContribLAMB

    ps = _params([torch.float32, torch.float16, torch.float32, torch.float16], "cuda", seed=1)
    opt = ContribLAMB(ps, lr=1e-2)
    n = opt._global_grad_norm(torch.device("cuda"))
    n32 = torch.cat([p.grad.float().flatten() for p in ps if p.dtype == torch.float32]).norm()
    n16 = torch.cat([p.grad.float().flatten() for p in ps if p.dtype == torch.float16]).norm()
    torch.testing.assert_close(n, torch.sqrt(n32 * n32 + n16 * n16).reshape(1), rtol=1e-5, atol=1e-6)
    before = [p.detach().clone() for p in ps]
    opt.step()
    assert all(not torch.equal(p, q) for p, q in zip(ps, before))
    bad = _params([torch.bfloat16], "cuda")
    with pytest.raises(RuntimeError, match="fp16 and fp32"):
        ContribLAMB(bad).step()
