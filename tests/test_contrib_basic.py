"""contrib: focal loss, index_mul_2d, clip_grad, FastLayerNorm vs PyTorch references
(reference tests: apex/contrib/test/{focal_loss,index_mul_2d,clip_grad,layer_norm})."""
import pytest
import torch
import torch.nn.functional as F

from tests.conftest import devices


def _sigmoid_focal_sum(x, y, alpha, gamma):
    """torchvision.ops.sigmoid_focal_loss(reduction='sum') written out (torchvision not installed)."""
    p = torch.sigmoid(x)
    ce = F.binary_cross_entropy_with_logits(x, y, reduction="none")
    p_t = p * y + (1 - p) * (1 - y)
    loss = ce * ((1 - p_t) ** gamma)
    alpha_t = alpha * y + (1 - alpha) * (1 - y)
    return (alpha_t * loss).sum()


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_focal_loss(device, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("fp32 on CPU")
    from beforeholiday_amd.contrib.focal_loss import focal_loss
    torch.manual_seed(0)
    N, C, real = 40, 12, 10
    x = torch.randn(N, C, device=device)
    cls = torch.randint(-1, real, (N,), device=device)
    cls[3] = -2  # ignored row
    num_pos = torch.tensor(7.0, device=device)
    xa = x.detach().clone().to(dtype).requires_grad_()
    loss = focal_loss.FocalLoss.apply(xa, cls, num_pos, real, 0.25, 2.0, 0.0)
    keep = cls != -2
    xr = x.detach().clone().requires_grad_()
    y = F.one_hot(cls.clamp(min=0), C).float() * (cls >= 0).float().unsqueeze(1)
    ref = _sigmoid_focal_sum(xr[keep][:, :real], y[keep][:, :real], 0.25, 2.0) / 7.0
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(loss.float(), ref, rtol=tol, atol=tol)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=tol * 10, atol=tol)


@pytest.mark.parametrize("device", devices())
def test_focal_loss_label_smoothing_cpu_gpu_consistency(device):
    from beforeholiday_amd.contrib.focal_loss import focal_loss
    torch.manual_seed(1)
    x = torch.randn(16, 8)
    cls = torch.randint(-1, 8, (16,))
    n = torch.tensor(5.0)
    a = x.clone().requires_grad_()
    la = focal_loss.FocalLoss.apply(a, cls, n, 8, 0.25, 1.5, 0.1)
    la.backward()
    b = x.to(device).requires_grad_()
    lb = focal_loss.FocalLoss.apply(b, cls.to(device), n.to(device), 8, 0.25, 1.5, 0.1)
    lb.backward()
    torch.testing.assert_close(lb.cpu(), la, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(b.grad.cpu(), a.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_index_mul_2d(device, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("fp32 on CPU")
    from beforeholiday_amd.contrib.index_mul_2d import index_mul_2d
    torch.manual_seed(2)
    n1, n, F_ = 17, 50, 33
    in1 = torch.randn(n1, F_, device=device, dtype=dtype, requires_grad=True)
    in2 = torch.randn(n, F_, device=device, dtype=dtype, requires_grad=True)
    idx = torch.randint(0, n1, (n,), device=device)
    r1 = in1.detach().double().requires_grad_()
    r2 = in2.detach().double().requires_grad_()
    out = index_mul_2d(in1, in2, idx)
    ref = r1[idx] * r2
    tol = 1e-5 if dtype == torch.float32 else 5e-3
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol)
    g = torch.randn(n, F_, device=device, dtype=torch.float64)
    # double backward through create_graph
    ga1, ga2 = torch.autograd.grad(out, (in1, in2), g.to(dtype), create_graph=True)
    gr1, gr2 = torch.autograd.grad(ref, (r1, r2), g, create_graph=True)
    torch.testing.assert_close(ga1.double(), gr1, rtol=tol * 10, atol=tol * 10)
    torch.testing.assert_close(ga2.double(), gr2, rtol=tol, atol=tol)
    (ga1.double().sum() + (ga2.double() ** 2).sum()).backward()
    (gr1.sum() + (gr2 ** 2).sum()).backward()
    torch.testing.assert_close(in1.grad.double(), r1.grad, rtol=tol * 10, atol=tol * 10)
    torch.testing.assert_close(in2.grad.double(), r2.grad, rtol=tol * 10, atol=tol * 10)


@pytest.mark.parametrize("device", devices())
def test_clip_grad_norm(device):
    from beforeholiday_amd.contrib.clip_grad import clip_grad_norm_
    torch.manual_seed(3)
    ps = [torch.nn.Parameter(torch.randn(s, device=device)) for s in [(10, 3), (7,), (300,)]]
    ps.append(torch.nn.Parameter(torch.randn(20, device=device, dtype=torch.float16)))
    for p in ps:
        p.grad = torch.randn_like(p) * 3
    ref = [p.grad.detach().clone().float() for p in ps]
    total = clip_grad_norm_(ps, 1.5)
    ref_norm = torch.linalg.norm(torch.stack([torch.linalg.norm(g) for g in ref]))
    torch.testing.assert_close(total.float(), ref_norm, rtol=1e-3, atol=1e-3)
    coef = min(1.0, 1.5 / (ref_norm.item() + 1e-6))
    for p, g in zip(ps, ref):
        torch.testing.assert_close(p.grad.float(), g * coef, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("hidden", [768, 1024, 5120])
def test_fast_layer_norm(device, hidden):
    from beforeholiday_amd.contrib.layer_norm import FastLayerNorm
    torch.manual_seed(4)
    m = FastLayerNorm(hidden).to(device)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    x = torch.randn(6, 5, hidden, device=device, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    w = m.weight.detach().clone().requires_grad_()
    b = m.bias.detach().clone().requires_grad_()
    y = m(x)
    yr = F.layer_norm(xr, (hidden,), w, b, 1e-5)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.weight.grad, w.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(m.bias.grad, b.grad, rtol=1e-3, atol=1e-3)
