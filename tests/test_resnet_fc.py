"""The fused ResNet's classifier on the MFMA GEMM (models/resnet.py ``_FcFn``, ``gemm.mm_nt``): output
and the three gradients against an fp32 ``F.linear`` reference, with the class dimension padded to a
multiple of 8 (10-way) and not (1000-way); repeated calls are bitwise identical."""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("n_cls", [10, 1000])
def test_fc_mfma_matches_fp32(n_cls, dt):
    from beforeholiday_amd.models.resnet import _FcFn

    torch.manual_seed(3)
    x = torch.randn(256, 2048, device="cuda").to(dt).requires_grad_()
    w = (torch.randn(n_cls, 2048, device="cuda") * 0.02).to(dt).requires_grad_()
    b = (torch.randn(n_cls, device="cuda") * 0.1).to(dt).requires_grad_()
    gy = torch.randn(256, n_cls, device="cuda").to(dt)
    y = _FcFn.apply(x, w, b)
    y.backward(gy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(gy.float())
    tol = dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=5e-3, atol=5e-3)
    assert y.shape == (256, n_cls) and y.dtype == dt
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=tol["rtol"], atol=tol["atol"] * 16)
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=tol["rtol"], atol=tol["atol"] * 16)
    g0 = (y.detach().clone(), x.grad.clone(), w.grad.clone())
    x.grad = w.grad = b.grad = None
    y2 = _FcFn.apply(x, w, b)
    y2.backward(gy)
    assert torch.equal(y2, g0[0]) and torch.equal(x.grad, g0[1]) and torch.equal(w.grad, g0[2])


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(256, 64), (1024, 256), (2048, 512), (1000, 2048), (8, 4096), (200, 72)])
def test_transpose16_kernel(shape, dt):
    from beforeholiday_amd._native import submodule

    x = torch.randn(*shape, device="cuda").to(dt)
    assert torch.equal(submodule("gemm").transpose(x), x.t().contiguous())
