"""FusedLayerNorm / FusedRMSNorm vs fp32 PyTorch (reference: tests/L0/run_fused_layer_norm/
test_fused_layer_norm.py -- contiguous & strided inputs, large batch, fp32/fp16/bf16 tolerances,
mixed dtypes, memory-efficient backward)."""
import pytest
import torch
import torch.nn.functional as F

from beforeholiday_amd.normalization import (FusedLayerNorm, FusedRMSNorm, MixedFusedLayerNorm, MixedFusedRMSNorm,
                                             manual_rms_norm)

from conftest import devices

TOL = {torch.float32: (1e-4, 1e-4), torch.float16: (5e-3, 5e-3), torch.bfloat16: (1.6e-2, 2e-2)}


def _ref_ln(x, shape, w, b, eps, rms):
    if rms:
        return manual_rms_norm(x.float(), shape, w.float() if w is not None else None, eps)
    return F.layer_norm(x.float(), shape, w.float() if w is not None else None,
                        b.float() if b is not None else None, eps)


def _check(device, batch, shape, dtype, affine, rms, mem_eff, mixed=False, strided=False):
    torch.manual_seed(0)
    x = (torch.randn(*batch, *shape) * 2 + 0.3)
    if strided:
        x = torch.randn(*batch, *shape[:-1], shape[-1] * 2)[..., ::2]
    x = x.to(device=device, dtype=dtype)
    cls = (MixedFusedRMSNorm if rms else MixedFusedLayerNorm) if mixed else (FusedRMSNorm if rms else FusedLayerNorm)
    kw = {} if mixed else {"elementwise_affine": affine}
    m = cls(shape, eps=1e-5, memory_efficient=mem_eff, **kw).to(device)
    if m.weight is not None:
        with torch.no_grad():
            m.weight.uniform_(0.5, 1.5)
            if getattr(m, "bias", None) is not None:
                m.bias.uniform_(-0.5, 0.5)
    if not mixed:
        m = m.to(dtype)
    xr = x.detach().float().cpu().requires_grad_(True)
    wr = m.weight.detach().float().cpu().requires_grad_(True) if m.weight is not None else None
    br = m.bias.detach().float().cpu().requires_grad_(True) if getattr(m, "bias", None) is not None else None
    yr = _ref_ln(xr, tuple(shape), wr, br, 1e-5, rms)
    xg = x.detach().requires_grad_(True)
    y = m(xg)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.to(device=device, dtype=y.dtype))
    rt, at = TOL[dtype]
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=rt, atol=at)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, rtol=rt * 4, atol=at * 4)
    if wr is not None:
        n = x.numel() // m.weight.numel()
        torch.testing.assert_close(m.weight.grad.float().cpu(), wr.grad, rtol=rt * 4, atol=at * 4 * max(1, n ** 0.5 / 8))
    if br is not None:
        n = x.numel() // m.weight.numel()
        torch.testing.assert_close(m.bias.grad.float().cpu(), br.grad, rtol=rt * 4, atol=at * 4 * max(1, n ** 0.5 / 8))
    if mixed:
        assert y.dtype == m.weight.dtype


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("shape", [(32,), (63,), (768,), (1024,), (4, 256), (5000,), (12288,)])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("affine", [True, False])
def test_fused_norm_fp32(device, shape, rms, affine):
    _check(device, (16, 3), shape, torch.float32, affine, rms, False)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(768,), (1024,), (2048,), (4096,), (8192,), (63,)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("mem_eff", [False, True])
def test_fused_norm_half_gpu(shape, dtype, rms, mem_eff):
    _check("cuda", (37,), shape, dtype, True, rms, mem_eff)


@pytest.mark.gpu
@pytest.mark.parametrize("rms", [False, True])
def test_fused_norm_large_batch_gpu(rms):
    _check("cuda", (65536,), (128,), torch.float16, True, rms, False)


@pytest.mark.gpu
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_mixed_dtypes_gpu(rms, dtype):
    _check("cuda", (8, 5), (1024,), dtype, True, rms, False, mixed=True)


@pytest.mark.parametrize("device", devices())
def test_strided_input(device):
    _check(device, (6,), (128,), torch.float32, True, False, False, strided=True)


@pytest.mark.gpu
def test_autocast_gpu():
    m = FusedLayerNorm(256).cuda()
    x = torch.randn(8, 256, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.dtype == torch.bfloat16


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("n2", [1024, 63, 12288])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_ln_backward_residual_grad(device, n2, dtype):
    """backward_affine(..., dresid): grad_input = LN backward + the residual branch's gradient, summed in
    fp32 in the dx kernel (wave-per-row and long-row kernels), against fp32 PyTorch autograd of
    y = LN(x), loss = <y, dy> + <x, dr>."""
    from beforeholiday_amd.ops import fused_layer_norm_cuda as ln

    if device == "cpu" and dtype != torch.float32:
        dtype_c = torch.float32
    else:
        dtype_c = dtype
    torch.manual_seed(0)
    x = torch.randn(37, n2, device=device).to(dtype_c)
    w = (1 + 0.1 * torch.randn(n2, device=device)).to(dtype_c)
    b = (0.1 * torch.randn(n2, device=device)).to(dtype_c)
    dy = torch.randn(37, n2, device=device).to(dtype_c)
    dr = torch.randn(37, n2, device=device).to(dtype_c)
    out, mean, invvar = ln.forward_affine(x, (n2,), w, b, 1e-5)
    gi, gw, gb = ln.backward_affine(dy, mean, invvar, x, (n2,), w, b, 1e-5, False, dr)
    xr = x.float().requires_grad_()
    wr, br = w.float().requires_grad_(), b.float().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (n2,), wr, br, 1e-5)
    ((yr * dy.float()).sum() + (xr * dr.float()).sum()).backward()
    tol = dict(rtol=2e-2, atol=2e-2) if dtype_c != torch.float32 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gi.float(), xr.grad, **tol)
    torch.testing.assert_close(gw.float(), wr.grad, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(gb.float(), br.grad, rtol=5e-2, atol=5e-2)
    # the same result as the unfused sum, within one rounding of the 16-bit output
    g0 = ln.backward_affine(dy, mean, invvar, x, (n2,), w, b, 1e-5, False)[0]
    torch.testing.assert_close(gi.float(), (g0.float() + dr.float()), rtol=1e-2, atol=1e-2)
