"""contrib multihead attention vs an explicit per-head PyTorch reference
(reference tests: apex/contrib/test/multihead_attn/test_*_multihead_attn.py, test_mha_fused_softmax.py)."""
import pytest
import torch
import torch.nn.functional as F

from tests.conftest import devices


def _ref_self(x, w_in, b_in, w_out, b_out, heads, pad=None, time=None):
    s, b, e = x.shape
    hd = e // heads
    qkv = F.linear(x, w_in, b_in).view(s, b * heads, 3, hd)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    scores = torch.bmm(q.transpose(0, 1), k.transpose(0, 1).transpose(1, 2)) * hd ** -0.5
    if time is not None:
        scores = scores.masked_fill(time.bool(), float("-inf"))
    if pad is not None:
        scores = scores.view(b, heads, s, s).masked_fill(pad.bool().view(b, 1, 1, s), float("-inf")).view(b * heads, s, s)
    p = torch.softmax(scores, -1)
    ctx = torch.bmm(p, v.transpose(0, 1)).transpose(0, 1).reshape(s, b, e)
    return F.linear(ctx, w_out, b_out)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("impl", ["fast", "default"])
@pytest.mark.parametrize("masking", [None, "pad", "time"])
def test_self_multihead_attn(device, impl, masking):
    from beforeholiday_amd.contrib.multihead_attn import SelfMultiheadAttn
    torch.manual_seed(0)
    s, b, e, h = 24, 3, 64, 4
    m = SelfMultiheadAttn(e, h, dropout=0.0, bias=True, impl=impl).to(device)
    x = torch.randn(s, b, e, device=device, requires_grad=True)
    pad = time = None
    kw = {}
    if masking == "pad":
        pad = torch.zeros(b, s, dtype=torch.bool, device=device)
        pad[1, 20:] = True
        kw["key_padding_mask"] = pad
    elif masking == "time":
        time = torch.triu(torch.ones(s, s, dtype=torch.bool, device=device), 1)
        kw["attn_mask"] = time
    out, _ = m(x, x, x, is_training=True, **kw)
    xr = x.detach().clone().requires_grad_()
    params = [p.detach().clone().requires_grad_() for p in (m.in_proj_weight, m.in_proj_bias, m.out_proj_weight,
                                                            m.out_proj_bias)]
    ref = _ref_self(xr, *params, h, pad, time)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)
    g = torch.randn_like(ref)
    out.backward(g)
    ref.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.in_proj_weight.grad, params[0].grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("device", devices())
def test_self_multihead_attn_norm_add_and_half(device):
    from beforeholiday_amd.contrib.multihead_attn import SelfMultiheadAttn
    torch.manual_seed(1)
    dtype = torch.float16 if device != "cpu" else torch.float32
    s, b, e, h = 16, 2, 32, 4
    m = SelfMultiheadAttn(e, h, dropout=0.0, bias=False, include_norm_add=True, impl="fast").to(device, dtype)
    x = torch.randn(s, b, e, device=device, dtype=dtype, requires_grad=True)
    out, _ = m(x, x, x, is_training=True)
    xr = x.detach().float().requires_grad_()
    ln = F.layer_norm(xr, (e,), m.lyr_nrm_gamma_weights.float(), m.lyr_nrm_beta_weights.float(), 1e-5)
    ref = xr + _ref_self(ln, m.in_proj_weight.float(), None, m.out_proj_weight.float(), None, h)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)
    out.float().sum().backward()
    ref.sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)


@pytest.mark.parametrize("device", devices())
def test_encdec_multihead_attn(device):
    from beforeholiday_amd.contrib.multihead_attn import EncdecMultiheadAttn
    torch.manual_seed(2)
    sq, sk, b, e, h = 10, 14, 2, 32, 4
    m = EncdecMultiheadAttn(e, h, dropout=0.0, bias=False, impl="fast").to(device)
    q = torch.randn(sq, b, e, device=device, requires_grad=True)
    kv = torch.randn(sk, b, e, device=device, requires_grad=True)
    out, _ = m(q, kv, kv, is_training=False)
    hd = e // h
    Q = F.linear(q, m.in_proj_weight_q).view(sq, b * h, hd)
    KV = F.linear(kv, m.in_proj_weight_kv).view(sk, b * h, 2, hd)
    p = torch.softmax(torch.bmm(Q.transpose(0, 1), KV[:, :, 0].transpose(0, 1).transpose(1, 2)) * hd ** -0.5, -1)
    ctx = torch.bmm(p, KV[:, :, 1].transpose(0, 1)).transpose(0, 1).reshape(sq, b, e)
    ref = F.linear(ctx, m.out_proj_weight)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("sk", [40, 512, 1000])
def test_mask_softmax_dropout(device, sk):
    """Dropout: the backward reproduces exactly the mask used in forward (regenerated on GPU)."""
    from beforeholiday_amd.contrib.multihead_attn import fast_mask_softmax_dropout_func
    torch.manual_seed(3)
    heads, b, sq, p = 2, 2, 8, 0.3
    x = torch.randn(b * heads, sq, sk, device=device, requires_grad=True)
    pad = torch.zeros(b, sk, dtype=torch.bool, device=device)
    pad[0, sk // 2:] = True
    y = fast_mask_softmax_dropout_func(True, heads, x, pad, False, p)
    sm = torch.softmax(x.detach().view(b, heads, sq, sk).masked_fill(pad.view(b, 1, 1, sk), float("-inf")), -1)
    sm = sm.view(b * heads, sq, sk)
    keep = (y.detach() != 0) | (sm == 0)
    frac = keep[sm > 0].float().mean().item()
    assert abs(frac - (1 - p)) < 0.05
    torch.testing.assert_close(y.detach()[keep & (sm > 0)], (sm / (1 - p))[keep & (sm > 0)], rtol=1e-5, atol=1e-6)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().clone().requires_grad_()
    smr = torch.softmax(xr.view(b, heads, sq, sk).masked_fill(pad.view(b, 1, 1, sk), float("-inf")), -1)
    yr = smr.view(b * heads, sq, sk) * keep.float() / (1 - p)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-5)
