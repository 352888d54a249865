"""MFMA fused short-sequence attention (kernels/attn.hip) vs an fp32 PyTorch reference.

Forward O = dropout(softmax(scale * Q K^T + mask)) V and the backward dQ / dK / dV, with q / k / v
as strided views of a fused [t, B*heads, 3, 64] QKV tensor (the MHA layout). Dropout is checked by
recovering the kernel's keep mask through V = I (O then equals the dropped probabilities) and
running the reference backward with that same mask.
"""
import pytest
import torch

from beforeholiday_amd import config

pytestmark = pytest.mark.gpu


def _fa():
    from beforeholiday_amd._native import submodule

    return submodule("fused_attention")


def _reference(q, k, v, scale, mask_mode, mask, heads, keep=None, p=0.0):
    # q [sq, BH, 64], k/v [sk, BH, 64] fp32 -> [sq, BH, 64]
    s = torch.einsum("qbd,kbd->bqk", q, k) * scale
    BH, sq, sk = s.shape
    if mask_mode == 1:
        s = s.view(-1, heads, sq, sk).masked_fill(mask.view(-1, 1, 1, sk).bool(), float("-inf")).view(BH, sq, sk)
    elif mask_mode == 2:
        s = (s.view(-1, heads, sq, sk) + mask.view(-1, 1, 1, sk).float()).view(BH, sq, sk)
    elif mask_mode == 3:
        s = s.masked_fill(mask.view(1, sq, sk).bool(), float("-inf"))
    pr = torch.softmax(s, -1).nan_to_num(0.0)
    if keep is not None:
        pr = pr * keep / (1 - p)
    return torch.einsum("bqk,kbd->qbd", pr, v)


def _make(sq, sk, B, heads, dtype, mask_mode, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    BH = B * heads
    q_src = torch.randn(sq, BH, 3, 64, device="cuda", dtype=dtype, generator=g)
    kv_src = torch.randn(sk, BH, 3, 64, device="cuda", dtype=dtype, generator=g) if sk != sq else q_src
    q, k, v = q_src[:, :, 0], kv_src[:, :, 1], kv_src[:, :, 2]
    mask = None
    if mask_mode == 1:
        mask = torch.rand(B, sk, device="cuda", generator=g) < 0.3
        mask[0, :] = True  # a fully masked batch row -> zeros
    elif mask_mode == 2:
        mask = torch.randn(B, sk, device="cuda", generator=g)
    elif mask_mode == 3:
        mask = torch.triu(torch.ones(sq, sk, device="cuda", dtype=torch.bool), diagonal=1)
    return q, k, v, mask


SHAPES = [(64, 64), (37, 50), (128, 128), (100, 128), (130, 64), (16, 120)]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mask_mode", [0, 1, 2, 3])
def test_forward_backward_no_dropout(dtype, shape, mask_mode):
    sq, sk = shape
    if mask_mode == 3 and sq != sk:
        pytest.skip("time mask is square in the MHA module")
    B, heads = 3, 2
    q, k, v, mask = _make(sq, sk, B, heads, dtype, mask_mode)
    scale = 64 ** -0.5
    out = _fa().forward(q, k, v, mask_mode, mask, heads, scale, 0.0, True, 123)
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _reference(qf, kf, vf, scale, mask_mode, mask, heads)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)

    dout = torch.randn_like(out)
    ref.backward(dout.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    _fa().backward(dout, q, k, v, mask_mode, mask, heads, scale, 0.0, True, 123, dq, dk, dv)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=tol, atol=tol * 2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("sq", [64, 96])
def test_dropout_mask_regenerated_in_backward(dtype, sq):
    sk, B, heads, p = 64, 2, 4, 0.25
    BH = B * heads
    q, k, _, _ = _make(sq, sk, B, heads, dtype, 0, seed=5)
    eye = torch.eye(64, device="cuda", dtype=dtype).unsqueeze(1).expand(64, BH, 64).contiguous()
    scale = 0.125
    o1 = _fa().forward(q, k, eye, 0, None, heads, scale, p, True, 777)
    o2 = _fa().forward(q, k, eye, 0, None, heads, scale, p, True, 777)
    assert torch.equal(o1, o2)  # counter-based RNG: same seed, same mask
    keep = (o1.float() != 0).permute(1, 0, 2).float()  # [BH, sq, sk]; P > 0 everywhere (no mask)
    frac = keep.mean().item()
    assert abs(frac - (1 - p)) < 0.03, frac
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, eye))
    ref = _reference(qf, kf, vf, scale, 0, None, heads, keep=keep, p=p)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(o1.float(), ref, rtol=tol, atol=tol)
    dout = torch.randn_like(o1)
    ref.backward(dout.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(eye)
    _fa().backward(dout, q, k, eye, 0, None, heads, scale, p, True, 777, dq, dk, dv)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=tol, atol=tol * 2)


def test_eval_mode_ignores_dropout():
    q, k, v, _ = _make(64, 64, 2, 2, torch.float16, 0)
    a = _fa().forward(q, k, v, 0, None, 2, 0.125, 0.5, False, 1)
    b = _fa().forward(q, k, v, 0, None, 2, 0.125, 0.0, True, 2)
    torch.testing.assert_close(a, b)


@pytest.mark.parametrize("impl", ["fast", "default"])
@pytest.mark.parametrize("mask", [None, "pad"])
def test_self_mha_module_fused_matches_unfused(impl, mask, monkeypatch):
    """The module's fused path (MFMA attention) vs its unfused path (baddbmm + softmax kernel + bmm)."""
    from beforeholiday_amd.contrib.multihead_attn import SelfMultiheadAttn

    torch.manual_seed(0)
    m = SelfMultiheadAttn(1024, 16, dropout=0.0, bias=True, impl=impl).cuda().half()
    x = torch.randn(64, 8, 1024, device="cuda", dtype=torch.half)
    kpm = (torch.rand(8, 64, device="cuda") < 0.2) if mask == "pad" else None

    def run(fused):
        config.set(mha_fused=fused)
        xi = x.clone().requires_grad_(True)
        m.zero_grad()
        out, _ = m(xi, xi, xi, key_padding_mask=kpm, need_weights=False, attn_mask=None, is_training=True)
        out.backward(torch.ones_like(out) * 0.01)
        return out.float(), xi.grad.float(), m.in_proj_weight.grad.float()

    o1, g1, w1 = run(True)
    o0, g0, w0 = run(False)
    torch.testing.assert_close(o1, o0, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(g1, g0, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(w1, w0, rtol=5e-2, atol=5e-2)


# ------------------------------------------------------------------------------------------ flash
def _reference_full(q, k, v, scale, mask_mode, mask, heads, fill, keep=None, p=0.0):
    s = torch.einsum("qbd,kbd->bqk", q, k) * scale
    BH, sq, sk = s.shape
    B = BH // heads
    if mask_mode == 1:
        m = mask.view(B, 1, 1, sk).expand(B, heads, sq, sk)
    elif mask_mode == 3:
        m = mask.view(1, 1, sq, sk).expand(B, heads, sq, sk)
    elif mask_mode == 4:
        m = mask.view(B, 1, sq, sk).expand(B, heads, sq, sk)
    elif mask_mode == 5:
        m = torch.ones(sq, sk, device=q.device, dtype=torch.bool).triu(1).view(1, 1, sq, sk).expand(B, heads, sq, sk)
    else:
        m = None
    s = s.view(B, heads, sq, sk)
    if mask_mode == 2:
        s = s + mask.view(B, 1, 1, sk).float()
    elif m is not None:
        s = s.masked_fill(m.bool(), fill)
    pr = torch.softmax(s.view(BH, sq, sk), -1).nan_to_num(0.0)
    if keep is not None:
        pr = pr * keep / (1 - p)
    return torch.einsum("bqk,kbd->qbd", pr, v)


FLASH_SHAPES = [(512, 512), (200, 300), (64, 1000), (129, 129), (1, 77)]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", FLASH_SHAPES)
@pytest.mark.parametrize("mask_mode", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("fill", [float("-inf"), -10000.0])
def test_flash_forward_backward(dtype, shape, mask_mode, fill):
    sq, sk = shape
    if mask_mode in (3, 5) and sq != sk:
        pytest.skip("time / causal masks are square")
    if mask_mode == 2 and fill != float("-inf"):
        pytest.skip("additive masks have no fill value")
    B, heads = 2, 3
    g = torch.Generator(device="cuda").manual_seed(sq * 7 + sk + mask_mode)
    q = torch.randn(sq, B * heads, 3, 64, device="cuda", dtype=dtype, generator=g)[:, :, 0]
    kv = torch.randn(sk, B * heads, 3, 64, device="cuda", dtype=dtype, generator=g)
    k, v = kv[:, :, 1], kv[:, :, 2]
    mask = None
    if mask_mode == 1:
        mask = torch.rand(B, sk, device="cuda", generator=g) < 0.3
    elif mask_mode == 2:
        mask = torch.randn(B, sk, device="cuda", generator=g)
    elif mask_mode == 3:
        mask = torch.rand(sq, sk, device="cuda", generator=g) < 0.2
    elif mask_mode == 4:
        mask = torch.rand(B, sq, sk, device="cuda", generator=g) < 0.25
        mask[0, 0, :] = True  # one fully masked row: zeros (-inf) / uniform (-10000)
    scale = 0.125
    o, lse = _fa().flash_forward(q, k, v, mask_mode, mask, heads, scale, 0.0, True, 5, fill)
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _reference_full(qf, kf, vf, scale, mask_mode, mask, heads, fill)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(o.float(), ref, rtol=tol, atol=tol)
    dout = torch.randn_like(o)
    ref.backward(dout.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    _fa().flash_backward(dout, q, k, v, o, lse, mask_mode, mask, heads, scale, 0.0, True, 5, fill, dq, dk, dv)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=tol, atol=tol * 2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_flash_dropout_regenerated(dtype):
    sq, sk, B, heads, p = 200, 64, 2, 2, 0.2
    BH = B * heads
    g = torch.Generator(device="cuda").manual_seed(11)
    q = torch.randn(sq, BH, 64, device="cuda", dtype=dtype, generator=g)
    k = torch.randn(sk, BH, 64, device="cuda", dtype=dtype, generator=g)
    eye = torch.eye(64, device="cuda", dtype=dtype).unsqueeze(1).expand(64, BH, 64).contiguous()
    o, lse = _fa().flash_forward(q, k, eye, 0, None, heads, 0.125, p, True, 99, float("-inf"))
    o2, _ = _fa().flash_forward(q, k, eye, 0, None, heads, 0.125, p, True, 99, float("-inf"))
    assert torch.equal(o, o2)
    keep = (o.float() != 0).permute(1, 0, 2).float()
    assert abs(keep.mean().item() - (1 - p)) < 0.03
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, eye))
    ref = _reference_full(qf, kf, vf, 0.125, 0, None, heads, float("-inf"), keep=keep, p=p)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(o.float(), ref, rtol=tol, atol=tol)
    dout = torch.randn_like(o)
    ref.backward(dout.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(eye)
    _fa().flash_backward(dout, q, k, eye, o, lse, 0, None, heads, 0.125, p, True, 99, float("-inf"), dq, dk, dv)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=tol, atol=tol * 2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("sq", [200, 64])
def test_flash_dropout_full_mask(dtype, sq):
    """Mask mode 4 (BERT's [B, sq, sk] padding mask, fill -10000) with dropout: the keep mask is
    recovered through V = I as above; masked scores have P = 0 except the fully masked row (uniform),
    whose gradient must still be blocked by the mask."""
    sk, B, heads, p = 64, 2, 2, 0.2
    BH = B * heads
    g = torch.Generator(device="cuda").manual_seed(13)
    q = torch.randn(sq, BH, 64, device="cuda", dtype=dtype, generator=g)
    k = torch.randn(sk, BH, 64, device="cuda", dtype=dtype, generator=g)
    mask = torch.rand(B, sq, sk, device="cuda", generator=g) < 0.25
    mask[1, 3, :] = True
    eye = torch.eye(64, device="cuda", dtype=dtype).unsqueeze(1).expand(64, BH, 64).contiguous()
    o, lse = _fa().flash_forward(q, k, eye, 4, mask, heads, 0.125, p, True, 7, -10000.0)
    keep = (o.float() != 0).permute(1, 0, 2).float()
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, eye))
    ref = _reference_full(qf, kf, vf, 0.125, 4, mask, heads, -10000.0, keep=keep, p=p)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(o.float(), ref, rtol=tol, atol=tol)
    dout = torch.randn_like(o)
    ref.backward(dout.float())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(eye)
    _fa().flash_backward(dout, q, k, eye, o, lse, 4, mask, heads, 0.125, p, True, 7, -10000.0, dq, dk, dv)
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=tol, atol=tol * 2)
