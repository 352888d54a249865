"""Fused scale-mask softmax and softmax cross-entropy vs PyTorch fp32 references (reference:
tests/L0/run_transformer/test_fused_softmax.py, apex/contrib/test/xentropy)."""
import pytest
import torch

from beforeholiday_amd.contrib.xentropy import SoftmaxCrossEntropyLoss
from beforeholiday_amd.transformer.enums import AttnMaskType
from beforeholiday_amd.transformer.functional import FusedScaleMaskSoftmax, GenericFusedScaleMaskSoftmax

from conftest import devices


def attention_mask_func(scores, mask):
    return scores.masked_fill(mask, -10000.0)


def _ref(x, mask, scale, causal):
    xf = x.float() * scale
    if causal:
        sq, sk = x.shape[-2:]
        m = torch.triu(torch.ones(sq, sk, dtype=torch.bool, device=x.device), 1)
        xf = xf.masked_fill(m, float("-inf"))
    elif mask is not None:
        xf = xf.masked_fill(mask, -10000.0)
    return torch.softmax(xf, -1)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("sk", [32, 128, 1000, 2048, 4096, 6000, 16384])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_scale_mask_softmax(device, sk, causal, dtype):
    if device == "cpu" and sk > 2048:
        pytest.skip("cpu reference path checked on small sizes")
    torch.manual_seed(0)
    b, np_, sq = 2, 3, (sk if causal else 8)
    if causal and sk > 4096:
        b, np_ = 1, 1
    x = (torch.randn(b, np_, sq, sk, device=device) * 4).to(dtype)
    mask = None if causal else (torch.rand(b, 1, sq, sk, device=device) > 0.7)
    if mask is not None:
        mask[0, 0, 0, :] = True  # fully masked row -> zeros
    sm = FusedScaleMaskSoftmax(dtype == torch.float16, dtype == torch.bfloat16,
                               AttnMaskType.causal if causal else AttnMaskType.padding, True, attention_mask_func,
                               True, 0.5)
    assert sm.is_kernel_available(mask, b, np_, sq, sk)
    xg = x.detach().requires_grad_(True)
    y = sm(xg, mask)
    xr = x.detach().float().requires_grad_(True)
    yr = _ref(xr, mask, 0.5, causal)
    if mask is not None:
        yr = torch.where(mask.all(-1, keepdim=True), torch.zeros_like(yr), yr)
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    tol = 2e-3 if dtype == torch.float16 else 1e-2
    torch.testing.assert_close(y.float(), yr.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(xg.grad.float(), xr.grad, rtol=tol * 4, atol=tol * 4)


@pytest.mark.parametrize("device", devices())
def test_generic_softmax_and_fallback(device):
    x = torch.randn(2, 2, 4, 40, device=device).half()
    mask = torch.rand(2, 1, 4, 40, device=device) > 0.5
    sm = GenericFusedScaleMaskSoftmax(True, False, True, attention_mask_func, True, 1.0)
    y = sm(x.requires_grad_(True), mask)
    y.float().sum().backward()
    ref = torch.softmax(x.float().masked_fill(mask, -10000.0), -1)
    torch.testing.assert_close(y.float(), ref, rtol=2e-3, atol=2e-3)
    fb = FusedScaleMaskSoftmax(False, False, AttnMaskType.padding, True, attention_mask_func, True, 2.0)
    assert not fb.is_kernel_available(mask, 2, 2, 4, 40)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
@pytest.mark.parametrize("dtype,half_to_float", [(torch.float32, False), (torch.float16, True), (torch.bfloat16, False)])
@pytest.mark.parametrize("V", [1000, 32003])
def test_xentropy(device, smoothing, dtype, half_to_float, V):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("cpu path in fp32")
    torch.manual_seed(0)
    N = 64
    logits = (torch.randn(N, V, device=device) * 3).to(dtype).requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=device)
    labels[:4] = 0  # padding_idx rows
    loss = SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing, 0, half_to_float)
    lr = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, labels, reduction="none", label_smoothing=smoothing)
    ref = ref.masked_fill(labels == 0, 0)
    g = torch.rand(N, device=device)
    loss.float().backward(g.to(loss.dtype).float() if loss.dtype == torch.float32 else g.to(loss.dtype).float())
    ref.backward(g)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(loss.float(), ref.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(logits.grad.float(), lr.grad, rtol=tol, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("V,shards", [(1000, 2), (50304, 4), (37, 1)])
def test_vocab_parallel_xent_kernels(dtype, V, shards):
    """Shard partials (one pass each) + combine == full-vocab cross-entropy; backward per shard."""
    from beforeholiday_amd._native import submodule
    xent = submodule("xentropy_cuda")
    torch.manual_seed(0)
    rows = 67
    logits = (torch.randn(rows, V, device="cuda") * 3).to(dtype)
    target = torch.randint(0, V, (rows,), device="cuda")
    ref = torch.nn.functional.cross_entropy(logits.float(), target, reduction="none")
    part = V // shards
    stats = torch.stack([xent.vocab_parallel_stats(logits[:, s * part:(s + 1) * part].contiguous(), target, s * part)
                         for s in range(shards)])
    loss, lse = xent.vocab_parallel_combine(stats, dtype)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(loss.float(), ref, rtol=tol, atol=tol)
    g = torch.rand(rows, device="cuda")
    lr = logits.float().requires_grad_()
    (torch.nn.functional.cross_entropy(lr, target, reduction="none") * g).sum().backward()
    for s in range(shards):
        shard = logits[:, s * part:(s + 1) * part].contiguous()
        dx = xent.backward(g, shard, lse, target - s * part, 0.0)
        torch.testing.assert_close(dx.float(), lr.grad[:, s * part:(s + 1) * part], rtol=tol, atol=tol)
