"""contrib conv_bias_relu vs torch conv2d + bias + ReLU (reference test: apex/contrib/test/conv_bias_relu)."""
import pytest
import torch
import torch.nn.functional as F

from tests.conftest import devices


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("variant", ["relu", "mask", "bias", "frozen"])
def test_conv_bias_relu(device, variant):
    from beforeholiday_amd.contrib import conv_bias_relu as cbr
    torch.manual_seed(0)
    dtype = torch.float16 if device != "cpu" else torch.float32
    x = torch.randn(2, 16, 10, 10, device=device).to(dtype).to(memory_format=torch.channels_last).requires_grad_()
    w = (torch.randn(32, 16, 3, 3, device=device) * 0.1).to(dtype).to(memory_format=torch.channels_last)
    w.requires_grad_()
    b = torch.randn(1, 32, 1, 1, device=device).to(dtype).requires_grad_()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    with torch.autocast("cuda", enabled=device != "cpu", dtype=torch.half):
        if variant == "relu":
            y = cbr.ConvBiasReLU(x, w, b, 1, 1)
        elif variant == "mask":
            mask = (torch.rand(2, 32, 10, 10, device=device) > 0.3).to(dtype)
            y = cbr.ConvBiasMaskReLU(x, w, b, mask, 1, 1)
        elif variant == "bias":
            y = cbr.ConvBias(x, w, b, 1, 1)
        else:
            scale = torch.rand(32, device=device) + 0.5
            y = cbr.ConvFrozenScaleBiasReLU(x, w, scale, b, 1, 1)
    c = F.conv2d(xr, wr, None, 1, 1)
    # the ReLU mask of the reference is taken from the kernel's own output: pre-activations within
    # fp16 rounding of 0 may legitimately flip sign between the fp16 kernel and the fp32 reference
    keep = (y.detach().float() > 0).float()
    if variant == "frozen":
        sc = scale.half().float() if dtype == torch.float16 else scale
        pre = c * sc.view(1, -1, 1, 1) + br
        torch.testing.assert_close(y.float(), torch.relu(pre.detach()), rtol=3e-2, atol=3e-2)
        ref = pre * keep
    else:
        ref = c + br
        if variant in ("relu", "mask"):
            torch.testing.assert_close(y.float(), (torch.relu(ref) * (mask.float() if variant == "mask" else 1)).detach(),
                                       rtol=3e-2, atol=3e-2)
            ref = ref * keep
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    g = torch.randn_like(ref)
    y.float().backward(g)
    ref.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol * 5)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=tol, atol=tol * 20)
    if variant != "frozen":
        torch.testing.assert_close(b.grad.float(), br.grad, rtol=tol, atol=tol * 20)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["relu", "mask", "bias", "frozen", "frozen_add"])
@pytest.mark.parametrize("shape", [(64, 128, 3, 1, 1, 28), (64, 256, 1, 0, 1, 56), (256, 512, 1, 0, 2, 32),
                                   (128, 128, 3, 1, 1, 14)])
def test_conv_bias_relu_fused_kernels(variant, shape):
    """Shapes the MFMA kernels cover (1x1 s1 / s2, 3x3 s1): ONE kernel per forward (affine epilogue),
    the backward on the MFMA dgrad / wgrad kernels -- against fp32 conv2d + bias / scale (+ z) + ReLU."""
    from beforeholiday_amd.contrib.conv_bias_relu import conv_bias_relu as cbr
    C, K, R, P, S, HW = shape
    torch.manual_seed(0)
    x = torch.randn(4, C, HW, HW, device="cuda").half().contiguous(memory_format=torch.channels_last).requires_grad_()
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).half().contiguous(
        memory_format=torch.channels_last).requires_grad_()
    b = (torch.randn(1, K, 1, 1, device="cuda") * 0.1).half().requires_grad_()
    assert cbr._kind(x.detach(), w.detach(), P, S) is not None  # the fused path, not MIOpen
    ho = HW // S
    scale = torch.rand(K, device="cuda") + 0.5
    mask = (torch.rand(4, K, ho, ho, device="cuda") > 0.3).half().contiguous(memory_format=torch.channels_last)
    z = torch.randn(4, K, ho, ho, device="cuda").half().contiguous(memory_format=torch.channels_last).requires_grad_()
    if variant == "relu":
        y = cbr.ConvBiasReLU(x, w, b, P, S)
    elif variant == "mask":
        y = cbr.ConvBiasMaskReLU(x, w, b, mask, P, S)
    elif variant == "bias":
        y = cbr.ConvBias(x, w, b, P, S)
    elif variant == "frozen":
        y = cbr.ConvFrozenScaleBiasReLU(x, w, scale, b, P, S)
    else:
        y = cbr.ConvFrozenScaleBiasAddReLU(x, w, scale, b, z, P, S)
    xr, wr, br, zr = (t.detach().float().requires_grad_() for t in (x, w, b, z))
    c = F.conv2d(xr, wr, None, S, P)
    if variant in ("frozen", "frozen_add"):
        pre = c * scale.view(1, -1, 1, 1) + br
        if variant == "frozen_add":
            pre = pre + zr
    else:
        pre = c + br
    keep = (y.detach().float() > 0).float()
    ref = pre if variant == "bias" else pre * keep  # ReLU mask (and the 0/1 mask) from the kernel's output
    torch.testing.assert_close(y.float(), (torch.relu(pre) * (mask.float() if variant == "mask" else 1)
                                           if variant != "bias" else pre).detach(), rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ref)
    y.float().backward(g)
    ref.backward(g)
    rel = lambda a, b_: float((a.float() - b_).norm() / b_.norm())  # noqa: E731
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    if variant in ("relu", "mask", "bias"):
        assert rel(b.grad, br.grad) < 2e-2
    if variant == "frozen_add":
        assert rel(z.grad, zr.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_contrib_bottleneck_fused_matches_fp32(stride):
    from beforeholiday_amd.contrib.bottleneck import Bottleneck
    torch.manual_seed(0)
    blk = Bottleneck(256, 64, 256 if stride == 1 else 512, stride=stride).cuda()
    for bn in (blk.bn1, blk.bn2, blk.bn3):
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    ref_state = {k: v.clone() for k, v in blk.state_dict().items()}
    x = torch.randn(4, 256, 28, 28, device="cuda")
    blk16 = blk.half().to(memory_format=torch.channels_last)
    for m in blk16.modules():
        if hasattr(m, "running_var"):
            m.float()
    xh = x.half().contiguous(memory_format=torch.channels_last).requires_grad_()
    y = blk16(xh)
    y.float().square().sum().backward()
    blk32 = Bottleneck(256, 64, 256 if stride == 1 else 512, stride=stride).cuda()
    blk32.load_state_dict(ref_state)
    xr = x.clone().requires_grad_()
    # fp32 reference through plain torch ops
    def frozen(bn, t):
        s, b = bn.get_scale_bias()
        return t * s + b
    out = torch.relu(frozen(blk32.bn1, F.conv2d(xr, blk32.conv1.weight, stride=stride)))
    out = torch.relu(frozen(blk32.bn2, F.conv2d(out, blk32.conv2.weight, padding=1)))
    idn = frozen(blk32.downsample[1], F.conv2d(xr, blk32.downsample[0].weight, stride=stride)) \
        if blk32.downsample is not None else xr
    yr = torch.relu(frozen(blk32.bn3, F.conv2d(out, blk32.conv3.weight)) + idn)
    yr.square().sum().backward()
    rel = lambda a, b_: float((a.detach().float() - b_.detach()).norm() / b_.detach().norm())  # noqa: E731
    assert rel(y, yr) < 2e-2
    assert rel(xh.grad, xr.grad) < 4e-2
    for (n, p), q in zip(blk16.named_parameters(), blk32.parameters()):
        assert rel(p.grad, q.grad) < 4e-2, n
