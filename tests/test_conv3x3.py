"""Direct 3x3 conv kernel (kernels/conv.hip) vs an fp32 F.conv2d reference: forward and the data
gradient through flipped weights, at ResNet-50 middle-conv shapes and awkward sizes (narrow images
packed side by side, several column tiles, partial row windows)."""
import pytest
import torch
import torch.nn.functional as F

from beforeholiday_amd.ops import conv as bhconv

SHAPES = [  # N, C, K, H, W
    (2, 64, 64, 56, 56), (3, 128, 128, 28, 28), (5, 256, 64, 14, 14), (7, 64, 128, 7, 7),
    (3, 64, 64, 9, 20), (2, 64, 128, 5, 33), (1, 192, 64, 3, 3), (9, 64, 64, 16, 16),
]


def test_dgrad_weight_identity_cpu():
    """conv_transpose form of the data gradient equals conv with the flipped, swapped weights."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 8, 6, 7, generator=g)
    w = torch.randn(5, 8, 3, 3, generator=g)
    dy = torch.randn(2, 5, 6, 7, generator=g)
    ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=1, padding=1)
    got = F.conv2d(dy, bhconv.dgrad_weight(w).contiguous(), padding=1)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_forward_and_dgrad(dtype, shape):
    N, C, K, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(N * 1000 + C + K + H * 7 + W)
    x = torch.randn(N, C, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device="cuda", dtype=dtype, generator=g) * (1.0 / (3 * C ** 0.5))).contiguous(
        memory_format=torch.channels_last)
    assert bhconv.supported(x, w)
    y = bhconv.conv3x3(x, w)
    assert y.is_contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    tol = 2e-2 if dtype == torch.float16 else 6e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    dy = torch.randn(N, K, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    if C % 64 == 0 and K % 64 == 0:
        dx = bhconv.conv3x3_dgrad(dy, w)
        ref_dx = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=1, padding=1)
        torch.testing.assert_close(dx.float(), ref_dx, rtol=tol, atol=tol)


def test_conv3x3_module_cpu_fallback():
    from beforeholiday_amd.models.resnet import Conv3x3
    m = Conv3x3(8, 8, 3, stride=1, padding=1, bias=False, mode="direct")
    x = torch.randn(2, 8, 5, 5)
    torch.testing.assert_close(m(x), F.conv2d(x, m.weight, padding=1))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["direct", "auto"])
def test_conv3x3_module_grads_match_miopen(mode):
    from beforeholiday_amd.models.resnet import Conv3x3
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(64, 128, 3, padding=1, bias=False).cuda().half().to(memory_format=torch.channels_last)
    m = Conv3x3(64, 128, 3, stride=1, padding=1, bias=False, mode=mode).cuda().half().to(
        memory_format=torch.channels_last)
    m.weight.data.copy_(ref.weight.data)
    x = torch.randn(4, 64, 14, 14, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = m(xa), ref(xb)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(ya.float(), yb.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=2e-2, atol=2e-2)
    # the weight gradient is the MFMA wgrad kernel ("direct") or the faster of it and MIOpen ("auto"); MIOpen
    # accumulates split-K partials in an unfixed order: compare to scale
    wr = ref.weight.grad.float()
    torch.testing.assert_close(m.weight.grad.float(), wr, rtol=5e-2, atol=1e-2 * wr.abs().max().item())


WGRAD_SHAPES = [  # N, C, K, H, W, R
    (2, 64, 64, 56, 56, 3), (3, 128, 128, 28, 28, 3), (5, 256, 64, 14, 14, 3), (7, 64, 128, 7, 7, 3),
    (9, 64, 64, 16, 16, 3), (3, 64, 192, 13, 13, 3), (4, 128, 64, 5, 5, 3), (2, 64, 256, 14, 14, 3),
    (2, 64, 256, 56, 56, 1), (4, 256, 128, 14, 14, 1), (1, 64, 64, 7, 16, 1), (2, 128, 64, 28, 28, 1),
    # 1x1 with K % 256, C % 128 and >= 4 such tiles: 256 x 128 tiles on 64-pixel windows (pixel count
    # % 64), else 112
    (4, 256, 512, 28, 28, 1), (1, 256, 512, 16, 16, 1), (64, 512, 2048, 7, 7, 1), (2, 128, 256, 28, 28, 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_conv_wgrad_kernel(dtype, shape):
    """kernels/conv_wgrad.hip vs fp32 torch.nn.grad.conv2d_weight: 56/28/14/7-wide windows, ragged
    widths (13, 5), partial row windows, single-split (direct store) and multi-split (reduce) launches."""
    N, C, K, H, W, R = shape
    g = torch.Generator(device="cuda").manual_seed(N * 100 + C + K + H + R)
    x = torch.randn(N, C, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    assert bhconv.wgrad_supported(x, dy, R)
    gw = bhconv.conv_wgrad(x, dy, R)
    assert gw.shape == (K, C, R, R) and gw.dtype == dtype
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, R, R), dy.float(), stride=1, padding=(R - 1) // 2)
    scale = ref.abs().max().item()
    tol = 1e-2 if dtype == torch.float16 else 2e-2
    torch.testing.assert_close(gw.float(), ref, rtol=tol, atol=tol * scale)
    # bitwise reproducible (fixed-order split reduction)
    assert torch.equal(gw, bhconv.conv_wgrad(x, dy, R))


@pytest.mark.gpu
def test_conv_wgrad_fallback_shapes():
    """Widths without an instantiated window geometry (W = 20 -> 5 groups) and 1x1 pixel counts that
    are not a multiple of 112 report unsupported and take the convolution_backward path."""
    x = torch.randn(2, 64, 9, 20, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(2, 64, 9, 20, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    assert not bhconv.wgrad_supported(x, dy, 3)
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 64, 3, 3), dy.float(), stride=1, padding=1)
    torch.testing.assert_close(bhconv.conv_wgrad(x, dy, 3).float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    x1 = x[:, :, :5, :5].contiguous(memory_format=torch.channels_last)
    dy1 = dy[:, :, :5, :5].contiguous(memory_format=torch.channels_last)
    assert not bhconv.wgrad_supported(x1, dy1, 1)
    ref1 = torch.nn.grad.conv2d_weight(x1.float(), (64, 64, 1, 1), dy1.float())
    torch.testing.assert_close(bhconv.conv_wgrad(x1, dy1, 1).float(), ref1, rtol=2e-2,
                               atol=2e-2 * ref1.abs().max().item())


S2_SHAPES = [  # N, C, K, H_in, W_in: the ResNet-50 downsample layers (output pixel counts a multiple of 112)
    (4, 256, 512, 56, 56), (4, 512, 1024, 28, 28), (16, 1024, 2048, 14, 14), (16, 64, 128, 14, 14),
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", S2_SHAPES)
def test_conv_wgrad_stride2_kernel(dtype, shape):
    """1x1 / stride-2 weight gradient on the MFMA wgrad kernel (x read at the even pixels in place)
    vs fp32 torch.nn.grad.conv2d_weight(stride=2)."""
    N, C, K, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(N * 10 + C + K + H)
    x = torch.randn(N, C, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H // 2, W // 2, device="cuda", dtype=dtype, generator=g).contiguous(
        memory_format=torch.channels_last)
    assert bhconv.wgrad_supported(x, dy, 1, 2)
    assert not bhconv.wgrad_supported(x, dy, 1)  # shape mismatch at stride 1
    gw = bhconv.conv_wgrad_s2(x, dy)
    assert gw.shape == (K, C, 1, 1) and gw.dtype == dtype
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, 1, 1), dy.float(), stride=2)
    tol = 1e-2 if dtype == torch.float16 else 2e-2
    torch.testing.assert_close(gw.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())
    assert torch.equal(gw, bhconv.conv_wgrad_s2(x, dy))


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [False, True])
@pytest.mark.parametrize("mode", ["gemm", "auto"])
def test_conv1x1_stride2_module_matches_conv2d(mode, gather):
    """ResNet downsample 1x1 / stride 2 (models/resnet.py Conv1x1S2) vs nn.Conv2d(stride=2): the
    default path (MIOpen forward / data gradient, in-place stride-2 MFMA wgrad) and the gathered
    path (BH_CONV1X1_S2=gather: quarter-resolution input, GEMM forward, GEMM + scatter data
    gradient, MFMA wgrad kernel)."""
    from beforeholiday_amd.models.resnet import Conv1x1S2
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(256, 512, 1, stride=2, bias=False).cuda().half().to(memory_format=torch.channels_last)
    m = Conv1x1S2(256, 512, 1, stride=2, bias=False, mode=mode, gather=gather).cuda().half().to(
        memory_format=torch.channels_last)
    m.weight.data.copy_(ref.weight.data)
    x = torch.randn(16, 256, 28, 28, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = m(xa), ref(xb)
    assert ya.shape == yb.shape == (16, 512, 14, 14)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(ya.float(), yb.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=2e-2, atol=2e-2)
    assert torch.count_nonzero(xa.grad[:, :, 1::2, :]) == 0  # odd rows / columns get no gradient
    wr = ref.weight.grad.float()
    torch.testing.assert_close(m.weight.grad.float(), wr, rtol=2e-2, atol=1e-2 * wr.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_stem_conv_kernel(dtype):
    """kernels/conv_stem.hip (7x7 / stride 2 / pad 3, 3 -> 64 at 224x224) vs fp32 F.conv2d: image
    borders (zero padding) and every output row block."""
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(3, 3, 224, 224, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda", dtype=dtype, generator=g) * 0.1).contiguous(
        memory_format=torch.channels_last)
    assert bhconv.stem_supported(x, w)
    y = bhconv.stem_conv(x, w)
    assert y.shape == (3, 64, 112, 112) and y.is_contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    tol = 2e-2 if dtype == torch.float16 else 6e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_stem_conv_module_grads():
    from beforeholiday_amd.models.resnet import StemConv
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().half().to(memory_format=torch.channels_last)
    m = StemConv(3, 64, 7, stride=2, padding=3, bias=False, mode="gemm").cuda().half().to(
        memory_format=torch.channels_last)
    m.weight.data.copy_(ref.weight.data)
    x = torch.randn(2, 3, 224, 224, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    ya, yb = m(x), ref(x)
    torch.testing.assert_close(ya.float(), yb.float(), rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    wr = ref.weight.grad.float()
    torch.testing.assert_close(m.weight.grad.float(), wr, rtol=5e-2, atol=1e-2 * wr.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_stem_wgrad_kernel(dtype):
    """kernels/conv_stem.hip weight gradient vs fp32 torch.nn.grad.conv2d_weight (image borders,
    several persistent row walks: 3 images x 112 rows over at most 512 workgroups)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(5, 3, 224, 224, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(5, 64, 112, 112, device="cuda", dtype=dtype, generator=g).contiguous(
        memory_format=torch.channels_last)
    gw = bhconv.stem_wgrad(x, dy)
    assert gw.shape == (64, 3, 7, 7) and gw.dtype == dtype
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 3, 7, 7), dy.float(), stride=2, padding=3)
    tol = 1e-2 if dtype == torch.float16 else 2e-2
    torch.testing.assert_close(gw.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())
    assert torch.equal(gw, bhconv.stem_wgrad(x, dy))  # fixed-order reduction


N64_SHAPES = [(802816, 256), (200704, 64), (4096, 128), (96, 256), (32, 64)]  # M, K


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", N64_SHAPES)
@pytest.mark.parametrize("resid", [False, True])
def test_gemm_n64_kernel(dtype, shape, resid):
    """kernels/gemm_n64.hip (a [M, K] . b [64, K]^T (+ resid)) vs an fp32 torch.mm, including grids
    with fewer strips than waves and the persistent loop at ResNet-50 56x56 sizes."""
    M, K = shape
    g = torch.Generator(device="cuda").manual_seed(M + K)
    a = torch.randn(M, K, device="cuda", dtype=dtype, generator=g)
    b = torch.randn(64, K, device="cuda", dtype=dtype, generator=g) * K ** -0.5
    r = torch.randn(M, 64, device="cuda", dtype=dtype, generator=g) if resid else None
    assert bhconv.gemm_n64_supported(a, b)
    c = bhconv.gemm_n64(a, b, r)
    ref = a.float() @ b.float().t() + (r.float() if resid else 0)
    tol = 1e-2 if dtype == torch.float16 else 3e-2
    torch.testing.assert_close(c.float(), ref, rtol=tol, atol=tol)
    assert not bhconv.gemm_n64_supported(a[:M - 1] if M > 32 else a[:, :K - 8].contiguous(), b)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 64, 64, 56, 56, 3), (4, 128, 128, 28, 28, 3), (3, 256, 256, 14, 14, 3),
                                   (4, 512, 512, 7, 7, 3), (2, 64, 128, 13, 13, 3), (2, 64, 256, 56, 56, 1),
                                   (4, 128, 512, 28, 28, 1), (4, 256, 64, 14, 14, 1), (16, 256, 1024, 14, 14, 1)])
def test_conv_wgrad_bn_prologue(dtype, shape):
    """Weight gradient with the folded BatchNorm + ReLU prologue (x raw, relu(x * scale + shift) applied to
    the LDS tiles) ~ the plain kernel on the materialised activation, and close to fp32
    conv2d_weight; zero padding stays zero (scale / shift with relu(shift) > 0 would otherwise leak)."""
    N, C, K, H, W, R = shape
    g = torch.Generator(device="cuda").manual_seed(N * 7 + C + K + H + R)
    x = torch.randn(N, C, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    scale = torch.rand(C, device="cuda", generator=g) + 0.5
    shift = torch.rand(C, device="cuda", generator=g) + 0.1  # relu(0 * s + b) = b > 0: padding must not see it
    assert bhconv.wgrad_supported(x, dy, R)
    a = bhconv.bn_relu_apply(x, scale, shift).contiguous(memory_format=torch.channels_last)
    gw = bhconv.conv_wgrad(x, dy, R, scale, shift)
    ref = torch.nn.grad.conv2d_weight(a.float(), (K, C, R, R), dy.float(), stride=1, padding=(R - 1) // 2)
    tol = 1e-2 if dtype == torch.float16 else 2e-2
    # the kernel's fused multiply-add may round an input differently from torch's mul + add by one ulp
    torch.testing.assert_close(gw.float(), bhconv.conv_wgrad(a, dy, R).float(), rtol=0,
                               atol=0.1 * tol * ref.abs().max().item())
    torch.testing.assert_close(gw.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_stem_forward_statistics_epilogue(dtype):
    """Stem conv with the BatchNorm statistics partials in its epilogue: the same output as the plain
    stem kernel, and partials summing to the statistics of the stored output about kshift."""
    from beforeholiday_amd._native import submodule

    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(6, 3, 224, 224, device="cuda", dtype=dtype, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) * 0.1).to(dtype)
    k = torch.randn(64, device="cuda", generator=g) * 0.1
    y, part = submodule("conv_cuda").stem_forward_stats(x, w, k)
    assert torch.equal(y, bhconv.stem_conv(x, w))
    assert part.shape[0] == 2 and part.shape[2] == 64
    d = y.float().permute(0, 2, 3, 1).reshape(-1, 64) - k
    ref = torch.stack([d.sum(0), (d * d).sum(0)])
    got = part.sum(1)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_resnet_stem_statistics_path_matches_unfolded():
    """The fused ResNet stem with the statistics epilogue (conv -> BN + ReLU + max pool from the
    partials) vs the statistics pass: same pooled output, stem / BatchNorm gradients and running
    statistics to rounding (stem only: a whole random fp16 network amplifies rounding differences)."""
    from beforeholiday_amd.models import resnet as R

    torch.manual_seed(0)
    m = R.resnet50_fused(layers=(1, 1, 1, 1)).cuda().to(memory_format=torch.channels_last).half()
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.float()
    x = torch.randn(8, 3, 224, 224, device="cuda").half().contiguous(memory_format=torch.channels_last)
    assert m._stem_stats_ok(x)
    state0 = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.randn(8, 64, 56, 56, device="cuda").half().contiguous(memory_format=torch.channels_last)
    outs = []
    for fold in (True, False):
        m.load_state_dict(state0)
        if fold:
            y, part = R._StemStatsFn.apply(x, m.conv1.weight, R._kshift(m.bn1))
            out = m.bn1.forward_from_stats(y, part)
        else:
            out = m.bn1(m.conv1(x))
        out.backward(g)
        outs.append((out.detach(), m.conv1.weight.grad.clone(), m.bn1.weight.grad.clone(), m.bn1.bias.grad.clone(),
                     m.bn1.running_mean.clone(), m.bn1.running_var.clone(), m.bn1.num_batches_tracked.clone()))
        m.zero_grad(set_to_none=True)
    assert int(outs[0][6]) == int(outs[1][6]) == int(state0["bn1.num_batches_tracked"]) + 1
    for a, b in zip(outs[0][:6], outs[1][:6]):
        assert float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)) < 1e-2
