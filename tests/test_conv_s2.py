"""Stride-2 3x3 / pad-1 convolution kernels (the ResNet-50 downsampling blocks' middle conv):
forward and data gradient on the implicit-GEMM MFMA kernel (kernels/conv_igemm.hip), weight gradient
on the strided-halo MFMA wgrad kernel (kernels/conv_wgrad.hip, S = 2), each against a plain fp32
PyTorch convolution of the same operands; the BatchNorm + ReLU prologue and the statistics epilogue
against the same math in fp32; bitwise run-to-run repeatability (no atomics)."""
import pytest
import torch

SHAPES = [  # (N, C, H, K): layer2 / layer3 / layer4 shapes, a ragged batch (pixel tile tail)
    (8, 128, 56, 128), (8, 256, 28, 256), (8, 512, 14, 512), (3, 128, 56, 128), (2, 64, 14, 192),
]


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _tol(dt):
    return 1e-2 if dt == torch.float16 else 3e-2


def _data(n, c, h, k, dt, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, c, h, h, device="cuda", generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(k, c, 3, 3, device="cuda", generator=g) / (3 * c ** 0.5)).to(dt) \
        .contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, k, h // 2, h // 2, device="cuda", generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    return x, w, dy


def _conv_ref(x, w):
    return torch.nn.functional.conv2d(x.float(), w.float(), stride=2, padding=1)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
def test_s2_forward_dgrad_wgrad_match_fp32(shape, dt):
    from beforeholiday_amd.ops import conv as bhconv

    n, c, h, k = shape
    x, w, dy = _data(n, c, h, k, dt)
    assert bhconv.s2_supported(x, w)
    y, part = bhconv.conv3x3_s2(x, w)
    assert y.shape == (n, k, h // 2, h // 2) and y.is_contiguous(memory_format=torch.channels_last)
    assert part.numel() == 0
    assert _rel(y, _conv_ref(x, w)) < _tol(dt)
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    torch.nn.functional.conv2d(xr, wr, stride=2, padding=1).backward(dy.float())
    dx = bhconv.conv3x3_s2_dgrad(dy, w, (h, h))
    assert dx.shape == x.shape
    assert _rel(dx, xr.grad) < _tol(dt)
    dw = bhconv.conv_wgrad(x, dy, 3, stride=2)
    assert bhconv.wgrad_supported(x, dy, 3, 2)
    assert _rel(dw, wr.grad) < _tol(dt)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(8, 128, 56, 128), (4, 256, 28, 256), (4, 512, 14, 512)])
def test_s2_bn_prologue_and_stats_epilogue(shape):
    """conv(relu(x * scale + shift)) with the padding of the NORMALISED activation zero, and the
    output's statistics partials about kshift; the wgrad kernel's prologue on the staged x tiles."""
    from beforeholiday_amd.ops import conv as bhconv

    n, c, h, k = shape
    dt = torch.float16
    x, w, dy = _data(n, c, h, k, dt, seed=1)
    scale = torch.rand(c, device="cuda") + 0.5
    shift = torch.randn(c, device="cuda") * 0.5
    kshift = torch.randn(k, device="cuda") * 0.1
    y, part = bhconv.conv3x3_s2(x, w, scale, shift, stats=True, kshift=kshift)
    a = bhconv.bn_relu_apply(x, scale, shift)  # rounded to fp16 as the kernel's prologue rounds
    assert _rel(y, _conv_ref(a, w)) < 1e-2
    yf = y.float().transpose(0, 1).reshape(k, -1) - kshift.view(-1, 1)
    assert part.dim() == 3 and part.size(0) == 2 and part.size(2) == k
    assert _rel(part[0].sum(0), yf.sum(1)) < 1e-4
    assert _rel(part[1].sum(0), yf.square().sum(1)) < 1e-4
    wr = w.float().requires_grad_()
    torch.nn.functional.conv2d(a.float(), wr, stride=2, padding=1).backward(dy.float())
    dw = bhconv.conv_wgrad(x, dy, 3, scale, shift, stride=2)
    assert _rel(dw, wr.grad) < 1e-2


@pytest.mark.gpu
def test_s2_large_grid_and_repeatable():
    """The layer-2 downsampling conv at batch 256 (200k output pixels, 1568 pixel tiles; the dgrad's four
    phases 6272 workgroups): matches fp32 and is bitwise repeatable in all three directions."""
    from beforeholiday_amd.ops import conv as bhconv

    x, w, dy = _data(256, 128, 56, 128, torch.float16, seed=2)
    y0, _ = bhconv.conv3x3_s2(x, w)
    dx0 = bhconv.conv3x3_s2_dgrad(dy, w, (56, 56))
    dw0 = bhconv.conv_wgrad(x, dy, 3, stride=2)
    for _ in range(2):
        assert torch.equal(bhconv.conv3x3_s2(x, w)[0], y0)
        assert torch.equal(bhconv.conv3x3_s2_dgrad(dy, w, (56, 56)), dx0)
        assert torch.equal(bhconv.conv_wgrad(x, dy, 3, stride=2), dw0)
    sl = slice(0, 16)  # fp32 reference on a slice of the batch (the kernel computed the whole)
    assert _rel(y0[sl], _conv_ref(x[sl], w)) < 1e-2
    xr = x[sl].float().requires_grad_()
    torch.nn.functional.conv2d(xr, w.float(), stride=2, padding=1).backward(dy[sl].float())
    assert _rel(dx0[sl], xr.grad) < 1e-2
    wr = w.float().requires_grad_()
    torch.nn.functional.conv2d(x.float(), wr, stride=2, padding=1).backward(dy.float())
    assert _rel(dw0, wr.grad) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("pro", [False, True])
def test_s2_lds_staged_kernel_matches_register_staged(pro):
    """Config.igemm_lds: the LDS-DMA-staged implicit GEMM (k_igemm_lds) and the register-staged one
    (k_igemm) compute the same sums in the same order per output (fp32 accumulation over the same k-steps),
    so forward (with / without the BatchNorm prologue, with statistics) and data gradient agree bitwise."""
    from beforeholiday_amd import config
    from beforeholiday_amd.ops import conv as bhconv

    n, c, h, k = 4, 256, 28, 256
    x, w, dy = _data(n, c, h, k, torch.float16, seed=3)
    g = torch.Generator(device="cuda").manual_seed(4)
    sc = (torch.rand(c, device="cuda", generator=g) + 0.5) if pro else None
    sh = (torch.randn(c, device="cuda", generator=g) * 0.2) if pro else None
    outs = {}
    for lds in (False, True):
        with config.override(igemm_lds=lds):
            y, part = bhconv.conv3x3_s2(x, w, pro_scale=sc, pro_shift=sh, stats=True)
            dx = bhconv.conv3x3_s2_dgrad(dy, w, (h, h))
        torch.cuda.synchronize()
        outs[lds] = (y, part, dx)
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
    ref = _conv_ref(torch.relu(x.float() * sc[None, :, None, None] + sh[None, :, None, None]) if pro else x, w)
    assert _rel(outs[True][0], ref) < 1e-2
