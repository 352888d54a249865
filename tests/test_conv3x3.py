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
    # both weight gradients are MIOpen's (fp16 split-K accumulation, order not fixed): compare to scale
    wr = ref.weight.grad.float()
    torch.testing.assert_close(m.weight.grad.float(), wr, rtol=5e-2, atol=1e-2 * wr.abs().max().item())
