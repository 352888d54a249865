"""MFMA GEMM with fused dense epilogues (kernels/gemm.hip) vs an fp32 PyTorch reference.

Covers tile-boundary shapes (M, N not multiples of the 128x128 tile, K not a multiple of the
64-deep K-step), every epilogue (bias, ReLU / sigmoid / GELU / tanh-GELU with the pre-activation
aux, dActivation with the fixed-order bias-gradient partials) and both 16-bit dtypes. The
forward check uses random (asymmetric) operands so a transposed C/D map cannot pass.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ACTS = {0: lambda x: x, 1: torch.relu, 2: torch.sigmoid, 3: F.gelu, 4: lambda x: F.gelu(x, approximate="tanh")}


def _gm():
    from beforeholiday_amd._native import submodule

    return submodule("gemm")


def _dact(pre_or_out, act):
    a = pre_or_out.float()
    if act == 1:
        return (a > 0).float()
    if act == 2:
        return a * (1 - a)
    if act == 3:
        return 0.5 * (1 + torch.erf(a * 0.7071067811865476)) + a * 0.3989422804014327 * torch.exp(-0.5 * a * a)
    if act == 4:
        k = 0.7978845608028654
        t = torch.tanh(k * (a + 0.044715 * a ** 3))
        return 0.5 * (1 + t) + 0.5 * a * (1 - t * t) * k * (1 + 3 * 0.044715 * a * a)
    return torch.ones_like(a)


SHAPES = [(128, 128, 64), (300, 264, 72), (1, 8, 8), (257, 136, 520), (1536, 3072, 1024), (77, 1000, 16)]
# tile-boundary shapes for the 256x256 kernels (K % 64 == 0: LDS-DMA paths)
BIG_SHAPES = [(256, 256, 64), (520, 776, 192), (1000, 264, 1024), (2048, 2056, 128), (4096, 4096, 512)]
MODES = [0, 1, 2, 3, 4]


@pytest.fixture(autouse=True)
def _pin_mfma():
    gm = _gm()
    gm.set_force_mfma(True)
    yield
    gm.set_force_mfma(False)
    gm.set_tile_mode(0)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", BIG_SHAPES)
@pytest.mark.parametrize("mode", MODES)
def test_tile_kernels(dtype, shape, mode):
    """every tile configuration (auto, 128x128, 256x256, 256x128 three-stage, 256x256 ping-pong)
    on edge shapes, forward with bias + GELU + aux and backward with dGELU + bias-grad partials"""
    M, N, K = shape
    _gm().set_tile_mode(mode)
    torch.manual_seed(M + N + K + mode)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) / K ** 0.5
    b = torch.randn(N, device="cuda", dtype=dtype)
    y, pre = _gm().linear_act(x, w, b, 3, True)
    ref_pre = x.float() @ w.float().t() + b.float()
    tol = 2e-2 if dtype == torch.float16 else 6e-2
    torch.testing.assert_close(pre.float(), ref_pre, rtol=tol, atol=tol)
    torch.testing.assert_close(y.float(), F.gelu(ref_pre), rtol=tol, atol=tol)
    dy = torch.randn(M, K, device="cuda", dtype=dtype)
    wt = torch.randn(N, K, device="cuda", dtype=dtype) / K ** 0.5  # W^T of a [K, N] weight
    aux = torch.randn(M, N, device="cuda", dtype=dtype)
    dx, db = _gm().linear_dact(dy, wt, aux, 3, True)
    ref = (dy.float() @ wt.float().t()) * _dact(aux, 3)
    torch.testing.assert_close(dx.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(db.float(), ref.sum(0), rtol=tol, atol=tol * max(1.0, M ** 0.5))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act", [0, 1, 2, 3, 4])
def test_linear_act(dtype, shape, act):
    M, N, K = shape
    torch.manual_seed(M + N + K + act)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) / K ** 0.5
    b = torch.randn(N, device="cuda", dtype=dtype)
    y, pre = _gm().linear_act(x, w, b, act, True)
    ref_pre = x.float() @ w.float().t() + b.float()
    ref = ACTS[act](ref_pre)
    tol = 2e-2 if dtype == torch.float16 else 6e-2
    torch.testing.assert_close(pre.float(), ref_pre, rtol=tol, atol=tol)
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    y2, _ = _gm().linear_act(x, w, None, act, False)
    torch.testing.assert_close(y2.float(), ACTS[act](x.float() @ w.float().t()), rtol=tol, atol=tol)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_linear_dact_bgrad(dtype, shape, act):
    M, N, K = shape  # dy [M, K] . W [K, N]  -> dx [M, N]; wt = W^T [N, K]
    torch.manual_seed(7 * M + N + K + act)
    dy = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(K, N, device="cuda", dtype=dtype) / K ** 0.5
    aux = torch.randn(M, N, device="cuda", dtype=dtype)
    if act == 2:
        aux = torch.sigmoid(aux)
    dx, db = _gm().linear_dact(dy, w.t().contiguous(), aux, act, True)
    ref = (dy.float() @ w.float()) * _dact(aux, act)
    tol = 2e-2 if dtype == torch.float16 else 6e-2
    torch.testing.assert_close(dx.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(db.float(), ref.sum(0), rtol=tol, atol=tol * max(1.0, M ** 0.5))


def test_strided_inputs_fall_back_or_match():
    x = torch.randn(64, 256, device="cuda", dtype=torch.float16)[:, :128]  # lda = 256
    w = torch.randn(96, 128, device="cuda", dtype=torch.float16)
    y, _ = _gm().linear_act(x, w, None, 0, False)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=2e-2, atol=2e-2)
