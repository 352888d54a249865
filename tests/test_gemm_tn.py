"""The transposed-operand ping-pong GEMM (kernels/gemm_tn.hip, ``_C.gemm.weight_grad_tn``): dW = dY^T X of a dense
layer against the fp32 PyTorch product, whole and split-K, fp16 / bf16, with row strides wider than the rows."""
import pytest
import torch


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _gm():
    from beforeholiday_amd._native import submodule

    return submodule("gemm")


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("T,N,K,splits", [(1024, 256, 256, 0), (2048, 512, 768, 1), (2048, 512, 768, 3),
                                           (8192, 1024, 4096, 0), (8192, 3072, 1024, 0), (4096, 1024, 1024, 2)])
def test_weight_grad_tn_matches_fp32(T, N, K, splits, dt):
    torch.manual_seed(0)
    dy = torch.randn(T, N, device="cuda").to(dt)
    x = torch.randn(T, K, device="cuda").to(dt)
    assert _gm().weight_grad_tn_supported(dy, x)
    out = _gm().weight_grad_tn(dy, x, splits)
    ref = dy.float().t() @ x.float()
    assert out.shape == (N, K) and out.dtype == dt
    assert _rel(out, ref) < (2e-3 if dt == torch.float16 else 1e-2)


@pytest.mark.gpu
def test_weight_grad_tn_strided_rows_and_determinism():
    torch.manual_seed(1)
    big_dy = torch.randn(2048, 1024 + 256, device="cuda").half()
    big_x = torch.randn(2048, 512 + 64, device="cuda").half()
    dy, x = big_dy[:, 256:], big_x[:, :512]  # row strides wider than the rows
    out = _gm().weight_grad_tn(dy, x, 4)
    assert _rel(out, dy.float().t() @ x.float()) < 2e-3
    assert torch.equal(out, _gm().weight_grad_tn(dy, x, 4))  # fixed-order split reduction


@pytest.mark.gpu
def test_weight_grad_tn_rejects_unsupported():
    dy = torch.randn(1000, 256, device="cuda").half()  # T % 64 != 0
    x = torch.randn(1000, 256, device="cuda").half()
    assert not _gm().weight_grad_tn_supported(dy, x)
    with pytest.raises(RuntimeError):
        _gm().weight_grad_tn(dy, x, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("mg_dtype", [torch.float32, torch.float16])
def test_wgrad_gemm_accum_on_tn_kernel(mg_dtype):
    """fused_weight_gradient_mlp_cuda's main_grad += d_output^T input through the transposed-operand GEMM
    (fp32 or 16-bit main_grad, 3-D [seq, batch, hidden] operands as Megatron passes them)."""
    from beforeholiday_amd._native import submodule

    torch.manual_seed(2)
    x = torch.randn(1024, 8, 1024, device="cuda").half()
    dy = torch.randn(1024, 8, 512, device="cuda").half()
    mg = torch.randn(512, 1024, device="cuda").to(mg_dtype)
    ref = mg.float() + dy.reshape(-1, 512).float().t() @ x.reshape(-1, 1024).float()
    wg = submodule("fused_weight_gradient_mlp_cuda")
    (wg.wgrad_gemm_accum_fp32 if mg_dtype == torch.float32 else wg.wgrad_gemm_accum_fp16)(x, dy, mg)
    assert _rel(mg, ref) < (1e-5 if mg_dtype == torch.float32 else 2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,K,N,splits", [(1024, 256, 256, 0), (8192, 3072, 1024, 0), (8192, 1024, 1024, 0),
                                           (8192, 1024, 4096, 0), (2048, 768, 512, 3), (4096, 4096, 1024, 1)])
def test_mm_nn_matches_fp32(M, K, N, splits, dt):
    """The NN layout (C = A @ Bt, both row-major: a data gradient dY @ W) of the same kernel."""
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda").to(dt)
    bt = (torch.randn(K, N, device="cuda") / K ** 0.5).to(dt)
    assert _gm().mm_nn_supported(a, bt)
    out = _gm().mm_nn(a, bt, splits)
    ref = a.float() @ bt.float()
    assert out.shape == (M, N) and _rel(out, ref) < (2e-3 if dt == torch.float16 else 1e-2)
