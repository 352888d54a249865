"""FusedDense / FusedDenseGeluDense / MLP / wgrad accumulation vs. plain PyTorch fp32 references
(reference tests: tests/L0/run_mlp/test_mlp.py, apex/contrib fused_dense tests)."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from tests.conftest import devices

TOL = {torch.float32: dict(rtol=1e-4, atol=1e-4), torch.float16: dict(rtol=2e-2, atol=2e-2),
       torch.bfloat16: dict(rtol=5e-2, atol=5e-2)}


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_fused_dense(device, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("CPU reference path runs fp32")
    from beforeholiday_amd.fused_dense import FusedDense
    torch.manual_seed(0)
    m = FusedDense(64, 40).to(device, dtype)
    ref = nn.Linear(64, 40).to(device)
    with torch.no_grad():
        ref.weight.copy_(m.weight.float())
        ref.bias.copy_(m.bias.float())
    x = torch.randn(3, 10, 64, device=device, dtype=dtype, requires_grad=True)
    xr = x.detach().float().requires_grad_()
    y = m(x)
    yr = ref(xr)
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, **TOL[dtype])
    scale = dict(rtol=TOL[dtype]["rtol"], atol=TOL[dtype]["atol"] * 10)
    torch.testing.assert_close(m.weight.grad.float(), ref.weight.grad, **scale)
    torch.testing.assert_close(m.bias.grad.float(), ref.bias.grad, **scale)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_dense_gelu_dense(device, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("CPU reference path runs fp32")
    from beforeholiday_amd.fused_dense import FusedDenseGeluDense
    torch.manual_seed(1)
    m = FusedDenseGeluDense(32, 96, 48).to(device, dtype)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.2)
    params = [p.detach().float().clone().requires_grad_() for p in (m.weight, m.bias, m.weight2, m.bias2)]
    x = torch.randn(20, 32, device=device, dtype=dtype, requires_grad=True)
    xr = x.detach().float().requires_grad_()
    y = m(x)
    yr = F.linear(F.gelu(F.linear(xr, params[0], params[1])), params[2], params[3])
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, **TOL[dtype])
    for p, r in zip((m.weight, m.bias, m.weight2, m.bias2), params):
        torch.testing.assert_close(p.grad.float(), r.grad, rtol=TOL[dtype]["rtol"], atol=TOL[dtype]["atol"] * 10)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("activation", ["relu", "sigmoid", "none"])
@pytest.mark.parametrize("bias", [True, False])
def test_mlp(device, activation, bias):
    from beforeholiday_amd.mlp import MLP
    sizes = [48, 64, 32, 8]
    torch.manual_seed(2)
    mlp = MLP(sizes, bias=bias, activation=activation).to(device)
    layers = []
    for i in range(mlp.num_layers):
        lin = nn.Linear(sizes[i], sizes[i + 1], bias=bias)
        with torch.no_grad():
            lin.weight.copy_(mlp.weights[i])
            if bias:
                lin.bias.copy_(mlp.biases[i])
        layers.append(lin)
        if activation == "relu":
            layers.append(nn.ReLU())
        elif activation == "sigmoid":
            layers.append(nn.Sigmoid())
    ref = nn.Sequential(*layers).to(device)
    x = torch.empty(33, sizes[0], device=device).uniform_(-1, 1).requires_grad_()
    xr = x.detach().clone().requires_grad_()
    y, yr = mlp(x), ref(xr)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    y.mean().mul(10).backward()
    yr.mean().mul(10).backward()
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-6)
    for i in range(mlp.num_layers):
        lin = ref[i * (1 if activation == "none" else 2)]
        torch.testing.assert_close(mlp.weights[i].grad, lin.weight.grad, rtol=1e-4, atol=1e-6)
        if bias:
            torch.testing.assert_close(mlp.biases[i].grad, lin.bias.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("act", [1, 2, 3, 4])
def test_act_backward_bgrad(device, act):
    """The fused dActivation + bias-gradient pass vs autograd (odd widths exercise the scalar path)."""
    from beforeholiday_amd.ops import fused_dense as fd
    torch.manual_seed(3)
    for M, N in [(257, 40), (64, 1000), (3, 13)]:
        pre = torch.randn(M, N, device=device)
        fn = {1: torch.relu, 2: torch.sigmoid, 3: F.gelu, 4: lambda t: F.gelu(t, approximate="tanh")}[act]
        p = pre.clone().requires_grad_()
        out = fn(p)
        dy = torch.randn(M, N, device=device)
        out.backward(dy)
        aux = pre if act in (3, 4) else out.detach()
        dx, db = fd.act_backward(dy, aux, act, True)
        torch.testing.assert_close(dx, p.grad, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(db, p.grad.sum(0), rtol=1e-4, atol=1e-4)
        y = fd.bias_act_forward(pre, torch.ones(N, device=device), act)
        torch.testing.assert_close(y, fn(pre + 1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_wgrad_gemm_accum(device, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("CPU reference path runs fp32")
    from beforeholiday_amd.ops import fused_dense as fd
    torch.manual_seed(4)
    x = torch.randn(4, 16, 24, device=device, dtype=dtype)
    dy = torch.randn(4, 16, 40, device=device, dtype=dtype)
    main = torch.randn(40, 24, device=device)
    expect = main + dy.reshape(-1, 40).float().t() @ x.reshape(-1, 24).float()
    fd.wgrad_gemm_accum_fp32(x, dy, main)
    torch.testing.assert_close(main, expect, rtol=1e-3, atol=1e-2)
    if dtype != torch.float32:
        m16 = torch.zeros(40, 24, device=device, dtype=dtype)
        fd.wgrad_gemm_accum_fp16(x, dy, m16)
        prod = dy.reshape(-1, 40).float().t() @ x.reshape(-1, 24).float()
        torch.testing.assert_close(m16.float(), prod, rtol=5e-2, atol=5e-1)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8192, 1024), (3, 77, 40), (1000, 4096), (5, 8)])
def test_bias_grad_colsum(device, dtype, shape):
    """bias_grad == fp32 column sum over all leading dims (covers the split partial + finalize kernels)."""
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("cpu reference path is exercised in fp32")
    from beforeholiday_amd.ops.fused_dense import bias_grad

    torch.manual_seed(0)
    dy = torch.randn(shape, device=device).to(dtype)
    ref = dy.float().reshape(-1, shape[-1]).sum(0)
    out = bias_grad(dy)
    assert out.dtype == dtype and out.shape == (shape[-1],)
    tol = 1e-3 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * max(1.0, shape[0] ** 0.5))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("p,use_bias", [(0.1, True), (0.0, True), (0.3, False)])
def test_bias_dropout_add_native(dtype, p, use_bias):
    """Fused bias-dropout-add (kernels/dense.hip) vs an fp32 PyTorch reference driven by the kernel's
    own keep bits; backward: dropout-masked dx, bias grad = column sum, residual grad = dout."""
    from beforeholiday_amd.ops import fused_dense as fd

    torch.manual_seed(0)
    s, b, h = 96, 4, 1024
    x = torch.randn(s, b, h, device="cuda", dtype=dtype, requires_grad=True)
    bias = torch.randn(h, device="cuda", dtype=dtype, requires_grad=True) if use_bias else None
    res = torch.randn(s, b, h, device="cuda", dtype=dtype, requires_grad=True)
    out = fd._BiasDropoutAddFn.apply(x, bias, res, p, False)
    keep_bits = fd._fd().bias_dropout_add(x.detach(), bias.detach() if use_bias else None, res.detach(), p, 123)[1]
    assert out.grad_fn is not None
    if p > 0:
        assert keep_bits.numel() * 8 == x.numel()
        bits = torch.stack([(keep_bits >> k) & 1 for k in range(8)], -1).reshape(x.shape).float()
        frac = bits.mean().item()
        assert abs(frac - (1 - p)) < 0.01, frac
    # reference with the mask from the fused call's own saved bits
    ctx_keep = out.grad_fn.saved_tensors[0]
    if p > 0:
        m = torch.stack([(ctx_keep >> k) & 1 for k in range(8)], -1).reshape(x.shape).float() / (1 - p)
    else:
        m = torch.ones(x.shape, device="cuda")
    xb = x.detach().float() + (bias.detach().float() if use_bias else 0)
    ref = res.detach().float() + xb * m
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    dout = torch.randn_like(out)
    out.backward(dout)
    dx_ref = dout.float() * m
    torch.testing.assert_close(x.grad.float(), dx_ref, atol=tol, rtol=tol)
    torch.testing.assert_close(res.grad.float(), dout.float(), atol=0, rtol=0)
    if use_bias:
        torch.testing.assert_close(bias.grad.float(), dx_ref.reshape(-1, h).sum(0), atol=tol * 20, rtol=tol)


@pytest.mark.parametrize("device", devices())
def test_bias_dropout_add_eval_matches_reference(device):
    """Eval mode (no dropout): both the HIP path and the CPU path equal residual + x + bias exactly."""
    from beforeholiday_amd.models.transformer_lm import bias_dropout_add

    torch.manual_seed(0)
    x, res = torch.randn(16, 2, 64, device=device), torch.randn(16, 2, 64, device=device)
    bias = torch.randn(64, device=device)
    out = bias_dropout_add(x, bias, res, 0.1, training=False)
    torch.testing.assert_close(out, res + (x + bias), atol=1e-6, rtol=1e-6)


@pytest.mark.gpu
def test_bias_dropout_add_seeds_give_unrelated_masks():
    """Keyed hash: the mask of seed s2 is not the mask of seed s1 re-indexed by i ^ (s1 ^ s2) (the
    failure mode of XOR-ing a raw seed into the index), and two seeds agree on ~p^2 + (1-p)^2."""
    from beforeholiday_amd.ops import fused_dense as fd

    x = torch.zeros(256, 1024, device="cuda", dtype=torch.bfloat16)
    res = torch.zeros_like(x)

    def bits(seed):
        kb = fd._fd().bias_dropout_add(x, None, res, 0.5, seed)[1]
        return torch.stack([(kb >> k) & 1 for k in range(8)], -1).reshape(-1)

    b1, b2 = bits(5), bits(5 ^ 64)
    idx = torch.arange(b1.numel(), device="cuda")
    assert not torch.equal(b2, b1[idx ^ 64])
    agree = (b1 == b2).float().mean().item()
    assert abs(agree - 0.5) < 0.01, agree
    assert abs(b1.float().mean().item() - 0.5) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("MKC", [(8192, 1024, 1024), (4096, 768, 3072), (8192, 512, 512), (8192, 3072, 1024),
                                 (1000, 256, 256)])
def test_weight_grad_matches_fp32(MKC, dt):
    """ops.fused_dense.weight_grad: dY^T . X on the MFMA weight-gradient kernel where the static shape
    rule takes it (<= ~2.2M weight elements, >= 4096 tokens), the library GEMM otherwise."""
    from beforeholiday_amd.ops import fused_dense as fd

    M, K, C = MKC
    torch.manual_seed(0)
    dy = torch.randn(M, K, device="cuda").to(dt)
    x = torch.randn(M, C, device="cuda").to(dt)
    got = fd.weight_grad(dy, x)
    ref = dy.float().t() @ x.float()
    assert got.shape == (K, C) and got.dtype == dt
    torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2 * M ** 0.5 / 8)
    assert torch.equal(fd.weight_grad(dy, x), got)  # fixed reduction order


@pytest.mark.gpu
@pytest.mark.parametrize("MKC", [(4096, 2048, 1024), (8192, 3072, 1024), (2048, 1024, 4096)])
def test_wgrad_kernel_wide_256x256_tiles(MKC):
    """The 1x1 weight-gradient kernel's 256 x 256 tiles (K, C % 256 and >= 32 tiles: the large
    transformer weights) on the [tokens, channels] views, against the fp32 product."""
    from beforeholiday_amd.ops import conv as bhconv

    M, K, C = MKC
    torch.manual_seed(1)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    x4, dy4 = x.view(1, 1, M, C).permute(0, 3, 1, 2), dy.view(1, 1, M, K).permute(0, 3, 1, 2)
    assert bhconv.wgrad_supported(x4, dy4, 1)
    got = bhconv.conv_wgrad(x4, dy4, 1).view(K, C).float()
    ref = dy.float().t() @ x.float()
    assert float((got - ref).norm() / ref.norm()) < 4e-3


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("V,H,n,pad", [(30592, 1024, 8192, None), (2, 1024, 8192, None), (512, 1000, 4100, 3),
                                       (64, 7, 333, None)])
def test_embedding_backward_matches_fp32(dtype, V, H, n, pad):
    """ops.fused_dense.embedding: forward = F.embedding, weight gradient = fp32 index_add reference
    (runs far longer than one sort chunk when V is small), padding row zero, bitwise repeatable."""
    from beforeholiday_amd.ops import fused_dense as fd

    g = torch.Generator(device="cuda").manual_seed(V + H + n)
    ids = torch.randint(0, V, (n,), device="cuda", generator=g).view(-1, 1) if n % 2 else \
        torch.randint(0, V, (n // 2, 2), device="cuda", generator=g)
    w = (torch.randn(V, H, device="cuda", generator=g) * 0.1).to(dtype).requires_grad_(True)
    out = fd.embedding(ids, w, pad)
    torch.testing.assert_close(out, F.embedding(ids, w.detach(), pad), rtol=0, atol=0)
    dy = torch.randn(out.shape, device="cuda", generator=g).to(dtype)
    out.backward(dy)
    ref = torch.zeros(V, H, device="cuda").index_add_(0, ids.reshape(-1), dy.reshape(-1, H).float())
    if pad is not None:
        ref[pad] = 0
    tol = 1e-5 if dtype == torch.float32 else (1e-2 if dtype == torch.float16 else 4e-2)
    torch.testing.assert_close(w.grad.float(), ref, rtol=tol, atol=tol * max(1.0, (n / V) ** 0.5))
    g1 = w.grad.clone()
    w.grad = None
    fd.embedding(ids, w, pad).backward(dy)
    assert torch.equal(w.grad, g1)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_dense_mfma_paths_large(dtype):
    """16-bit FusedDense / FusedDenseGeluDense / MLP at >= 4096 rows: forward on the MFMA GEMM with the
    bias (GELU) epilogue, weight gradients on the MFMA weight-gradient kernel, dGELU + bias gradient in
    the data-gradient epilogue -- vs fp32 PyTorch."""
    from beforeholiday_amd.fused_dense import FusedDense, FusedDenseGeluDense
    from beforeholiday_amd.mlp import MLP

    torch.manual_seed(5)
    tol = dict(rtol=3e-2, atol=3e-2) if dtype == torch.float16 else dict(rtol=6e-2, atol=6e-2)
    x = (torch.randn(4096, 256, device="cuda") * 0.5).to(dtype).requires_grad_()
    xr = x.detach().float().requires_grad_()

    m = FusedDense(256, 128).cuda().to(dtype)
    w, b = m.weight.detach().float().requires_grad_(), m.bias.detach().float().requires_grad_()
    y, yr = m(x), F.linear(xr, w, b)
    torch.testing.assert_close(y.float(), yr, **tol)
    g = torch.randn_like(yr) * 0.1
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    torch.testing.assert_close(m.weight.grad.float(), w.grad, rtol=tol["rtol"], atol=tol["atol"] * 20)
    torch.testing.assert_close(m.bias.grad.float(), b.grad, rtol=tol["rtol"], atol=tol["atol"] * 20)

    x.grad = None
    xr.grad = None
    m2 = FusedDenseGeluDense(256, 512, 128).cuda().to(dtype)
    with torch.no_grad():  # (as test_fused_dense_gelu_dense: the 16-bit hidden activation rounds relative to
        for p in m2.parameters():  # its magnitude, so keep the two-layer outputs O(1))
            p.mul_(0.2)
    ps = [p.detach().float().requires_grad_() for p in (m2.weight, m2.bias, m2.weight2, m2.bias2)]
    y2 = m2(x)
    yr2 = F.linear(F.gelu(F.linear(xr, ps[0], ps[1])), ps[2], ps[3])
    torch.testing.assert_close(y2.float(), yr2, **tol)
    y2.backward(g.to(dtype))
    yr2.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    for p, r in zip((m2.weight, m2.bias, m2.weight2, m2.bias2), ps):
        torch.testing.assert_close(p.grad.float(), r.grad, rtol=tol["rtol"], atol=tol["atol"] * 20)

    for act in ("relu", "none"):
        x.grad = None
        mlp = MLP([256, 512, 128], bias=True, activation=act).cuda().to(dtype)
        ws = [t.detach().float().requires_grad_() for t in list(mlp.weights) + list(mlp.biases)]
        xr3 = x.detach().float().requires_grad_()
        h = xr3
        for i in range(2):
            h = F.linear(h, ws[i], ws[2 + i])
            h = torch.relu(h) if act == "relu" else h
        y3 = mlp(x)
        torch.testing.assert_close(y3.float(), h, **tol)
        y3.backward(g.to(dtype))
        h.backward(g)
        # (16-bit hidden activations and pre-activation gradients: a rare element lands ~1 rounding step
        # of the hidden layer past the single-layer tolerance)
        torch.testing.assert_close(x.grad.float(), xr3.grad, rtol=tol["rtol"], atol=2 * tol["atol"])
        for p, r in zip(list(mlp.weights) + list(mlp.biases), ws):
            torch.testing.assert_close(p.grad.float(), r.grad, rtol=tol["rtol"], atol=tol["atol"] * 20)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_reference_named_extensions_match_fp32(dt):
    """``import fused_dense_cuda`` / ``mlp_cuda`` after install_apex_aliases() reach the same native entry
    points as the Python layers (bindings/dense.cpp weight_grad / data_grad): linear_bias_backward,
    linear_gelu_linear_backward and mlp backward against fp32 autograd, at a token count (8192) where the
    weight gradients take the MFMA kernels (gemm_tn for the 1024 x 2048 weights, the 1x1 wgrad kernel for
    the 512 x 1024 one)."""
    import importlib

    import beforeholiday_amd

    beforeholiday_amd.install_apex_aliases()
    fd = importlib.import_module("fused_dense_cuda")
    mlp = importlib.import_module("mlp_cuda")
    torch.manual_seed(0)
    T, K, N = 8192, 1024, 2048
    x = (torch.randn(T, K, device="cuda") * 0.5).to(dt)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
    b = (torch.randn(N, device="cuda") * 0.1).to(dt)
    dy = torch.randn(T, N, device="cuda").to(dt)

    def rel(a, r):
        return float((a.float() - r).norm() / r.norm().clamp_min(1e-12))

    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    (torch.nn.functional.linear(xr, wr, br) * dy.float()).sum().backward()
    dx, dw, db = fd.linear_bias_backward(x, w, dy)
    assert rel(dx, xr.grad) < 1e-2 and rel(dw, wr.grad) < 1e-2 and rel(db, br.grad) < 1e-2

    w2 = (torch.randn(512, N, device="cuda") / N ** 0.5).to(dt)
    b2 = (torch.randn(512, device="cuda") * 0.1).to(dt)
    dy2 = torch.randn(T, 512, device="cuda").to(dt)
    gelu_in, out1, out2 = fd.linear_gelu_linear_forward(x, w, b, w2, b2)
    xr, wr, br, w2r, b2r = (t.float().requires_grad_() for t in (x, w, b, w2, b2))
    o2 = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(xr, wr, br)), w2r, b2r)
    (o2 * dy2.float()).sum().backward()
    g = fd.linear_gelu_linear_backward(x, gelu_in, out1, w, w2, dy2)
    for got, want in zip(g, (xr.grad, wr.grad, br.grad, w2r.grad, b2r.grad)):
        assert rel(got, want) < 2e-2

    # mlp_cuda: two ReLU layers with biases
    ws = [w, w2]
    bs = [b, b2]
    outs = mlp.forward(1, 1, [x] + ws + bs)
    xr = x.float().requires_grad_()
    wsr = [t.float().requires_grad_() for t in ws]
    bsr = [t.float().requires_grad_() for t in bs]
    h = xr
    for wi, bi in zip(wsr, bsr):
        h = torch.relu(torch.nn.functional.linear(h, wi, bi))
    (h * dy2.float()).sum().backward()
    x_req = x.clone().requires_grad_()
    grads = mlp.backward(1, 1, dy2, outs, [x_req] + ws + bs)
    # two ReLU masks taken from 16-bit activations: an exact 16-bit pipeline (fp32 accumulation, every
    # output rounded) is itself 1.2 % (fp16) / 3.2 % (bf16) from fp32 autograd in dx at this shape
    # (emulated on the CPU), so the bf16 gate is looser
    tol = 2e-2 if dt == torch.float16 else 4e-2
    for got, want in zip(grads, [xr.grad] + [t.grad for t in wsr] + [t.grad for t in bsr]):
        assert rel(got, want) < tol
