"""1x1 convolution GEMMs with BatchNorm prologue / epilogues (kernels/conv_bn.hip) against fp32 PyTorch.

Shapes are the ResNet-50 bottleneck's 1x1 layers (channels) on small pixel counts. Each GPU case
compares the HIP kernel with the fp32 reference of ``ops.conv_bn`` (``F.linear`` on the fp32 upcast,
BatchNorm prologue applied in fp32 and rounded like the kernel): the output to fp16 / bf16 rounding,
the statistics partial sums to fp32 summation-order tolerance.
"""
import pytest
import torch

from beforeholiday_amd.ops import conv_bn

SHAPES = [  # (K, N): forward and data-gradient directions of the bottleneck 1x1 convs
    (64, 64), (64, 256), (256, 64), (128, 512), (512, 128), (256, 1024), (1024, 256), (512, 2048), (128, 128),
]


def _tol(dt):
    return dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=5e-3, atol=5e-3)


def _data(M, K, N, dt, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    a = (torch.randn(M, K, generator=g)).to(dt).to(dev)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).to(dev)
    return a, b


def _stats_close(got, ref, rows):
    # partial sums over rows: fp32 accumulation in different orders
    torch.testing.assert_close(got.float().cpu(), ref.float().cpu(), rtol=2e-3, atol=2e-3 * rows ** 0.5)


def test_reference_cpu_matches_definition():
    a, b = _data(64, 64, 64, torch.float32, "cpu")
    sc, sh = torch.rand(64) + 0.5, torch.randn(64)
    c, part = conv_bn.c1x1(a, b, sc, sh, epi="stats")
    ref = torch.relu(a * sc + sh) @ b.t()
    torch.testing.assert_close(c, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv_bn.sum_parts(part, 64)[:64], ref.sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN", SHAPES)
def test_c1x1_plain_and_stats(KN, dt):
    K, N = KN
    M = 2048
    a, b = _data(M, K, N, dt, "cuda")
    assert conv_bn.supported(a, b, epi="stats")
    kshift = torch.randn(N, device="cuda") * 0.1
    c, part = conv_bn.c1x1(a, b, epi="stats", kshift=kshift)
    rc, rpart = conv_bn.c1x1(a.cpu(), b.cpu(), epi="stats", kshift=kshift.cpu())
    torch.testing.assert_close(c.float().cpu(), rc.float(), **_tol(dt))
    # statistics of the stored output: compare against the reference statistics of OUR output
    cf = c.float().cpu() - kshift.cpu()
    _stats_close(conv_bn.sum_parts(part, M)[:2 * N], torch.cat([cf.sum(0), (cf * cf).sum(0)]), M)
    assert float(conv_bn.sum_parts(part, M)[-1]) == M
    c2, p2 = conv_bn.c1x1(a, b)
    torch.testing.assert_close(c2, c, rtol=0, atol=0)
    assert p2.numel() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN", [(64, 256), (128, 512), (256, 1024), (512, 2048), (64, 64)])
def test_c1x1_bn_prologue(KN, dt):
    """conv3 of the bottleneck: input = relu(BN2(y2)) applied on the fly."""
    K, N = KN
    M = 1024
    a, b = _data(M, K, N, dt, "cuda", seed=1)
    sc = (torch.rand(K) + 0.5).cuda()
    sh = torch.randn(K).cuda() * 0.5
    c, part = conv_bn.c1x1(a, b, sc, sh, epi="stats")
    rc, _ = conv_bn.c1x1(a.cpu(), b.cpu(), sc.cpu(), sh.cpu(), epi="stats")
    torch.testing.assert_close(c.float().cpu(), rc.float(), **_tol(dt))
    cf = c.float().cpu()
    _stats_close(conv_bn.sum_parts(part)[:N], cf.sum(0), M)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KNHW", [(64, 256, 8, 8), (256, 512, 12, 8), (512, 1024, 4, 16)])
def test_c1x1_stride2_gather(KNHW, dt):
    K, N, H, W = KNHW
    n = 4
    a, b = _data(n * H * W, K, N, dt, "cuda", seed=2)
    assert conv_bn.supported(a, b, s2=(H, W), epi="stats")
    c, part = conv_bn.c1x1(a, b, s2=(H, W), epi="stats")
    ref = torch.nn.functional.conv2d(a.float().cpu().view(n, H, W, K).permute(0, 3, 1, 2),
                                     b.float().cpu().view(N, K, 1, 1), stride=2)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, N)
    torch.testing.assert_close(c.float().cpu(), ref, **_tol(dt))
    _stats_close(conv_bn.sum_parts(part)[:N], c.float().cpu().sum(0), ref.size(0))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN", [(64, 256), (256, 64), (128, 512), (64, 64)])
def test_c1x1_residual(KN, dt):
    K, N = KN
    M = 1024
    a, b = _data(M, K, N, dt, "cuda", seed=3)
    r = torch.randn(M, N, device="cuda").to(dt)
    c, _ = conv_bn.c1x1(a, b, resid=r)
    ref = (a.float() @ b.float().t() + r.float())
    torch.testing.assert_close(c.float(), ref, **_tol(dt))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN", [(256, 64), (512, 128), (1024, 256), (64, 64), (128, 256)])
@pytest.mark.parametrize("resid", [False, True])
def test_c1x1_bn_backward_epilogue(KN, dt, resid):
    """Data gradient dA = dY . W with the previous BatchNorm's backward sums in the epilogue:
    sum(dz), sum(dz * (y - mean)), dz = dA * (y*scale + shift > 0) -- syncbn.backward_reduce."""
    from beforeholiday_amd.ops import syncbn

    K, N = KN
    M = 1024
    a, b = _data(M, K, N, dt, "cuda", seed=4)
    y = (torch.randn(M, N) * 2 + 0.3).to(dt).cuda()
    sc = (torch.rand(N) + 0.5).cuda()
    sh = torch.randn(N).cuda() * 0.3
    mean = torch.randn(N).cuda() * 0.1
    r = torch.randn(M, N, device="cuda").to(dt) if resid else None
    if not conv_bn.supported(a, b, resid=resid, epi="bwd"):
        pytest.skip("shape outside the backward-epilogue kernel")
    c, part = conv_bn.c1x1(a, b, resid=r, epi="bwd", by=y, bscale=sc, bshift=sh, bmean=mean)
    ref = a.float() @ b.float().t() + (r.float() if resid else 0)
    torch.testing.assert_close(c.float(), ref, **_tol(dt))
    # the sums must equal syncbn.backward_reduce of (dA as stored, y) -- the unfused path
    x4 = y.view(1, 1, M, N).permute(0, 3, 1, 2)
    dy4 = c.view(1, 1, M, N).permute(0, 3, 1, 2)
    sums, _, _ = syncbn.backward_reduce(dy4.cpu().float(), x4.cpu().float(), None, mean.cpu(), None, sc.cpu(),
                                        sh.cpu(), True, None, False)
    _stats_close(conv_bn.sum_parts(part), sums, M)


@pytest.mark.gpu
def test_c1x1_rejects_unsupported():
    a = torch.randn(100, 64, device="cuda", dtype=torch.float16)  # M % 32 != 0
    b = torch.randn(64, 64, device="cuda", dtype=torch.float16)
    assert not conv_bn.supported(a, b)
    with pytest.raises(RuntimeError):
        conv_bn.c1x1(a, b)


# ---------------------------------------------------------------- 3x3 kernel with BatchNorm folding
def _conv3x3_ref(x, w, sc=None, sh=None):
    xf = x.float()
    if sc is not None:
        xf = torch.relu(xf * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)).to(x.dtype).float()
    return torch.nn.functional.conv2d(xf, w.float(), padding=1)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (4, 128, 28, 28), (8, 256, 14, 14), (8, 512, 7, 7), (3, 64, 9, 13)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv3x3_bn_forward(shape, dt, pro):
    from beforeholiday_amd._native import submodule

    n, c, h, w_ = shape
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, c, h, w_, generator=g).to(dt).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, generator=g) / (9 * c) ** 0.5).to(dt).cuda().contiguous(memory_format=torch.channels_last)
    sc = (torch.rand(c, generator=g) + 0.5).cuda() if pro else None
    sh = (torch.randn(c, generator=g) * 0.5).cuda() if pro else None
    kshift = torch.randn(c, generator=g).cuda() * 0.1
    y, part = submodule("conv_cuda").conv3x3_bn_forward(x, w, sc, sh, True, kshift)
    ref = _conv3x3_ref(x, w, sc, sh)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, c).cpu() - kshift.cpu()
    _stats_close(conv_bn.sum_parts(part)[:2 * c], torch.cat([yf.sum(0), (yf * yf).sum(0)]), yf.size(0))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (8, 256, 14, 14), (8, 512, 7, 7)])
def test_conv3x3_bn_dgrad_epilogue(shape, dt):
    from beforeholiday_amd._native import submodule
    from beforeholiday_amd.ops import syncbn

    n, c, h, w_ = shape
    g = torch.Generator().manual_seed(6)
    dy = torch.randn(n, c, h, w_, generator=g).to(dt).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, generator=g) / (9 * c) ** 0.5).to(dt).cuda().contiguous(memory_format=torch.channels_last)
    y1 = (torch.randn(n, c, h, w_, generator=g) * 2 + 0.2).to(dt).cuda().contiguous(memory_format=torch.channels_last)
    sc, sh = (torch.rand(c, generator=g) + 0.5).cuda(), (torch.randn(c, generator=g) * 0.3).cuda()
    mean = (torch.randn(c, generator=g) * 0.1).cuda()
    dx, part = submodule("conv_cuda").conv3x3_bn_dgrad(dy, w, y1, sc, sh, mean, True)
    ref = torch.nn.grad.conv2d_input(dy.shape, w.float(), dy.float(), padding=1)
    torch.testing.assert_close(dx.float(), ref, **_tol(dt))
    sums, _, _ = syncbn.backward_reduce(dx.float().cpu(), y1.float().cpu(), None, mean.cpu(), None, sc.cpu(),
                                        sh.cpu(), True, None, False)
    _stats_close(conv_bn.sum_parts(part), sums, n * h * w_)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN", [(512, 128), (1024, 256), (256, 1024), (512, 2048), (128, 512)])
@pytest.mark.parametrize("epi", ["stats", "bwd"])
def test_gemm_bn_epilogues(KN, dt, epi):
    """Tiled MFMA GEMM (kernels/gemm.hip) with the BatchNorm statistics / backward-sum epilogues."""
    from beforeholiday_amd.ops import syncbn

    K, N = KN
    M = 1000  # not a multiple of the tile: the last slab is partial
    a, b = _data(M, K, N, dt, "cuda", seed=7)
    kshift = torch.randn(N, device="cuda") * 0.1
    y = (torch.randn(M, N) * 2 + 0.3).to(dt).cuda()
    sc, sh = (torch.rand(N) + 0.5).cuda(), torch.randn(N).cuda() * 0.3
    mean = torch.randn(N).cuda() * 0.1
    if epi == "stats":
        c, part = conv_bn.gemm_bn(a, b, "stats", kshift=kshift)
    else:
        c, part = conv_bn.gemm_bn(a, b, "bwd", by=y, bscale=sc, bshift=sh, bmean=mean)
    torch.testing.assert_close(c.float(), a.float() @ b.float().t(), **_tol(dt))
    cf = c.float().cpu()
    if epi == "stats":
        d = cf - kshift.cpu()
        ref = torch.cat([d.sum(0), (d * d).sum(0)])
    else:
        ref, _, _ = syncbn.backward_reduce(cf.t().reshape(1, N, M, 1), y.float().cpu().t().reshape(1, N, M, 1), None,
                                           mean.cpu(), None, sc.cpu(), sh.cpu(), True, None, False)
    _stats_close(conv_bn.sum_parts(part), ref, M)


def test_c1x1_scatter_reference_cpu():
    a = torch.randn(2 * 3 * 4, 8)
    b = torch.randn(16, 8)
    base = torch.randn(2 * 6 * 8, 16)
    out, _ = conv_bn.c1x1(a, b, s2=(6, 8), s2_scatter=True, resid=base.clone())
    ref = base.clone().view(2, 6, 8, 16)
    ref[:, ::2, ::2, :] += (a @ b.t()).view(2, 3, 4, 16)
    torch.testing.assert_close(out.view(2, 6, 8, 16), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KNHW", [(512, 256, 8, 8), (1024, 512, 12, 8), (256, 64, 4, 16)])
def test_c1x1_stride2_scatter_accumulate(KNHW, dt):
    """dX += scatter(dY_ds . W_ds): the downsample data gradient added at the even pixels in place."""
    K, N, H, W = KNHW
    n = 4
    a, _ = _data(n * (H // 2) * (W // 2), K, N, dt, "cuda", seed=8)
    w = (torch.randn(K, N) / K ** 0.5).to(dt).cuda()  # forward weight [Cout=K, Cin=N]: b_trans
    base = torch.randn(n * H * W, N, device="cuda").to(dt)
    assert conv_bn.supported(a, w, b_trans=True, s2=(H, W), s2_scatter=True)
    ref = base.float().clone().view(n, H, W, N)
    ref[:, ::2, ::2, :] += (a.float() @ w.float()).view(n, H // 2, W // 2, N)
    out, _ = conv_bn.c1x1(a, w, b_trans=True, s2=(H, W), s2_scatter=True, resid=base)
    assert out.data_ptr() == base.data_ptr()
    torch.testing.assert_close(out.float().view(n, H, W, N), ref, **_tol(dt))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("MKN", [(33000, 256, 512), (16500, 512, 1024), (12544, 512, 2048)])
def test_gemm_bn_stats_pingpong(MKN, dt):
    """Grids of >= 256 256x256 tiles take the ping-pong kernel with the statistics epilogue (the
    ResNet-50 conv3 / downsample layers of stages 2-4); partial last tile included."""
    M, K, N = MKN
    a, b = _data(M, K, N, dt, "cuda", seed=11)
    kshift = torch.randn(N, device="cuda") * 0.1
    c, part = conv_bn.gemm_bn(a, b, "stats", kshift=kshift)
    assert part.shape == (2, (M + 63) // 64, N)
    torch.testing.assert_close(c.float(), a.float() @ b.float().t(), **_tol(dt))
    d = c.float() - kshift
    ref = torch.cat([d.sum(0), (d * d).sum(0)]).cpu()
    _stats_close(conv_bn.sum_parts(part).cpu(), ref, M)


def _bwd_sums_ref(c, y, sc, sh, mean):
    # the ReLU mask in float64: y * sc is exact there, so the sign matches the kernels' fused fmaf
    # (a float32 mul + add can round a tiny positive pre-activation to zero or flip it)
    cf, yf = c.float(), y.float()
    dz = cf * ((y.double() * sc.double() + sh.double()) > 0).float()
    return torch.cat([dz.sum(0), (dz * (yf - mean)).sum(0)])


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("MKN", [(200704, 128, 512), (50176, 256, 1024), (12544, 512, 2048), (50000, 1024, 256),
                                 (200704, 512, 128)])
@pytest.mark.parametrize("mode", ["bwd", "plain_resid", "bwd_resid"])
def test_gemm_bn_large_bwd_and_resid(MKN, dt, mode):
    """The ResNet-50 (batch 256) data-gradient GEMMs at their real row counts (12.5k - 200k rows, so
    the large-grid slab partials and the ping-pong kernel's backward-sums / residual epilogues are
    exercised): C = A.B^T (+ resid) against the fp32 product, and the previous BatchNorm's backward
    sums against an fp32 reduction of OUR stored output."""
    M, K, N = MKN
    torch.manual_seed(13)
    a, b = _data(M, K, N, dt, "cuda", seed=13)
    resid = (torch.randn(M, N, device="cuda") * 0.5).to(dt) if "resid" in mode else None
    y = (torch.randn(M, N, device="cuda") * 2 + 0.3).to(dt)
    sc, sh = torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda") * 0.3
    mean = torch.randn(N, device="cuda") * 0.1
    if mode.startswith("bwd"):
        c, part = conv_bn.gemm_bn(a, b, "bwd", by=y, bscale=sc, bshift=sh, bmean=mean, resid=resid)
        assert part.shape == (2, (M + 63) // 64, N)
    else:
        c, part = conv_bn.gemm_bn(a, b, "plain", resid=resid)
        assert part is None
    ref = a.float() @ b.float().t()
    if resid is not None:
        ref = ref + resid.float()
    torch.testing.assert_close(c.float(), ref, **_tol(dt))
    if part is not None:
        _stats_close(conv_bn.sum_parts(part).cpu(), _bwd_sums_ref(c, y, sc, sh, mean).cpu(), M)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("KN,epi", [((64, 256), "stats"), ((256, 64), "stats"), ((64, 64), "pro"),
                                    ((256, 64), "bwd"), ((64, 256), "bwd")])
def test_c1x1_large_m(KN, epi, dt):
    """The strip kernel at the ResNet-50 stage-1 row count (256 x 56 x 56 = 802,816 rows): the
    grid-wide partial layout and sum_parts at the model's real scale."""
    K, N = KN
    M = 256 * 56 * 56
    torch.manual_seed(17)
    a, b = _data(M, K, N, dt, "cuda", seed=17)
    kshift = torch.randn(N, device="cuda") * 0.1
    if epi == "bwd":
        y = (torch.randn(M, N, device="cuda") * 2 + 0.3).to(dt)
        sc, sh = torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda") * 0.3
        mean = torch.randn(N, device="cuda") * 0.1
        w = b.t().contiguous()  # the data gradient reads the forward weight [K, N] transposed
        assert conv_bn.supported(a, w, epi="bwd", b_trans=True)
        c, part = conv_bn.c1x1(a, w, epi="bwd", by=y, bscale=sc, bshift=sh, bmean=mean, b_trans=True)
        torch.testing.assert_close(c.float(), a.float() @ b.float().t(), **_tol(dt))
        _stats_close(conv_bn.sum_parts(part).cpu(), _bwd_sums_ref(c, y, sc, sh, mean).cpu(), M)
        return
    if epi == "pro":
        ps, pb = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
        c, part = conv_bn.c1x1(a, b, pro_scale=ps, pro_shift=pb, epi="stats", kshift=kshift)
        af = torch.relu(a.float() * ps + pb).to(dt).float()
    else:
        c, part = conv_bn.c1x1(a, b, epi="stats", kshift=kshift)
        af = a.float()
    torch.testing.assert_close(c.float(), af @ b.float().t(), **_tol(dt))
    d = c.float() - kshift
    _stats_close(conv_bn.sum_parts(part, M)[:2 * N].cpu(), torch.cat([d.sum(0), (d * d).sum(0)]).cpu(), M)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_s2_gather_scatter_add(dtype):
    """The 16-byte-vector stride-2 pixel gather / scatter-add of the 1x1 stride-2 convolutions vs torch's
    strided views (bitwise: one add per element)."""
    from beforeholiday_amd.ops import conv_bn

    torch.manual_seed(0)
    x = torch.randn(3, 40, 14, 10, device="cuda", dtype=dtype).contiguous(memory_format=torch.channels_last)
    q = conv_bn.s2_gather(x)
    assert q.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(q, x[:, :, ::2, ::2])
    full = torch.randn(3 * 14 * 10, 40, device="cuda", dtype=dtype)
    quarter = torch.randn(3 * 7 * 5, 40, device="cuda", dtype=dtype)
    ref = full.clone()
    ref.view(3, 14, 10, 40)[:, ::2, ::2, :].add_(quarter.view(3, 7, 5, 40))
    out = conv_bn.s2_scatter_add(full, quarter, 3, 14, 10)
    assert out.data_ptr() == full.data_ptr() and torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_pool_broadcast(dtype):
    """The global-average-pool backward kernel vs torch's expand + channels_last copy (fp32 scale, one
    rounding, so equal to rounding of g / hw)."""
    from beforeholiday_amd._native import submodule

    g = torch.randn(5, 48, device="cuda", dtype=dtype)
    out = submodule("conv_bn").pool_broadcast(g, 7, 3, 1.0 / 21)
    ref = (g.float() / 21).view(5, 48, 1, 1).expand(5, 48, 7, 3)
    assert out.is_contiguous(memory_format=torch.channels_last) and out.shape == (5, 48, 7, 3)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-3)
