"""SyncBatchNorm / batch-norm kernels vs torch batch norm (fp32 reference), single and multi rank.

Modelled on tests/distributed/synced_batchnorm/{single_gpu_unit_test,two_gpu_unit_test}.py.
"""
import pytest
import torch
import torch.nn.functional as F

from beforeholiday_amd.parallel import SyncBatchNorm, PythonSyncBatchNorm, convert_syncbn_model

from _dist import run_distributed
from conftest import devices


def _ref_bn(x, w, b, z=None, relu=False, eps=1e-5):
    xf = x.float()
    y = F.batch_norm(xf, None, None, w.float(), b.float(), training=True, eps=eps)
    if z is not None:
        y = y + z.float()
    if relu:
        y = torch.relu(y)
    return y


# (2, 4096, 3, 3) / (2, 8200, 2, 1): channels_last shapes past the flat kernels' LDS cap (5 C floats in the
# data gradient, 2 C in the forward), which take the channel-owned 2-D kernels instead
SHAPES = [(8, 64, 14, 14), (4, 24, 7, 7), (16, 256, 1, 1), (3, 40, 9, 5), (32, 128), (2, 2048, 7, 7),
          (2, 4096, 3, 3), (2, 8200, 2, 1)]
TOL = {torch.float32: 2e-4, torch.float16: 4e-3, torch.bfloat16: 3e-2}


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("channels_last", [False, True])
@pytest.mark.parametrize("fuse", ["none", "relu", "add_relu"])
def test_syncbn_single_rank(device, shape, dtype, channels_last, fuse):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("cpu reference path is exercised in fp32")
    if channels_last and len(shape) != 4:
        pytest.skip("channels_last needs 4D")
    torch.manual_seed(0)
    C = shape[1]
    x = (torch.randn(shape) * 2 + 0.5).to(dtype)
    z = torch.randn(shape).to(dtype) if fuse == "add_relu" else None
    dy = torch.randn(shape).to(dtype)
    bn = SyncBatchNorm(C, fuse_relu=(fuse != "none"), channel_last=channels_last)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn = bn.to(device)
    x, dy = x.to(device), dy.to(device)
    if z is not None:
        z = z.to(device)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
        dy = dy.contiguous(memory_format=torch.channels_last)
        if z is not None:
            z = z.contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().cpu().requires_grad_(True)
    zr = z.detach().float().cpu().requires_grad_(True) if z is not None else None
    wr = bn.weight.detach().float().cpu().requires_grad_(True)
    br = bn.bias.detach().float().cpu().requires_grad_(True)
    yr = _ref_bn(xr, wr, br, zr, fuse != "none")
    yr.backward(dy.float().cpu())

    xg = x.detach().requires_grad_(True)
    zg = z.detach().requires_grad_(True) if z is not None else None
    y = bn(xg, zg) if zg is not None else bn(xg)
    y.backward(dy)
    tol = TOL[dtype]
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, rtol=tol * 5, atol=tol * 5)
    torch.testing.assert_close(bn.weight.grad.float().cpu(), wr.grad, rtol=tol * 10, atol=tol * 20)
    torch.testing.assert_close(bn.bias.grad.float().cpu(), br.grad, rtol=tol * 10, atol=tol * 20)
    if zg is not None:
        torch.testing.assert_close(zg.grad.float().cpu(), zr.grad, rtol=tol * 5, atol=tol * 5)
    # running stats: momentum 0.1 from (0, 1)
    xf = x.float().cpu()
    dims = [0] + list(range(2, xf.dim()))
    n = xf.numel() // C
    torch.testing.assert_close(bn.running_mean.cpu(), 0.1 * xf.mean(dims), rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var.cpu(), 0.9 + 0.1 * xf.var(dims, unbiased=True), rtol=1e-3, atol=1e-3)
    if channels_last:
        assert y.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("device", devices())
def test_syncbn_eval_matches_torch(device):
    torch.manual_seed(1)
    bn = SyncBatchNorm(32).to(device)
    ref = torch.nn.BatchNorm2d(32).to(device)
    ref.load_state_dict(bn.state_dict())
    for _ in range(3):
        x = torch.randn(4, 32, 6, 6, device=device)
        bn(x), ref(x)
    bn.eval(), ref.eval()
    x = torch.randn(4, 32, 6, 6, device=device)
    torch.testing.assert_close(bn(x), ref(x), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-5, atol=1e-5)


def test_fused_resnet_matches_unfused_cpu():
    from beforeholiday_amd.models import resnet18_like
    from beforeholiday_amd.models.resnet import Bottleneck, ResNet

    torch.manual_seed(0)
    ref = resnet18_like(num_classes=10)

    def norm(c, fuse_relu=False):
        return SyncBatchNorm(c, fuse_relu=fuse_relu)

    fused = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, norm_layer=norm, fused=True)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn(2, 3, 32, 32)
    torch.testing.assert_close(fused(x), ref(x), rtol=1e-4, atol=1e-4)


def _dist_syncbn(rank, world, channels_last):
    torch.manual_seed(0)
    N, C = 4 * world, 16
    x = torch.randn(N, C, 5, 5) * 3 + 1
    dy = torch.randn(N, C, 5, 5)
    ref = torch.nn.BatchNorm2d(C)
    for impl in (SyncBatchNorm, PythonSyncBatchNorm):
        bn = impl(C)
        bn.load_state_dict(ref.state_dict())
        xs = x[rank * 4:(rank + 1) * 4].clone().requires_grad_(True)
        y = bn(xs)
        y.backward(dy[rank * 4:(rank + 1) * 4])
        r = torch.nn.BatchNorm2d(C)
        r.load_state_dict(ref.state_dict())
        xr = x.clone().requires_grad_(True)
        yr = r(xr)
        yr.backward(dy)
        torch.testing.assert_close(y, yr[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(xs.grad, xr.grad[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(bn.running_mean, r.running_mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(bn.running_var, r.running_var, rtol=1e-5, atol=1e-5)
        # weight grads are local sums; DDP averages them -> all_reduce(sum) equals the full-batch grad
        gw = bn.weight.grad.clone()
        torch.distributed.all_reduce(gw)
        torch.testing.assert_close(gw, r.weight.grad, rtol=1e-4, atol=1e-4)


def test_syncbn_two_ranks_gloo():
    run_distributed(_dist_syncbn, 2, False)


def test_convert_syncbn_model():
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.Sequential(torch.nn.BatchNorm1d(4)),
                            torch.nn.InstanceNorm2d(8))
    m[1].running_mean.fill_(0.3)
    c = convert_syncbn_model(m)
    assert isinstance(c[1], SyncBatchNorm) and isinstance(c[2][0], SyncBatchNorm)
    assert isinstance(c[3], torch.nn.InstanceNorm2d)
    assert float(c[1].running_mean[0]) == pytest.approx(0.3)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("momentum", [0.1, None])
def test_num_batches_and_cumulative_momentum(device, momentum):
    torch.manual_seed(3)
    bn = SyncBatchNorm(16, momentum=momentum).to(device)
    ref = torch.nn.BatchNorm2d(16, momentum=momentum).to(device)
    for _ in range(3):
        x = torch.randn(4, 16, 5, 5, device=device)
        bn(x), ref(x)
    assert int(bn.num_batches_tracked) == 3
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gemm", "auto", "miopen"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_conv1x1_gemm_matches_conv(dtype, mode):
    from beforeholiday_amd.models.resnet import Conv1x1
    torch.manual_seed(0)
    m = Conv1x1(64, 96, 1, bias=False, mode=mode).cuda().to(dtype)
    x = torch.randn(4, 64, 14, 14, device="cuda", dtype=dtype).to(memory_format=torch.channels_last)
    x.requires_grad_()
    y = m(x)
    xr = x.detach().float().requires_grad_()
    w = m.weight.detach().float().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, w)
    tol = 1e-3 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(m.weight.grad.float(), w.grad, rtol=tol, atol=tol * 20)


def _dist_syncbn_uneven(rank, world):
    """Different per-rank batch sizes (reference: tests/distributed/synced_batchnorm/
    two_gpu_test_different_batch_size.py): stats are count-weighted, so the split run equals BN
    over the concatenated batch."""
    torch.manual_seed(1)
    sizes = [3 + 2 * r for r in range(world)]
    off = [sum(sizes[:r]) for r in range(world)]
    C = 8
    x = torch.randn(sum(sizes), C, 4, 3) * 2 - 0.5
    dy = torch.randn_like(x)
    ref = torch.nn.BatchNorm2d(C)
    for impl in (SyncBatchNorm, PythonSyncBatchNorm):
        bn = impl(C)
        bn.load_state_dict(ref.state_dict())
        sl = slice(off[rank], off[rank] + sizes[rank])
        xs = x[sl].clone().requires_grad_(True)
        bn(xs).backward(dy[sl])
        r = torch.nn.BatchNorm2d(C)
        r.load_state_dict(ref.state_dict())
        xr = x.clone().requires_grad_(True)
        yr = r(xr)
        yr.backward(dy)
        torch.testing.assert_close(xs.grad, xr.grad[sl], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(bn.running_mean, r.running_mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(bn.running_var, r.running_var, rtol=1e-5, atol=1e-5)


def test_syncbn_uneven_batches_gloo():
    run_distributed(_dist_syncbn_uneven, 2)


def _dist_syncbn_groups(rank, world):
    """Sub-group sync (reference: tests/distributed/synced_batchnorm/test_groups.py): 4 ranks in
    two BN groups of 2; each group's statistics are those of its own two shards only."""
    from beforeholiday_amd.parallel import create_syncbn_process_group
    group = create_syncbn_process_group(2)
    torch.manual_seed(2)
    C, n = 6, 3
    x = torch.randn(world * n, C, 5) + torch.arange(world * n).view(-1, 1, 1) * 0.1
    dy = torch.randn_like(x)
    g0 = (rank // 2) * 2
    for impl in (SyncBatchNorm, PythonSyncBatchNorm):
        bn = impl(C, process_group=group)
        xs = x[rank * n:(rank + 1) * n].clone().requires_grad_(True)
        y = bn(xs)
        y.backward(dy[rank * n:(rank + 1) * n])
        r = torch.nn.BatchNorm1d(C)
        xr = x[g0 * n:(g0 + 2) * n].clone().requires_grad_(True)
        yr = r(xr)
        yr.backward(dy[g0 * n:(g0 + 2) * n])
        loc = slice((rank - g0) * n, (rank - g0 + 1) * n)
        torch.testing.assert_close(y, yr[loc], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(xs.grad, xr.grad[loc], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(bn.running_var, r.running_var, rtol=1e-5, atol=1e-5)


def test_syncbn_process_subgroups_gloo():
    run_distributed(_dist_syncbn_groups, 4)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape,pool", [((4, 64, 18, 18), (3, 2, 1)), ((2, 16, 9, 7), (3, 2, 1)),
                                        ((2, 32, 8, 8), (2, 2, 0)), ((3, 8, 11, 10), (3, 1, 1))])
def test_bn_relu_maxpool_fused(device, dtype, shape, pool):
    """ResNet stem: SyncBN(fuse_relu, fuse_maxpool) == max_pool2d(relu(batch_norm(x))) fwd + bwd."""
    torch.manual_seed(7)
    C = shape[1]
    x = (torch.randn(shape, device=device) * 2 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    bn = SyncBatchNorm(C, channel_last=True, fuse_relu=True, fuse_maxpool=pool).to(device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    w, b = bn.weight.detach().clone(), bn.bias.detach().clone()
    xs = x.clone().requires_grad_(True)
    y = bn(xs)
    xr = x.float().clone().requires_grad_(True)
    yr = F.max_pool2d(_ref_bn(xr, w, b, relu=True), *pool)
    tol = TOL[dtype]
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    gy = torch.randn_like(yr)
    y.backward(gy.to(dtype))
    yr.backward(gy)
    # ties between equal rounded values may route a gradient differently: compare in norm
    err = (xs.grad.float() - xr.grad).norm() / xr.grad.norm()
    assert err < (2e-3 if dtype == torch.float32 else 3e-2), float(err)
    assert int(bn.num_batches_tracked) == 1
    bn.eval()
    ye = bn(x)
    ref_e = F.max_pool2d(torch.relu(F.batch_norm(x.float(), bn.running_mean, bn.running_var, w, b, False)), *pool)
    torch.testing.assert_close(ye.float(), ref_e, rtol=tol, atol=tol)


@pytest.mark.parametrize("device", devices())
def test_maxpool_ties_and_nan_match_torch(device):
    """Exact argmax semantics: first maximum of the window wins, NaN propagates."""
    x = torch.randint(0, 3, (2, 16, 9, 9), device=device).float().contiguous(memory_format=torch.channels_last)
    x[0, 3, 4, 4] = float("nan")
    from beforeholiday_amd.ops import syncbn
    y, idx = syncbn.maxpool_forward(x, None, None, False, 3, 2, 1, True)
    yr, _ = F.max_pool2d(x, 3, 2, 1, return_indices=True)
    torch.testing.assert_close(y, yr, equal_nan=True)
    gy = torch.randn_like(yr).contiguous(memory_format=torch.channels_last)
    gx = syncbn.maxpool_backward(gy, idx, 9, 9, 3, 2, 1)
    xr = x.clone().requires_grad_(True)
    F.max_pool2d(xr, 3, 2, 1).backward(gy)
    torch.testing.assert_close(gx, xr.grad)


def test_fused_stem_resnet_matches_unfused_cpu():
    from beforeholiday_amd.models import resnet18_like
    from beforeholiday_amd.models.resnet import Bottleneck, ResNet

    torch.manual_seed(0)
    ref = resnet18_like(num_classes=10)

    def norm(c, fuse_relu=False, fuse_maxpool=None):
        return SyncBatchNorm(c, fuse_relu=fuse_relu, channel_last=True, fuse_maxpool=fuse_maxpool)

    fused = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, norm_layer=norm, fused=True, stem_pool_fused=True)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(fused(x), ref(x), rtol=1e-3, atol=3e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 64, 9, 7), (3, 24, 5, 5), (64, 16)])
def test_relu_bitmask_forward(shape):
    """forward_mask packs (x*scale + shift + z > 0) 8 channels per byte, row-major [rows, C/8], and the
    BN + add + ReLU autograd function takes that path (z is not saved for backward)."""
    from beforeholiday_amd.ops import syncbn

    torch.manual_seed(3)
    C = shape[1]
    x = torch.randn(shape, device="cuda", dtype=torch.float16)
    z = torch.randn(shape, device="cuda", dtype=torch.float16)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
        z = z.contiguous(memory_format=torch.channels_last)
    scale = torch.rand(C, device="cuda") + 0.5
    shift = torch.randn(C, device="cuda") * 0.1
    assert syncbn.mask_ok(x, z)
    y, mask = syncbn.forward_mask(x, z, scale, shift)
    view = (lambda t: t.permute(0, 2, 3, 1).reshape(-1, C)) if x.dim() == 4 else (lambda t: t)
    pre = view(x).float() * scale + shift + view(z).float()
    bits = (pre > 0).to(torch.int32).view(-1, C // 8, 8)
    ref = (bits << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8)
    assert mask.shape == (pre.shape[0], C // 8) and mask.dtype == torch.uint8
    torch.testing.assert_close(mask, ref, rtol=0, atol=0)
    torch.testing.assert_close(view(y).float(), torch.relu(pre), rtol=4e-3, atol=4e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["allgather", "allreduce"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("channels_last", [True, False])
def test_multirank_stats_kernels_on_shards(mode, dtype, channels_last):
    """The native multi-rank path of SyncBatchNorm (the one every 8-GPU BN layer takes), driven on one
    GPU: W shards -> per-shard payloads (stats_local / stats_local_sums) -> the collective emulated by
    stacking / summing -> merge_ranks / merge_sums, vs fp32 full-batch statistics and running stats."""
    from beforeholiday_amd.ops import syncbn as sb

    torch.manual_seed(7)
    W, C = 4, 64
    shards = [torch.randn(3 + r, C, 7, 5, device="cuda") * 2.5 + 40 for r in range(W)]  # uneven, large mean
    if channels_last:
        shards = [s.to(memory_format=torch.channels_last) for s in shards]
    shards = [s.to(dtype) for s in shards]
    full = torch.cat([s.float() for s in shards])
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    rm = torch.randn(C, device="cuda") + 39.0
    rv = torch.rand(C, device="cuda") + 1.0
    rm_ref, rv_ref = rm.clone(), rv.clone()
    if mode == "allgather":
        g = torch.stack([sb.stats_local(s) for s in shards])
        mean, invstd, scale, shift, count = sb.merge_ranks(g, w, b, rm, rv, 0.1, 1e-5)
    else:
        tot = sum(sb.stats_local_sums(s, rm) for s in shards)
        mean, invstd, scale, shift, count = sb.merge_sums(tot, w, b, rm, rv, 0.1, 1e-5)
    m_ref = full.mean((0, 2, 3))
    v_ref = full.var((0, 2, 3), unbiased=False)
    n = full.numel() // C
    torch.testing.assert_close(mean, m_ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(invstd, torch.rsqrt(v_ref + 1e-5), rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(scale, w * torch.rsqrt(v_ref + 1e-5), rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(shift, b - m_ref * w * torch.rsqrt(v_ref + 1e-5), rtol=2e-4, atol=2e-3)
    assert float(count[0]) == n
    torch.testing.assert_close(rm, 0.9 * rm_ref + 0.1 * m_ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(rv, 0.9 * rv_ref + 0.1 * v_ref * n / (n - 1), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gemm", "auto"])
def test_fused_resnet_residual_grad_folded_into_conv1(mode):
    """Bottleneck backward with the residual-branch gradient summed inside conv1's data-gradient GEMM
    (beta = 1) equals the plain autograd sum (same model with MIOpen 1x1 convolutions)."""
    from beforeholiday_amd.models import resnet as R
    torch.manual_seed(0)

    def build(m):
        old, R._CONV1X1_MODE = R._CONV1X1_MODE, m
        try:
            torch.manual_seed(0)
            norm = lambda c, fuse_relu=False, fuse_maxpool=None: SyncBatchNorm(  # noqa: E731
                c, channel_last=True, fuse_relu=fuse_relu, fuse_maxpool=fuse_maxpool)
            return R.ResNet(R.Bottleneck, [2, 2, 1, 1], num_classes=10, norm_layer=norm, fused=True,
                            stem_pool_fused=True).cuda().to(memory_format=torch.channels_last)
        finally:
            R._CONV1X1_MODE = old

    ref, fold = build("miopen"), build(mode)
    fold.load_state_dict(ref.state_dict())
    assert any(isinstance(m, R.Conv1x1) for m in fold.modules())
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    xr, xf = x.clone().requires_grad_(), x.clone().requires_grad_()
    ref(xr).square().sum().backward()
    fold(xf).square().sum().backward()
    torch.testing.assert_close(xf.grad, xr.grad, rtol=2e-3, atol=2e-3)
    for (n, p), q in zip(fold.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=2e-3, atol=2e-3, msg=n)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("G,C", [(1, 64), (37, 256), (515, 2048), (1024, 64), (2048, 64), (7168, 128), (20000, 192)])
def test_merge_parts_equals_sum_parts_then_merge_sums(device, G, C):
    """Single-rank finalize from conv-epilogue partials [2, G, C] (one kernel) == sum_parts +
    merge_sums, bit for bit (same summation order), including the running-stat update; and both match
    the fp64 statistics of the partials."""
    from beforeholiday_amd.ops import conv_bn, syncbn as sb

    g = torch.Generator().manual_seed(G)
    n = 4096.0 * G
    rm0 = torch.randn(C, generator=g) * 0.1
    rv0 = torch.rand(C, generator=g) + 0.5
    d = torch.randn(G, C, generator=g) * 3 + 1
    part = torch.stack([d * 64, d * d * 64 + 4096]).contiguous().to(device)
    w = (torch.rand(C, generator=g) + 0.5).to(device)
    b = torch.randn(C, generator=g).to(device)
    rm_a, rv_a, rm_b, rv_b = (t.clone().to(device) for t in (rm0, rv0, rm0, rv0))
    out_a = sb.merge_parts(part, n, w, b, rm_a, rv_a, 0.1, 1e-5)
    out_b = sb.merge_sums(conv_bn.sum_parts(part, n), w, b, rm_b, rv_b, 0.1, 1e-5)
    for a_, b_ in zip(list(out_a) + [rm_a, rv_a], list(out_b) + [rm_b, rv_b]):
        torch.testing.assert_close(a_.cpu(), b_.cpu(), rtol=0 if device == "cuda" else 1e-6, atol=0 if device == "cuda" else 1e-6)
    s1 = part[0].double().sum(0).cpu()
    s2 = part[1].double().sum(0).cpu()
    mean = rm0.double() + s1 / n
    var = (s2 - s1 * s1 / n) / n
    torch.testing.assert_close(out_a[0].cpu().double(), mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out_a[1].cpu().double(), (var + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
