"""contrib: groupbn, bottleneck (+ spatial H-split with halo exchange), halo exchangers, nccl_p2p,
peer_memory, fmha (reference tests: apex/contrib/test/{groupbn,bottleneck,peer_memory,fmha})."""
import types

import pytest
import torch
import torch.nn.functional as F

from tests._dist import run_distributed
from tests.conftest import devices


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("fuse_relu", [False, True])
def test_groupbn_nhwc(device, fuse_relu):
    from beforeholiday_amd.contrib.groupbn import BatchNorm2d_NHWC
    torch.manual_seed(0)
    bn = BatchNorm2d_NHWC(16, fuse_relu=fuse_relu).to(device)
    ref = torch.nn.BatchNorm2d(16).to(device)
    x = torch.randn(4, 6, 6, 16, device=device, requires_grad=True)  # physical NHWC
    z = torch.randn(4, 6, 6, 16, device=device, requires_grad=True) if fuse_relu else None
    y = bn(x, z)
    xr = x.detach().permute(0, 3, 1, 2).clone().requires_grad_()
    yr = ref(xr)
    if fuse_relu:
        zr = z.detach().permute(0, 3, 1, 2).clone().requires_grad_()
        yr = torch.relu(yr + zr)
    yr = yr.permute(0, 2, 3, 1)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad.permute(0, 2, 3, 1), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)


def _ref_bottleneck(m, x):
    def fbn(bn, t):
        s, b = bn.get_scale_bias()
        return t * s + b
    out = torch.relu(fbn(m.bn1, F.conv2d(x, m.conv1.weight, stride=m.stride)))
    out = torch.relu(fbn(m.bn2, F.conv2d(out, m.conv2.weight, padding=1)))
    out = fbn(m.bn3, F.conv2d(out, m.conv3.weight))
    idn = fbn(m.downsample[1], F.conv2d(x, m.downsample[0].weight, stride=m.stride)) if m.downsample is not None else x
    return torch.relu(out + idn)


def _randomize_bn(m):
    with torch.no_grad():
        for mod in m.modules():
            if mod.__class__.__name__ == "FrozenBatchNorm2d":
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("stride,cin", [(1, 32), (2, 16)])
def test_bottleneck(device, stride, cin):
    from beforeholiday_amd.contrib.bottleneck import Bottleneck
    torch.manual_seed(1)
    m = Bottleneck(cin, 8, 32, stride=stride).to(device)
    _randomize_bn(m)
    x = torch.randn(2, cin, 8, 8, device=device).to(memory_format=torch.channels_last).requires_grad_()
    y = m(x)
    xr = x.detach().clone().requires_grad_()
    yr = _ref_bottleneck(m, xr)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g)
    grads = [w.grad.clone() for w in m.w_conv]
    for w in m.w_conv:
        w.grad = None
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    for a, w in zip(grads, m.w_conv):
        torch.testing.assert_close(a, w.grad, rtol=1e-4, atol=1e-3)


def _spatial(rank, world):
    from beforeholiday_amd.contrib.bottleneck import Bottleneck, SpatialBottleneck
    from beforeholiday_amd.contrib.bottleneck.halo_exchangers import HaloExchangerSendRecv
    torch.manual_seed(2)
    ref = Bottleneck(16, 8, 16)
    _randomize_bn(ref)
    sp = SpatialBottleneck(16, 8, 16, spatial_parallel_args=(world, rank, None,
                                                            HaloExchangerSendRecv(list(range(world)), rank)))
    sp.load_state_dict(ref.state_dict())
    torch.manual_seed(3)
    H = 4 if world == 2 else 3
    x = torch.randn(2, 16, H * world, 6)
    xs = x[:, :, rank * H:(rank + 1) * H].clone().requires_grad_()
    y = sp(xs)
    xr = x.clone().requires_grad_()
    yr = ref(xr)
    torch.testing.assert_close(y, yr[:, :, rank * H:(rank + 1) * H], rtol=1e-4, atol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g[:, :, rank * H:(rank + 1) * H])
    yr.backward(g)
    torch.testing.assert_close(xs.grad, xr.grad[:, :, rank * H:(rank + 1) * H], rtol=1e-4, atol=1e-4)
    # weight grads are partial sums over the H shards
    wg = sp.conv2.weight.grad.clone()
    torch.distributed.all_reduce(wg)
    torch.testing.assert_close(wg, ref.conv2.weight.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("world", [2, 3])
def test_spatial_bottleneck_halo(world):
    """H split over 2 or 3 ranks (the middle rank has both neighbours): output, input gradient and the
    all-reduced conv2 weight gradient equal the unsplit block's."""
    run_distributed(_spatial, world)


def _halo_exchangers(rank, world):
    import torch.distributed as dist
    from beforeholiday_amd.contrib.bottleneck.halo_exchangers import (HaloExchangerAllGather,
                                                                      HaloExchangerSendRecv)
    from beforeholiday_amd.contrib.nccl_p2p import left_right_halo_exchange
    from beforeholiday_amd.contrib.peer_memory import PeerHaloExchanger1d, PeerMemoryPool
    ranks = list(range(world))
    lo = torch.full((1, 1, 3, 2), float(10 * rank + 1))
    ro = torch.full((1, 1, 3, 2), float(10 * rank + 2))
    for ex in (HaloExchangerSendRecv(ranks, rank), HaloExchangerAllGather(ranks, rank, dist.group.WORLD)):
        li, ri = ex.left_right_halo_exchange(lo, ro)
        exp_li = 10 * (rank - 1) + 2 if rank > 0 else 0.0
        exp_ri = 10 * (rank + 1) + 1 if rank < world - 1 else 0.0
        assert torch.all(li == exp_li) and torch.all(ri == exp_ri)
    li, ri = left_right_halo_exchange(dist.group.WORLD, rank - 1 if rank > 0 else -1,
                                      rank + 1 if rank < world - 1 else -1, lo, ro)
    assert torch.all(li == (10 * (rank - 1) + 2 if rank > 0 else 0.0))
    pool = PeerMemoryPool(0, 0, ranks)
    ex = PeerHaloExchanger1d(ranks, rank, pool, 1)
    y = torch.zeros(1, 2, 6, 3)
    y[:, :, 1:5] = float(rank + 1)
    ex(y, H_split=True, explicit_nhwc=False)
    if rank > 0:
        assert torch.all(y[:, :, 0] == rank)
    if rank < world - 1:
        assert torch.all(y[:, :, 5] == rank + 2)


def test_halo_exchangers_and_peer_memory():
    run_distributed(_halo_exchangers, 3)


@pytest.mark.parametrize("device", devices())
def test_fmha_varlen(device):
    from beforeholiday_amd.contrib.fmha import FMHA
    torch.manual_seed(4)
    h, d = 2, 16
    lens = [5, 9, 3]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device=device)
    qkv = torch.randn(sum(lens), 3 * h * d, device=device, requires_grad=True)
    cfg = types.SimpleNamespace(attention_probs_dropout_prob=0.0, num_attention_heads=h, hidden_size=h * d)
    out = FMHA(cfg)(qkv, cu, max(lens), is_training=True)
    refs = []
    q3 = qkv.view(-1, 3, h, d)
    for i, n in enumerate(lens):
        s = slice(int(cu[i]), int(cu[i + 1]))
        q, k, v = (q3[s, j].transpose(0, 1) for j in range(3))
        p = torch.softmax(q @ k.transpose(-1, -2) / d ** 0.5, -1)
        refs.append((p @ v).transpose(0, 1).reshape(n, h * d))
    ref = torch.cat(refs)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)
    g1 = torch.autograd.grad(out.sum(), qkv, retain_graph=True)[0]
    g2 = torch.autograd.grad(ref.sum(), qkv)[0]
    torch.testing.assert_close(g1, g2, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fmha_varlen_fused_attention_path(dtype):
    """head 64, <= 128 tokens: FMHA runs the MFMA fused attention kernel; compare with fp32 math."""
    from beforeholiday_amd.contrib.fmha import FMHA
    torch.manual_seed(5)
    h, d = 4, 64
    lens = [37, 64, 100, 1]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device="cuda")
    qkv = torch.randn(sum(lens), 3 * h * d, device="cuda", dtype=dtype, requires_grad=True)
    cfg = types.SimpleNamespace(attention_probs_dropout_prob=0.0, num_attention_heads=h, hidden_size=h * d)
    out = FMHA(cfg)(qkv, cu, max(lens), is_training=True)
    qf = qkv.detach().float().requires_grad_(True)
    q3 = qf.view(-1, 3, h, d)
    refs = []
    for i, n in enumerate(lens):
        s = slice(int(cu[i]), int(cu[i + 1]))
        q, k, v = (q3[s, j].transpose(0, 1) for j in range(3))
        p = torch.softmax(q @ k.transpose(-1, -2) / d ** 0.5, -1)
        refs.append((p @ v).transpose(0, 1).reshape(n, h * d))
    ref = torch.cat(refs)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)
    g = torch.randn_like(out)
    g1 = torch.autograd.grad(out, qkv, g)[0]
    g2 = torch.autograd.grad(ref, qf, g.float())[0]
    torch.testing.assert_close(g1.float(), g2, rtol=tol, atol=tol * 2)


def _spatial_gpu(rank, world, c_in, planes, hw):
    """fp16 H-split block on the MFMA kernels (two gloo ranks sharing one GPU) vs the unsplit block."""
    from beforeholiday_amd.contrib.bottleneck import Bottleneck, SpatialBottleneck
    from beforeholiday_amd.contrib.bottleneck.halo_exchangers import HaloExchangerAllGather
    torch.cuda.set_device(0)
    torch.manual_seed(2)
    ref = Bottleneck(c_in, planes, c_in)
    _randomize_bn(ref)
    ex = HaloExchangerAllGather(list(range(world)), rank, torch.distributed.group.WORLD)
    sp = SpatialBottleneck(c_in, planes, c_in, spatial_parallel_args=(world, rank, None, ex))
    sp.load_state_dict(ref.state_dict())
    ref = ref.cuda().half().to(memory_format=torch.channels_last)
    sp = sp.cuda().half().to(memory_format=torch.channels_last)
    torch.manual_seed(3)
    # batch 4: the 1x1 strip kernel tiles 32-row pixel strips (4 x 14 x 28 rows per rank)
    x = torch.randn(4, c_in, hw, hw, device="cuda").half().contiguous(memory_format=torch.channels_last)
    H = hw // world
    sl = slice(rank * H, (rank + 1) * H)
    xs = x[:, :, sl].contiguous(memory_format=torch.channels_last).requires_grad_()
    calls = []
    conv2d = torch.nn.functional.conv2d
    torch.nn.functional.conv2d = lambda *a, **k: (calls.append(a[0].shape), conv2d(*a, **k))[1]
    try:
        y = sp(xs)
    finally:
        torch.nn.functional.conv2d = conv2d
    assert not calls, f"library convolutions on the spatial path: {calls}"
    xr = x.clone().requires_grad_()
    yr = ref(xr)

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm())

    assert rel(y, yr[:, :, sl]) < 2e-3, rel(y, yr[:, :, sl])
    g = torch.randn_like(yr)
    y.backward(g[:, :, sl].contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    assert rel(xs.grad, xr.grad[:, :, sl]) < 1e-2, rel(xs.grad, xr.grad[:, :, sl])
    for a, b in zip(sp.w_conv, ref.w_conv):
        wg = a.grad.float().clone()
        torch.distributed.all_reduce(wg)
        assert rel(wg, b.grad) < 1e-2, rel(wg, b.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 64, 56), (512, 128, 28)])
def test_spatial_bottleneck_gpu_matches_unsplit(shape):
    run_distributed(_spatial_gpu, 2, *shape)
