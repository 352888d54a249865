"""Bottleneck blocks with the BatchNorms folded into the convolutions (models/resnet.py
``_forward_folded``: statistics from the conv epilogues, backward sums from the data-gradient
epilogues) against a plain fp32 PyTorch Bottleneck (nn.Conv2d + nn.BatchNorm2d) with the same
weights: output, input gradient, every parameter gradient, running statistics. A single block is
well conditioned, so fp16 / bf16 rounding stays at the 1e-2 level (a whole fp16 network at batch 8 on
64x64 images amplifies rounding through 16 BatchNorm backwards to ~30% in either implementation)."""
import os

import pytest
import torch


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _block(inplanes, planes, stride, dt, pg=None):
    from beforeholiday_amd.models import resnet as R
    from beforeholiday_amd.parallel import SyncBatchNorm

    torch.manual_seed(0)
    ds_ref = ds = None
    if stride != 1 or inplanes != planes * 4:
        ds_ref = torch.nn.Sequential(torch.nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                                     torch.nn.BatchNorm2d(planes * 4))
    ref = R.Bottleneck(inplanes, planes, stride, ds_ref).cuda()

    def norm(c, fuse_relu=False):
        return SyncBatchNorm(c, process_group=pg, channel_last=True, fuse_relu=fuse_relu)

    if ds_ref is not None:
        ds = torch.nn.Sequential(torch.nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False), norm(planes * 4))
    blk = R.Bottleneck(inplanes, planes, stride, ds, norm_layer=norm, fused=True).cuda()
    blk.load_state_dict(ref.state_dict())
    blk = blk.to(memory_format=torch.channels_last).to(dt)
    for m in blk.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.float()
    return R, ref, blk


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cfg", [(256, 64, 1, 56), (64, 64, 1, 56), (256, 128, 2, 56), (512, 128, 1, 28),
                                 (1024, 256, 1, 14)])
def test_folded_bottleneck_matches_fp32(cfg, dt):
    import copy

    inplanes, planes, stride, hw = cfg
    R, ref, blk = _block(inplanes, planes, stride, dt)
    x = torch.randn(8, inplanes, hw, hw, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    assert blk._fold_ok(x)
    xr = x.float().clone().requires_grad_()
    xf = x.clone().requires_grad_()
    # the measured baseline: the same PyTorch block run in the 16-bit dtype (conv + BatchNorm in dt, as
    # cuDNN / MIOpen would), against fp32 -- the folded block may be at most 1.5x as far from fp32 (+ 2e-3)
    ref_lp = copy.deepcopy(ref).to(memory_format=torch.channels_last).to(dt)
    xl = x.clone().requires_grad_()
    out_r, out_f, out_l = ref(xr), blk(xf), ref_lp(xl)
    def gate(e, base):
        return e <= 1.5 * base + 2e-3
    assert gate(_rel(out_f, out_r), _rel(out_l, out_r)), (_rel(out_f, out_r), _rel(out_l, out_r))
    g = torch.randn_like(out_r)
    out_r.backward(g)
    out_f.backward(g.to(dt))
    out_l.backward(g.to(dt))
    assert gate(_rel(xf.grad, xr.grad), _rel(xl.grad, xr.grad)), (_rel(xf.grad, xr.grad), _rel(xl.grad, xr.grad))
    for (n, p), q, l in zip(blk.named_parameters(), ref.parameters(), ref_lp.parameters()):
        assert gate(_rel(p.grad, q.grad), _rel(l.grad, q.grad)), (n, _rel(p.grad, q.grad), _rel(l.grad, q.grad))
    for (n, b), q, l in zip(blk.named_buffers(), ref.buffers(), ref_lp.buffers()):
        if "running" in n:
            assert gate(_rel(b, q), _rel(l, q)), (n, _rel(b, q), _rel(l, q))
        elif "num_batches" in n:
            assert int(b) == int(q), n


@pytest.mark.gpu
def test_folded_and_unfolded_paths_agree():
    """Same fp16 block through the folded and the unfolded fused paths: identical math up to rounding."""
    R, _, blk = _block(256, 64, 1, torch.float16)
    x = torch.randn(8, 256, 56, 56, device="cuda").half().contiguous(memory_format=torch.channels_last)
    old = R._FOLD_BN
    try:
        outs = []
        for fold in (True, False):
            R._FOLD_BN = fold
            xx = x.clone().requires_grad_()
            o = blk(xx)
            o.float().square().sum().backward()
            outs.append((o.detach(), xx.grad, [p.grad.clone() for p in blk.parameters()]))
            for p in blk.parameters():
                p.grad = None
    finally:
        R._FOLD_BN = old
    assert _rel(outs[0][0], outs[1][0]) < 5e-3
    # the folded path's bottleneck tail computes bn3's backward algebraically (no fp16 rounding of conv3's
    # output gradient), so the two 16-bit paths round differently; tests/test_bn_fold.py checks that the
    # folded one is at least as close to fp32
    assert _rel(outs[0][1], outs[1][1]) < 3e-2
    for a, b in zip(outs[0][2], outs[1][2]):
        assert _rel(a, b) < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(256, 64, 1, 56, 32), (512, 128, 1, 28, 128)])
def test_bn_apply_folded_into_conv2_and_conv3(cfg):  # BH_FOLD_APPLY=all vs none
    """bn1 + ReLU inside conv2 (3x3 halo prologue) and, at >= 100k pixels with <= 128 channels, bn2 +
    ReLU inside conv3 (strip-GEMM prologue; weight gradients through the wgrad kernel's LDS prologue):
    the same block with BH_FOLD_APPLY off (separate normalisation passes) agrees to rounding, including
    running statistics and num_batches_tracked."""
    inplanes, planes, stride, hw, batch = cfg
    R, _, blk = _block(inplanes, planes, stride, torch.float16)
    x = torch.randn(batch, inplanes, hw, hw, device="cuda").half().contiguous(memory_format=torch.channels_last)
    y2 = torch.empty(batch, planes, hw, hw, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    assert blk._fold_bn2(y2)
    old = R._FOLD_APPLY
    state0 = {k: v.clone() for k, v in blk.state_dict().items()}
    try:
        outs = []
        for fold in ("all", "none"):
            R._FOLD_APPLY = fold
            blk.load_state_dict(state0)
            xx = x.clone().requires_grad_()
            o = blk(xx)
            # per-sample mean: .mean() puts the fp16 gradients in the subnormal range, .sum() overflows them
            (o.float().square().sum() / x.shape[0]).backward()
            outs.append((o.detach(), xx.grad, [p.grad.clone() for p in blk.parameters()],
                         {k: v.clone() for k, v in blk.state_dict().items()}))
            for p in blk.parameters():
                p.grad = None
    finally:
        R._FOLD_APPLY = old
    assert _rel(outs[0][0], outs[1][0]) < 5e-3
    # the folded path's bottleneck tail computes bn3's backward algebraically (no fp16 rounding of conv3's
    # output gradient), so the two 16-bit paths round differently; tests/test_bn_fold.py checks that the
    # folded one is at least as close to fp32
    assert _rel(outs[0][1], outs[1][1]) < 3e-2
    for a, b in zip(outs[0][2], outs[1][2]):
        assert _rel(a, b) < 3e-2
    for k in outs[0][3]:
        if "running" in k:
            assert _rel(outs[0][3][k], outs[1][3][k]) < 1e-3, k
        elif "num_batches" in k:
            assert int(outs[0][3][k]) == int(outs[1][3][k]) == int(state0[k]) + 1, k


def _fold_two_ranks(rank, world, cfg):
    import torch.distributed as dist

    torch.cuda.set_device(0)  # both ranks share the one GPU of the box (gloo process group)
    singles = [dist.new_group([r]) for r in range(world)]
    C, planes, stride, HW, B = cfg
    torch.manual_seed(7)
    x = torch.randn(world * B, C, HW, HW, device="cuda").half().contiguous(memory_format=torch.channels_last)

    def run(pg, xs):
        _, _, blk = _block(C, planes, stride, torch.float16, pg)
        assert blk._fold_ok(xs)
        xx = xs.clone().requires_grad_()
        o = blk(xx)
        (o.float().square().sum() / x.shape[0]).backward()  # per-sample mean: fp16 gradients stay normal
        return (o.detach(), xx.grad, [p.grad.clone() for p in blk.parameters()],
                {k: v.clone() for k, v in blk.state_dict().items()})

    sl = slice(rank * B, (rank + 1) * B)
    o, gx, gp, st = run(None, x[sl])  # statistics over both ranks' halves
    for g in gp:
        dist.all_reduce(g)
    o1, gx1, gp1, st1 = run(singles[rank], x)  # the whole batch on this rank alone
    assert _rel(o, o1[sl]) < 5e-3, (rank, _rel(o, o1[sl]))
    assert _rel(gx, gx1[sl]) < 2e-2, (rank, _rel(gx, gx1[sl]))
    for i, (a, b) in enumerate(zip(gp, gp1)):
        assert _rel(a, b) < 2e-2, (rank, i, _rel(a, b))
    for k in st:
        if "running" in k:
            assert _rel(st[k], st1[k]) < 1e-3, (rank, k, _rel(st[k], st1[k]))
        elif "num_batches" in k:
            assert int(st[k]) == int(st1[k]) == 1, (rank, k, int(st[k]), int(st1[k]))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(256, 64, 1, 56, 32), (256, 128, 2, 56, 16), (512, 128, 1, 28, 128)])
def test_folded_block_two_ranks_equals_one_rank_double_batch(cfg):
    """The folded path at world 2 (statistics partials summed per rank, all-reduced, merged; backward
    sums all-reduced the same way): two gloo ranks on one GPU with half the batch each equal one rank
    with the whole batch -- outputs, input gradients, all-reduced parameter gradients, running stats.
    Shapes: layer 1 with bn2 folded into conv3 (>= 100k pixels per rank), the stride-2 downsample
    block, layer 2 with bn2 folded."""
    from _dist import run_distributed

    run_distributed(_fold_two_ranks, 2, cfg)


def _net_two_ranks(rank, world, exchange):
    import torch.distributed as dist
    from beforeholiday_amd.models import resnet as R

    torch.cuda.set_device(0)
    singles = [dist.new_group([r]) for r in range(world)]
    B = 16
    torch.manual_seed(11)
    x = torch.randn(world * B, 3, 224, 224, device="cuda").half().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (world * B,), device="cuda")

    def run(pg, xs, ys):
        # bench.py's model (resnet50_fused: own kernels for every convolution, the stem included). A
        # bare ResNet(fused=True) keeps nn.Conv2d for the stem, and MIOpen's per-process algorithm
        # search then picked one of two stem kernels depending on which rank's search ran first (two
        # losses, 2.3563458919525146 / 2.3563921451568604, swapping between runs)
        torch.manual_seed(0)
        net = R.resnet50_fused(process_group=pg, layers=(1, 1, 1, 1), num_classes=10)
        net = net.cuda().to(memory_format=torch.channels_last).half()
        for m in net.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                m.float()
        out = net(xs)
        loss = torch.nn.functional.cross_entropy(out.float(), ys, reduction="sum") / x.shape[0]
        loss.backward()
        return (loss.detach(), {n: p.grad.clone() for n, p in net.named_parameters()},
                {k: v.clone() for k, v in net.state_dict().items() if "running" in k})

    sl = slice(rank * B, (rank + 1) * B)
    pg = None
    if exchange == "ipc":  # bench.py's default on one node: statistics through HIP-IPC peer buffers
        from beforeholiday_amd.contrib.peer_memory import build_peer_allreduce

        pg = build_peer_allreduce(capacity=1 << 13)
        assert pg is not None, "IPC peer all-reduce setup / probe failed"
    loss, g, st = run(pg, x[sl], y[sl])
    dist.all_reduce(loss)
    for t in g.values():
        dist.all_reduce(t)
    dump = os.environ.get("BH_TEST_OPDUMP")  # debugging: per-op checksums of this run, one file per rank
    if dump:
        import _oplog

        _oplog.install()
        _oplog.start()
    loss1, g1, st1 = run(singles[rank], x, y)
    if dump:
        os.makedirs(dump, exist_ok=True)
        _oplog.stop(os.path.join(dump, f"{exchange}_rank{rank}.txt"))
    # the noise floor: the same single-rank step with the two halves of the batch swapped (another
    # summation order). Gradients that downstream BatchNorms nearly cancel (the stem BN's bias) are
    # rounding noise at any order; a world-size factor (the bug class this guards) sits far above it
    perm = torch.cat([torch.arange(B, world * B), torch.arange(0, B)]).cuda()
    loss1p, g1p, _ = run(singles[rank], x[perm], y[perm])
    # the loss gets the same swapped-order noise floor as the gradients (fp16 activations through 16
    # BatchNorms: another statistics summation order moves the loss by ~1e-3 relative)
    lo, l1, l1p = float(loss), float(loss1), float(loss1p)
    assert abs(lo - l1) < 3 * abs(l1p - l1) + 2e-3 * abs(l1), (rank, lo, l1, l1p)
    for n in g:
        floor = _rel(g1p[n], g1[n])
        assert _rel(g[n], g1[n]) < 3 * floor + 2e-2, (rank, n, _rel(g[n], g1[n]), floor)
    for k in st:
        assert _rel(st[k], st1[k]) < 2e-3, (rank, k, _rel(st[k], st1[k]))
    # both ranks ran the single-rank double batch on identical data and weights: bitwise identical
    # losses unless the two processes chose different kernels (tests/test_determinism.py)
    both = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(both, torch.tensor([l1], dtype=torch.float64))
    assert both[0].item() == both[1].item(), (rank, [b.item() for b in both], R.choice_table())


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["group", "ipc"])
def test_fused_resnet_two_ranks_equals_one_rank_double_batch(exchange):
    """The fused ResNet (stem statistics epilogue + folded bottlenecks + fused max pool, [1, 1, 1, 1]
    blocks at 224x224) on two gloo ranks sharing one GPU vs one rank with the double batch; SyncBN
    statistics through the gloo group or through the HIP-IPC PeerAllReduce (bench.py's default)."""
    from _dist import run_distributed

    run_distributed(_net_two_ranks, 2, exchange)


@pytest.mark.gpu
def test_block_output_with_second_consumer():
    """a folded block's output feeds the next block AND a second consumer (a feature tap).
    Autograd then accumulates the tap's gradient into the next block's masked conv1 data gradient in
    place: same storage, new version. The tail must notice (mask link version check) and redo its mask
    + column sums, so the result matches fp32 PyTorch blocks with the same tap."""
    R, ref_a, blk_a = _block(256, 64, 1, torch.float16)
    torch.manual_seed(1)
    _, ref_b, blk_b = _block(256, 64, 1, torch.float16)
    x = torch.randn(8, 256, 56, 56, device="cuda").half().contiguous(memory_format=torch.channels_last)
    tap = torch.randn(8, 256, 56, 56, device="cuda")
    xr = x.float().clone().requires_grad_()
    xf = x.clone().requires_grad_()
    outs = []
    for a, b, xx in ((ref_a, ref_b, xr), (blk_a, blk_b, xf)):
        ya = a(xx)
        yb = b(ya)
        loss = yb.float().square().sum() / 64 + (ya.float() * tap).sum()
        loss.backward()
        outs.append(yb)
    assert _rel(outs[1], outs[0]) < 2e-2
    assert _rel(xf.grad, xr.grad) < 6e-2
    for blk, ref in ((blk_a, ref_a), (blk_b, ref_b)):
        for (n, p), q in zip(blk.named_parameters(), ref.parameters()):
            assert _rel(p.grad, q.grad) < 6e-2, n


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(256, 64, 1, 56), (1024, 256, 1, 14)])
def test_conv3x3_bwd_epilogue_matches_reduce_pass(cfg):
    """Config.conv3x3_bwd_epi: bn1's backward sums from the 3x3 data-gradient epilogue (as the
    accumulators leave) == the separate k_bwd_reduce pass over (dA, y) -- same block, same gradients
    up to fp32 summation order."""
    from beforeholiday_amd import config

    inplanes, planes, stride, hw = cfg
    R, _, blk = _block(inplanes, planes, stride, torch.float16)
    x = torch.randn(8, inplanes, hw, hw, device="cuda").half().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in blk.state_dict().items()}
    outs = []
    for on in (True, False):
        config.set(conv3x3_bwd_epi=on)
        blk.load_state_dict(state0)
        xx = x.clone().requires_grad_()
        o = blk(xx)
        (o.float().square().sum() / x.shape[0]).backward()
        outs.append((xx.grad.clone(), [p.grad.clone() for p in blk.parameters()]))
        for p in blk.parameters():
            p.grad = None
    assert _rel(outs[0][0], outs[1][0]) < 2e-3
    for a, b in zip(outs[0][1], outs[1][1]):
        assert _rel(a, b) < 2e-3
