"""Run-to-run and rank-to-rank determinism of the fused ResNet step.

The reference's L1 harness compares whole training runs bitwise (``/root/reference/tests/L1/common/
compare.py:37-56``): that only works when every process runs the same kernels in the same reduction
order. Here: (1) one process repeats the same forward + backward and gets bit-identical loss and
gradients (no atomics / races in the conv, statistics or BatchNorm-backward kernels); (2) two
processes sharing one GPU compute the same single-rank step and agree bitwise, and their per-shape
kernel-choice tables are identical (``models/resnet.py`` ``_pick``)."""
import pytest
import torch


def _net(pg=None):
    from beforeholiday_amd.models import resnet as R
    from beforeholiday_amd.parallel import SyncBatchNorm

    def norm(c, fuse_relu=False, fuse_maxpool=None):
        return SyncBatchNorm(c, process_group=pg, channel_last=True, fuse_relu=fuse_relu, fuse_maxpool=fuse_maxpool)

    torch.manual_seed(0)
    net = R.resnet50_fused(process_group=pg, layers=(1, 1, 1, 1), num_classes=10)
    net = net.cuda().to(memory_format=torch.channels_last).half()
    for m in net.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.float()
    return net


def _step(net, x, y):
    for p in net.parameters():
        p.grad = None
    out = net(x)
    loss = torch.nn.functional.cross_entropy(out.float(), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), [p.grad.detach().clone() for p in net.parameters()]


def _inputs(n=16, hw=224):
    torch.manual_seed(11)
    x = torch.randn(n, 3, hw, hw, device="cuda").half().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (n,), device="cuda")
    return x, y


@pytest.mark.gpu
def test_fused_resnet_step_is_bitwise_repeatable():
    net = _net()
    state = {k: v.clone() for k, v in net.state_dict().items()}
    x, y = _inputs()
    l0, g0 = _step(net, x, y)
    net.load_state_dict(state)
    l1, g1 = _step(net, x, y)
    assert torch.equal(l0, l1), (float(l0), float(l1))
    names = [n for n, _ in net.named_parameters()]
    diff = [n for n, a, b in zip(names, g0, g1) if not torch.equal(a, b)]
    assert not diff, f"gradients differ between two identical steps: {diff}"


def _two_procs(rank, world):
    import torch.distributed as dist
    from beforeholiday_amd.models import resnet as R

    torch.cuda.set_device(0)
    single = [dist.new_group([r]) for r in range(world)][rank]
    net = _net(single)
    x, y = _inputs()
    loss, grads = _step(net, x, y)
    mine = torch.stack([loss.float().cpu()] + [g.float().double().sum().float().cpu() for g in grads])
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    picks = R.choice_table()
    allp = [None] * world
    dist.all_gather_object(allp, picks)
    assert all(p == allp[0] for p in allp), f"kernel choices differ across ranks: {allp}"
    bad = (allv[0] != allv[1]).nonzero().flatten().tolist()
    assert not bad, f"rank {rank}: rank 0 / rank 1 differ at {bad[:8]}: {allv[0][bad[:8]].tolist()} vs " \
                    f"{allv[1][bad[:8]].tolist()}"


@pytest.mark.gpu
def test_two_processes_same_step_bitwise_equal():
    from _dist import run_distributed

    run_distributed(_two_procs, 2)
