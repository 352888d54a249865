"""Peer-memory pool + 1-D halo exchanger (reference: apex/contrib/peer_memory, test:
apex/contrib/test/peer_memory/test_peer_halo_exchange_module.py).

CPU: the send/recv fallback on gloo ranks. GPU: two processes sharing one MI355X exchange halos
through HIP IPC mappings of each other's pool (dmabuf) and the push/pull kernel; checked against the
neighbours' known data for several epochs, both layouts, fp16 / fp32.
"""
import pytest
import torch
import torch.distributed as dist

from tests._dist import run_distributed


def _expected(y_list, r, h, dim):
    """Rank r's tensor after the exchange, computed from every rank's original tensor."""
    y = y_list[r].clone()
    n = y.size(dim)
    W = len(y_list)
    lo = y_list[r - 1].narrow(dim, n - 2 * h, h) if r > 0 else torch.zeros_like(y.narrow(dim, 0, h))
    hi = y_list[r + 1].narrow(dim, h, h) if r < W - 1 else torch.zeros_like(y.narrow(dim, 0, h))
    y.narrow(dim, 0, h).copy_(lo)
    y.narrow(dim, n - h, h).copy_(hi)
    return y


def _halo(rank, world, device, dtype):
    from beforeholiday_amd.contrib.peer_memory import PeerHaloExchanger1d, PeerMemoryPool
    if device == "cuda":
        torch.cuda.set_device(0)
    pool = PeerMemoryPool(1 << 20, 1 << 20, peer_ranks=list(range(world)))
    # the pool is native wherever a GPU and the extension are present (CPU tensors then take the
    # exchanger's send/recv fallback), ordinary tensors otherwise
    assert pool.native == (torch.cuda.is_available() and __import__("beforeholiday_amd")._native.available())
    h = 2
    ex = PeerHaloExchanger1d(list(range(world)), rank, pool, h)
    for epoch, (explicit_nhwc, channels_last) in enumerate([(False, True), (True, False), (False, False),
                                                            (False, True)]):
        ys = []
        for r in range(world):
            g = torch.Generator().manual_seed(100 * epoch + r)
            shape = (2, 12 + 2 * h, 7, 16) if explicit_nhwc else (2, 16, 12 + 2 * h, 7)
            y = torch.randn(shape, generator=g).to(dtype)
            if channels_last:
                y = y.contiguous(memory_format=torch.channels_last)
            ys.append(y)
        y = ys[rank].to(device)
        if channels_last:
            y = y.contiguous(memory_format=torch.channels_last)
        dist.barrier()
        ex(y, H_split=True, explicit_nhwc=explicit_nhwc, diagnostics=True)
        if device == "cuda":
            torch.cuda.synchronize()
        dim = 1 if explicit_nhwc else 2
        torch.testing.assert_close(y.cpu(), _expected(ys, rank, h, dim), rtol=0, atol=0)
    if device == "cuda":
        assert int(ex.err.item()) == 0
    dist.barrier()


@pytest.mark.parametrize("world", [2, 3])
def test_peer_halo_exchange_cpu(world):
    run_distributed(_halo, world, "cpu", torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_peer_halo_exchange_ipc_two_processes_one_gpu(dtype):
    run_distributed(_halo, 2, "cuda", dtype)


def _allreduce(rank, world, device):
    from beforeholiday_amd.contrib.peer_memory import PeerAllReduce, PeerMemoryPool
    if device == "cuda":
        torch.cuda.set_device(0)
    pool = PeerMemoryPool(1 << 20, 0, peer_ranks=list(range(world)))
    red = PeerAllReduce(pool, capacity=4096)
    for step, n in enumerate([1, 257, 4096, 33, 4096, 1000]):
        rows = [torch.randn(n, generator=torch.Generator().manual_seed(10 * step + r)) for r in range(world)]
        expect = torch.zeros(n)
        for r in range(world):  # rank order, fp32: the kernel's summation order
            expect = expect + rows[r]
        t = rows[rank].to(device)
        red.all_reduce_(t)
        torch.testing.assert_close(t.cpu(), expect, rtol=0, atol=0 if device == "cuda" else 1e-6)
    if device == "cuda":
        torch.cuda.synchronize()
        assert int(red.err.item()) == 0
    dist.barrier()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_peer_allreduce_ipc_processes_one_gpu(world):
    run_distributed(_allreduce, world, "cuda")


def test_peer_allreduce_cpu_fallback():
    run_distributed(_allreduce, 2, "cpu")


def _groupbn(rank, world, device, fuse_relu):
    from beforeholiday_amd.contrib import groupbn
    if device == "cuda":
        torch.cuda.set_device(0)
    N, H, W, C = 4, 5, 6, 24
    g = torch.Generator().manual_seed(0)
    xs = torch.randn(world * N, H, W, C, generator=g) * 2 + 0.5
    dys = torch.randn(world * N, H, W, C, generator=g)
    bn = groupbn.BatchNorm2d_NHWC(C, fuse_relu=fuse_relu, bn_group=world).to(device)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-0.2, 0.2, C))
    x = xs[rank * N:(rank + 1) * N].to(device).requires_grad_(True)
    for _ in range(3):  # several exchanges (epochs / slot parities)
        y = bn(x)
        y.backward(dys[rank * N:(rank + 1) * N].to(device))
    # fp32 full-batch reference
    xr = xs.permute(0, 3, 1, 2).clone().requires_grad_(True)
    w = torch.linspace(0.5, 1.5, C).requires_grad_(True)
    b = torch.linspace(-0.2, 0.2, C).requires_grad_(True)
    yr = torch.nn.functional.batch_norm(xr, None, None, w, b, True, 0.1, 1e-5)
    if fuse_relu:
        yr = torch.relu(yr)
    yr.backward(dys.permute(0, 3, 1, 2))
    torch.testing.assert_close(y.detach().cpu(), yr.detach().permute(0, 2, 3, 1)[rank * N:(rank + 1) * N],
                               rtol=1e-4, atol=1e-4)
    gx = x.grad.cpu() / 3  # three identical backward passes accumulated
    torch.testing.assert_close(gx, xr.grad.permute(0, 2, 3, 1)[rank * N:(rank + 1) * N], rtol=1e-4, atol=1e-4)
    if device == "cuda":
        assert groupbn.batch_norm._IPC[world].epoch == 6  # 3 forward + 3 backward exchanges went over IPC
        torch.cuda.synchronize()
    dist.barrier()


@pytest.mark.gpu
@pytest.mark.parametrize("fuse_relu", [False, True])
def test_groupbn_ipc_two_processes_one_gpu(fuse_relu):
    run_distributed(_groupbn, 2, "cuda", fuse_relu)


def test_groupbn_group_cpu():
    run_distributed(_groupbn, 2, "cpu", False)


def _allreduce_timeout(rank, world, device):
    """Rank 1 withholds its contribution: rank 0's bounded wait times out, its output is NaN (never
    its rank-local input) and check() raises; a following call raises before launching."""
    from beforeholiday_amd.contrib.peer_memory import PeerAllReduce, PeerMemoryPool
    from beforeholiday_amd.contrib.peer_memory.peer_memory import PeerTimeoutError
    torch.cuda.set_device(0)
    pool = PeerMemoryPool(1 << 20, 0, peer_ranks=list(range(world)))
    red = PeerAllReduce(pool, capacity=1024)
    t = torch.ones(100, device="cuda")
    red.all_reduce_(t)  # both ranks: a healthy exchange first
    torch.cuda.synchronize()
    assert float(t[0]) == world
    dist.barrier()
    red.max_spins = 1 << 12  # a short bounded wait for the withheld exchange
    if rank == 0:
        t = torch.ones(100, device="cuda")
        red.all_reduce_(t)
        torch.cuda.synchronize()
        assert torch.isnan(t.cpu()).all()
        with pytest.raises(PeerTimeoutError):
            red.check()
        with pytest.raises(PeerTimeoutError):
            red.all_reduce_(torch.ones(4, device="cuda"))
    dist.barrier()


@pytest.mark.gpu
def test_peer_allreduce_timeout_poisons_and_raises():
    run_distributed(_allreduce_timeout, 2, "cuda")


def _halo_timeout(rank, world, device):
    from beforeholiday_amd.contrib.peer_memory import PeerHaloExchanger1d, PeerMemoryPool
    from beforeholiday_amd.contrib.peer_memory.peer_memory import PeerTimeoutError
    torch.cuda.set_device(0)
    pool = PeerMemoryPool(1 << 20, 1 << 20, peer_ranks=list(range(world)))
    ex = PeerHaloExchanger1d(list(range(world)), rank, pool, 1, max_spins=1 << 12)
    dist.barrier()
    if rank == 0:  # rank 1 never publishes: rank 0's incoming high halo is NaN, and it raises
        y = torch.zeros(2, 8, 6, 16, device="cuda", dtype=torch.float16)
        with pytest.raises(PeerTimeoutError):
            ex(y, H_split=True, explicit_nhwc=True, diagnostics=True)
        assert torch.isnan(y[:, -1].float().cpu()).all() and not torch.isnan(y[:, :-1].float().cpu()).any()
    dist.barrier()


@pytest.mark.gpu
def test_peer_halo_timeout_poisons_and_raises():
    run_distributed(_halo_timeout, 2, "cuda")


def _build(rank, world, device, fail_rank):
    """build_peer_allreduce: IPC when every rank can set it up (GPU), None on EVERY rank otherwise --
    no native pool (CPU), or one rank failing its export (the others must not hang in the exchange)."""
    from beforeholiday_amd.contrib.peer_memory import build_peer_allreduce, peer_memory
    if device == "cuda":
        torch.cuda.set_device(0)
    if rank == fail_rank:
        def broken(*_a, **_k):
            raise RuntimeError("injected export failure")
        orig = peer_memory._pm

        class _Proxy:
            def __getattr__(self, name):
                return broken if name == "get_raw_ipc_address" else getattr(orig(), name)
        peer_memory._pm = lambda: _Proxy()
    red = build_peer_allreduce(capacity=1024)
    if device == "cpu" or fail_rank >= 0:
        assert red is None
    else:
        assert red is not None and red.G == world
        t = torch.full((300,), float(rank), device="cuda")
        red.all_reduce_(t)
        red.check()
        assert float(t[0]) == sum(range(world))
    dist.barrier()


def test_build_peer_allreduce_cpu_falls_back_on_every_rank():
    run_distributed(_build, 2, "cpu", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_build_peer_allreduce_ipc_consensus_one_gpu(fail_rank):
    run_distributed(_build, 2, "cuda", fail_rank)
