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
    assert pool.native == (device == "cuda")
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
