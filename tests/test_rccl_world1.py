"""RCCL code paths on a one-GPU box (world size 1, backend "nccl" = RCCL): the collectives the multi-GPU
bench runs -- SUM / AVG all-reduce, async work handles, DDP's bucketed all-reduce with the collectives forced
at world 1, and an all-reduce captured in a HIP graph and replayed -- checked against the local values.
(The 8-GPU scaling run is the driver's; this makes sure every RCCL call site has executed at least once.)
Plus the HIP-IPC PeerAllReduce with its device-resident epoch inside a captured graph (two processes on
one GPU, gloo for the setup)."""
import os
import socket
import traceback

import pytest
import torch

from tests._dist import run_distributed


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_worker(port, err_q):
    try:
        import torch.distributed as dist
        import torch.nn.functional as F

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
        # plain collectives: SUM, AVG (the DDP / ZeRO reduce op), async handles
        t = torch.arange(1000, device="cuda", dtype=torch.float32)
        ref = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        assert torch.equal(t, ref)
        w = dist.all_reduce(t, op=dist.ReduceOp.AVG, async_op=True)
        w.wait()
        assert torch.equal(t, ref)
        out = torch.empty(1000, device="cuda")
        dist.all_gather_into_tensor(out, ref)
        dist.reduce_scatter_tensor(t, out)
        assert torch.equal(t, ref)

        # DDP with the collectives forced at world 1: hooks, byte buckets, async AVG all-reduce, bucket views
        from beforeholiday_amd.parallel import DistributedDataParallel

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).cuda()
        ref_net = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).cuda()
        ref_net.load_state_dict(net.state_dict())
        ddp = DistributedDataParallel(net, bucket_cap_mb=0.002, force_collectives=True, gradient_as_bucket_view=True)
        assert ddp._collectives and ddp._use_avg
        x = torch.randn(32, 64, device="cuda")
        y = torch.randint(0, 10, (32,), device="cuda")
        for _ in range(2):  # the first backward builds the buckets, the second runs them
            for p in list(ddp.parameters()) + list(ref_net.parameters()):
                p.grad = None
            F.cross_entropy(ddp(x), y).backward()
            F.cross_entropy(ref_net(x), y).backward()
            for p, q in zip(ddp.module.parameters(), ref_net.parameters()):
                torch.testing.assert_close(p.grad, q.grad)
        assert len(ddp.bucket_sizes()) > 1

        # an RCCL all-reduce captured in a HIP graph, replayed with new inputs
        static = torch.zeros(4096, device="cuda")
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_reduce(static)  # warm-up outside capture (communicator setup)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            dist.all_reduce(static, op=dist.ReduceOp.SUM)
            static.mul_(2)
        for k in range(3):
            static.fill_(float(k + 1))
            g.replay()
            torch.cuda.synchronize()
            assert torch.all(static == 2.0 * (k + 1)), k
        dist.destroy_process_group()
    except Exception:
        err_q.put(traceback.format_exc())
        raise


@pytest.mark.gpu
def test_rccl_paths_world1():
    import torch.multiprocessing as mp

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    p.join(timeout=240)
    if p.is_alive():
        p.kill()
        raise AssertionError("RCCL world-1 worker timed out")
    if not q.empty():
        raise AssertionError(q.get())
    assert p.exitcode == 0


def _peer_graph(rank, world):
    from beforeholiday_amd.contrib.peer_memory import build_peer_allreduce

    torch.cuda.set_device(0)
    red = build_peer_allreduce(capacity=1024)
    assert red is not None, "IPC peer memory unavailable"
    static = torch.zeros(1000, device="cuda")
    # warm-up exchange outside the capture, then the captured one replayed with fresh inputs: the device
    # epoch advances on every replay, so no replay can pass on a previous replay's flags
    static.fill_(1.0)
    red.all_reduce_(static)
    torch.cuda.synchronize()
    assert torch.all(static == world)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        red.all_reduce_(static)
    for k in range(4):
        static.fill_(float((rank + 1) * (k + 1)))
        g.replay()
        torch.cuda.synchronize()
        want = float((k + 1) * world * (world + 1) // 2)
        assert torch.all(static == want), (k, static[:4].tolist(), want)
    red.check()
    assert int(red.epoch_dev.item()) == 2 + 4  # probe + warm-up + four replays (the capture itself does not run)


@pytest.mark.gpu
def test_peer_allreduce_captured_in_graph():
    run_distributed(_peer_graph, 2)
