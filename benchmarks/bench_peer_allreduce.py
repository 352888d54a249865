"""Latency of the SyncBN statistics exchange through HIP-IPC peer memory (contrib/peer_memory
PeerAllReduce: push this rank's [2C+1] payload into every peer's slot, epoch flag, bounded wait, sum
the rows in rank order -- one kernel, no collective launch) vs the same all-reduce over gloo.

Two processes share the one GPU of a gpurun box, so "peer" memory is local HBM: this measures the
kernel + flag protocol latency per call (what 106 calls per ResNet-50 step pay at N > 1), not xGMI
link time. JSON lines: C, payload floats, peer us/call (event-timed over ``--iters`` back-to-back
calls, max over ranks), gloo us/call (host-timed).

    python benchmarks/bench_peer_allreduce.py [--iters 200]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, init_file, iters, q):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from beforeholiday_amd.contrib.peer_memory import build_peer_allreduce

    red = build_peer_allreduce(capacity=1 << 13)
    rows = []
    for C in (64, 256, 1024, 2048):
        n = 2 * C + 1
        t = torch.full((n,), float(rank + 1), device="cuda")
        ok = True
        if red is not None:
            for _ in range(10):
                t.fill_(float(rank + 1))
                red.all_reduce_(t)
            torch.cuda.synchronize()
            ok = bool(torch.all(t == sum(r + 1 for r in range(world))).item())
            dist.barrier()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                red.all_reduce_(t)
            e.record()
            torch.cuda.synchronize()
            red.check()
            peer_us = s.elapsed_time(e) * 1e3 / iters
        else:
            peer_us = None
        dist.barrier()
        tc = t.cpu()
        t0 = time.perf_counter()
        for _ in range(max(10, iters // 10)):
            dist.all_reduce(tc)
        gloo_us = (time.perf_counter() - t0) * 1e6 / max(10, iters // 10)
        mx = torch.tensor([peer_us or 0.0, gloo_us], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        rows.append({"C": C, "floats": n, "world": world, "peer_us_per_call": None if peer_us is None else
                     round(float(mx[0]), 2), "gloo_us_per_call": round(float(mx[1]), 1), "sum_correct": ok})
    if rank == 0:
        q.put(rows)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    fd, init_file = tempfile.mkstemp(prefix="bh_pa_")
    os.close(fd)
    os.unlink(init_file)
    procs = [ctx.Process(target=_rank, args=(r, args.world, init_file, args.iters, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad or q.empty():
        sys.exit(f"bench_peer_allreduce: ranks failed ({bad})")
    for row in q.get():
        print(json.dumps(row))


if __name__ == "__main__":
    main()
