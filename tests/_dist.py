"""Multi-process test helper: runs ``fn(rank, world, *args)`` in ``world`` spawned processes with a
gloo (CPU) process group over a FileStore, and re-raises the first failure."""
import os
import tempfile
import traceback

import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, init_file, fn, args, err_q):
    try:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
        fn(rank, world, *args)
        dist.barrier()
    except Exception:
        err_q.put((rank, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_distributed(fn, world=2, *args):
    ctx = mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    fd, init_file = tempfile.mkstemp(prefix="bh_pg_")
    os.close(fd)
    os.unlink(init_file)
    procs = [ctx.Process(target=_worker, args=(r, world, init_file, fn, args, err_q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    errs = []
    while not err_q.empty():
        errs.append(err_q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    if errs:
        raise AssertionError("distributed worker failed:\n" + "\n".join(f"[rank {r}] {tb}" for r, tb in errs))
    for p in procs:
        assert p.exitcode == 0, f"worker exit code {p.exitcode}"
