"""Probe: can two RCCL ranks share one MI355X? (NCCL refuses "duplicate GPU"; this records what RCCL does.)

Spawns 2 children (no HIP in the parent), each runs init_process_group("nccl") on cuda:0, one fp32
all_reduce and one fp16 all_reduce with ReduceOp.AVG, and prints the result. Run under `timeout`.
"""
import os
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    t = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    h = torch.full((4096,), float(rank + 1), device="cuda", dtype=torch.float16)
    dist.all_reduce(h, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    print(f"rank {rank}: sum={t[0].item()} avg16={h[0].item()}", flush=True)
    dist.destroy_process_group()


def main():
    if os.environ.get("RANK") is not None:
        return child()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT="29533")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    sys.exit(max(p.wait() for p in procs))


if __name__ == "__main__":
    main()
