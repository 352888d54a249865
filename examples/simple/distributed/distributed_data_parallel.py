"""Minimal amp + DistributedDataParallel example (reference:
examples/simple/distributed/distributed_data_parallel.py). One process per GPU:

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 distributed_data_parallel.py

``--backend gloo --device cpu`` runs the same script on CPU ranks.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")))
from beforeholiday_amd import amp  # noqa: E402
from beforeholiday_amd.parallel import DistributedDataParallel  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--opt-level", default="O1")
    ap.add_argument("--steps", type=int, default=500)
    a = ap.parse_args(argv)
    torch.distributed.init_process_group(a.backend)
    rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
    if a.device == "cuda":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    torch.manual_seed(0)
    N, D_in, D_out = 64, 1024, 16
    x = torch.randn(N, D_in, device=device)  # each rank: its own slice of a global batch
    y = torch.randn(N, D_out, device=device)
    model = torch.nn.Linear(D_in, D_out).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    model, opt = amp.initialize(model, opt, opt_level=a.opt_level, verbosity=0)
    model = DistributedDataParallel(model)
    loss_fn = torch.nn.MSELoss()
    for t in range(a.steps):
        opt.zero_grad()
        loss = loss_fn(model(x), y)
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
    if rank == 0:
        print(f"final loss {loss.detach().item():.6f} on {world} ranks", flush=True)
    torch.distributed.destroy_process_group()
    return float(loss.detach())


if __name__ == "__main__":
    main()
