"""Spawn one training process per GPU (reference: apex/parallel/multiproc.py:1-35).

``python -m beforeholiday_amd.parallel.multiproc train.py <args>`` starts ``world_size`` (number of
visible GPUs counted without a HIP call, or ``--world-size``) children of ``train.py`` with ``--rank i --world-size N`` appended
and the torch.distributed env vars set (127.0.0.1 rendezvous), and exits with the first failing
child's code. Children are separate processes, never an exec of this one.
"""
from __future__ import annotations

import os
import subprocess
import sys

from .launch import rank_env, visible_gpu_count


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    world_size = None
    if "--world-size" in argv:
        i = argv.index("--world-size")
        world_size = int(argv[i + 1])
        del argv[i:i + 2]
    if world_size is None:
        # counted from the KFD topology: the launcher never initialises HIP before its children
        world_size = max(1, visible_gpu_count())
    port = os.environ.get("MASTER_PORT", "29511")
    procs = []
    for rank in range(world_size):
        env = rank_env(rank, world_size, int(port))
        stdout = None if rank == 0 else open(f"GPU_{rank}.log", "w")
        procs.append(subprocess.Popen([sys.executable] + argv + ["--rank", str(rank), "--world-size", str(world_size)],
                                      env=env, stdout=stdout))
    rc = 0
    for p in procs:
        r = p.wait()
        if r != 0 and rc == 0:
            rc = r
    return rc


if __name__ == "__main__":
    sys.exit(main())
