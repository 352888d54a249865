"""One-process-per-GPU launching without touching HIP in the parent.

The parent of a multi-rank job must not initialise the GPU before it starts its children (on this
platform a process that initialised HIP must never be replaced, and a parent holding a HIP context
per device also steals memory from every rank). So:

* :func:`visible_gpu_count` counts devices from the KFD topology in sysfs (``gpu_id != 0`` nodes),
  filtered by ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` exactly as
  the runtime would: no HIP call, no ``torch.cuda``.
* :func:`spawn_ranks` starts ``world`` children of a script with ``RANK`` / ``LOCAL_RANK`` /
  ``WORLD_SIZE`` / ``MASTER_ADDR`` (127.0.0.1) / ``MASTER_PORT`` set, waits for all of them, and
  returns the first non-zero exit code; when one child fails the others are terminated (a rank
  stuck in a collective whose peer died would otherwise hang until the RCCL timeout).

Reference behaviour: ``apex/parallel/multiproc.py:1-35`` (spawn ``world_size`` children with
``--rank``) and the metric definition ``world_size*batch/batch_time`` of
``examples/imagenet/main_amp.py:150,172,384-400`` which needs one process per GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

_KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _kfd_gpu_count() -> int:
    try:
        nodes = os.listdir(_KFD_NODES)
    except OSError:
        return 0
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(_KFD_NODES, node, "gpu_id")) as f:
                if int(f.read().strip() or "0") != 0:
                    n += 1
        except (OSError, ValueError):
            continue
    return n


def _env_filter(count: int) -> int:
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is None:
            continue
        ids = [v for v in val.split(",") if v.strip() != ""]
        if not ids:
            return 0
        count = min(count, len(ids)) if count else len(ids)
    return count


def visible_gpu_count() -> int:
    """Number of GPUs a child process would see, computed without any HIP call."""
    return _env_filter(_kfd_gpu_count())


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR=env.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: the only mode the host driver supports
    return env


def spawn_ranks(cmd: Sequence[str], world: int, port: Optional[int] = None, quiet_ranks: bool = False,
                poll_s: float = 0.2) -> int:
    """Run ``cmd`` as ``world`` ranks (children, never an exec). Returns 0 or the first failing code.

    ``quiet_ranks``: send stdout of ranks > 0 to /dev/null (rank 0 prints the result line)."""
    port = port or int(os.environ.get("MASTER_PORT", "0")) or free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        out = subprocess.DEVNULL if (quiet_ranks and r > 0) else None
        procs.append(subprocess.Popen(list(cmd), env=rank_env(r, world, port), stdout=out))
    rc = 0
    alive = set(range(world))
    try:
        while alive:
            for r in sorted(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"[launch] rank {r} exited with {code}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    for o in alive:
                        procs[o].send_signal(signal.SIGTERM)
            if alive:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        raise
    finally:
        deadline = time.time() + 30
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return rc


def maybe_spawn(world: int, argv: Optional[Sequence[str]] = None, script: Optional[str] = None) -> Optional[int]:
    """If this process is not already a rank (no ``WORLD_SIZE`` in the env) and ``world > 1``, run
    ``world`` copies of the current script as ranks and return the combined exit code; else None
    (the caller continues as a single rank / as the rank the launcher made it)."""
    if world <= 1 or "WORLD_SIZE" in os.environ:
        return None
    script = script or os.path.abspath(sys.argv[0])
    argv = list(sys.argv[1:] if argv is None else argv)
    return spawn_ranks([sys.executable, script] + argv, world, quiet_ranks=True)
