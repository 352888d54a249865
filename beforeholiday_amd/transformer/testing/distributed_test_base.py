"""Multi-process unittest bases (reference: apex/transformer/testing/distributed_test_base.py:30-133).

Each test method of a subclass runs in ``world_size`` spawned processes that join one process group
(FileStore rendezvous) with the class's ``DISTRIBUTED_BACKEND``:

* ``NcclDistributedTestBase`` — RCCL, one rank per GPU (up to 4),
* ``GlooDistributedTestBase`` — CPU ranks, so model-parallel logic is testable without GPUs,
* ``UccDistributedTestBase`` — requires torch_ucc (not shipped on ROCm; raises).

Self-contained (torch's internal MultiProcessTestCase needs packages this image does not ship).
Inside a rank, ``self.rank`` / ``self.world_size`` are set and the default group is initialised.
"""
import functools
import os
import tempfile
import traceback
import unittest

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HAS_TORCH_UCC = False
try:
    import torch_ucc  # noqa: F401
    HAS_TORCH_UCC = True
except ImportError:
    pass

_CHILD_ENV = "BH_DIST_TEST_CHILD"


def _child(cls, method, rank, world, init_file, err_q):
    os.environ[_CHILD_ENV] = "1"
    try:
        self = cls(method)
        self.rank = rank
        self.file_name = init_file
        dist.init_process_group(backend=cls.DISTRIBUTED_BACKEND, init_method=f"file://{init_file}", rank=rank,
                                world_size=world)
        if cls.DISTRIBUTED_BACKEND != "gloo":
            torch.cuda.set_device(rank % torch.cuda.device_count())
        self.setUp()
        try:
            getattr(self, method)()
        finally:
            self.tearDown()
        dist.barrier()
    except unittest.SkipTest as e:
        err_q.put((rank, "SKIP", str(e)))
    except Exception:
        err_q.put((rank, "FAIL", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


class DistributedTestBase(unittest.TestCase):
    DISTRIBUTED_BACKEND = None
    TIMEOUT = 300

    def __init__(self, methodName="runTest"):
        super().__init__(methodName)
        if os.environ.get(_CHILD_ENV) != "1" and methodName != "runTest":
            setattr(self, methodName, functools.partial(self._spawn_and_run, methodName))

    @property
    def world_size(self) -> int:
        return min(torch.cuda.device_count(), 4)

    def _setup_pre_spawn(self):
        pass

    def _spawn_and_run(self, method):
        self._setup_pre_spawn()
        world = int(self.world_size)
        if world < 1:
            raise unittest.SkipTest("no devices for this backend")
        ctx = mp.get_context("spawn")
        err_q = ctx.SimpleQueue()
        fd, init_file = tempfile.mkstemp(prefix="bh_dtb_")
        os.close(fd)
        os.unlink(init_file)
        procs = [ctx.Process(target=_child, args=(type(self), method, r, world, init_file, err_q))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=self.TIMEOUT)
        for p in procs:
            if p.is_alive():
                p.kill()
        msgs = []
        while not err_q.empty():
            msgs.append(err_q.get())
        if os.path.exists(init_file):
            os.unlink(init_file)
        fails = [m for m in msgs if m[1] == "FAIL"]
        if fails:
            raise AssertionError("\n".join(f"[rank {r}] {tb}" for r, _, tb in fails))
        skips = [m for m in msgs if m[1] == "SKIP"]
        if skips:
            raise unittest.SkipTest(skips[0][2])
        for p in procs:
            assert p.exitcode == 0, f"rank process exited with {p.exitcode}"


class NcclDistributedTestBase(DistributedTestBase):
    DISTRIBUTED_BACKEND = "nccl"


class GlooDistributedTestBase(DistributedTestBase):
    DISTRIBUTED_BACKEND = "gloo"

    @property
    def world_size(self) -> int:
        return int(os.environ.get("BH_TEST_WORLD_SIZE", "4"))


class UccDistributedTestBase(DistributedTestBase):
    DISTRIBUTED_BACKEND = "ucc"

    def _setup_pre_spawn(self) -> None:
        if not HAS_TORCH_UCC:
            raise unittest.SkipTest("UCC backend requires torch_ucc, which is not installed")
