"""Peer-memory pool and 1-D halo exchanger (reference: apex/contrib/peer_memory/{peer_memory,
peer_halo_exchanger_1d}.py, apex/contrib/csrc/peer_memory/peer_memory{.cpp,_cuda.cu}).

MI355X path (GPU tensors, native extension present): :class:`PeerMemoryPool` allocates one raw
device block per rank, exports it as a HIP IPC handle (dmabuf-backed on this driver), all-gathers
the handles over the process group and opens every peer's block, so ``allocate_peer_tensors``
returns the SAME pool offset viewed in every peer's memory (direct loads / stores over xGMI).
:class:`PeerHaloExchanger1d` runs ``peer_memory_cuda.push_pull_halos_1d``: stage the outgoing
halos in this rank's transfer slots, publish an epoch flag into each neighbour's memory, wait
(bounded) for the neighbours' flags and pull their slots straight into the input halos -- one kernel,
no collective, no host synchronisation (see kernels/peer_memory.hip for the protocol).

Fallback (CPU tensors / no extension, e.g. gloo tests): the pool hands out ordinary tensors and the
exchanger moves halos with point-to-point send/recv between neighbours.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ... import _native
from ..nccl_p2p.nccl_p2p import _exchange

_ALIGN = 256
_VIEW = {torch.float16: "blob_view_half", torch.bfloat16: "blob_view_bfloat16", torch.float32: "blob_view_float",
         torch.int32: "blob_view_int"}


def _pm():
    return _native.submodule("peer_memory_cuda")


class PeerMemoryPool(object):
    """``static_size`` + ``dynamic_size`` bytes per rank, shared with ``peer_ranks`` (default: the
    ranks of this node). ``allocate_peer_tensors`` returns one view per peer rank, all at the same offset."""

    def __init__(self, static_size, dynamic_size, peer_ranks=None, group=None, consensus=False):
        """``consensus=True``: a rank whose allocation / export / peer mapping fails does not raise
        alone (which would leave its peers waiting in the handle exchange): every rank of ``group``
        learns the outcome and all of them raise :class:`PeerSetupError` together."""
        rank = dist.get_rank()
        world = dist.get_world_size()
        if peer_ranks is None:
            from ...parallel.launch import visible_gpu_count

            ngpus = max(1, min(visible_gpu_count() or torch.cuda.device_count(), world))
            base = (rank // ngpus) * ngpus
            peer_ranks = list(range(base, base + ngpus))
        assert rank in peer_ranks, f"rank {rank} is not among peer_ranks {peer_ranks}"
        self.peer_ranks = list(peer_ranks)
        self.peer_rank = self.peer_ranks.index(rank)
        self.alignment = _ALIGN
        self.static_size = (static_size + _ALIGN - 1) // _ALIGN * _ALIGN
        self.dynamic_size = (dynamic_size + _ALIGN - 1) // _ALIGN * _ALIGN
        self.static_offset = 0
        self.dynamic_offset = 0
        self.native = torch.cuda.is_available() and _native.available()
        self.raw = None
        self.peer_raw = None
        if self.native:
            pm = _pm()
            handle, failure = b"", ""
            try:
                # (an empty pool still exports one block: its peers' mapping handshake is collective)
                self.raw = pm.allocate_raw(max(_ALIGN, self.static_size + self.dynamic_size))
                handle = pm.get_raw_ipc_address(self.raw).numpy().tobytes()
            except Exception as e:  # noqa: BLE001 - reported to every rank below
                if not consensus:
                    raise
                failure = repr(e)
            handles = [None] * world
            dist.all_gather_object(handles, handle, group=group)
            bad = [r for r in self.peer_ranks if not handles[r]]
            if bad:  # every rank sees the same gathered list: all of them raise here
                self._release()
                raise PeerSetupError(f"PeerMemoryPool: ranks {bad} could not export an IPC block"
                                     + (f" ({failure})" if rank in bad else ""))
            table = torch.from_numpy(np.frombuffer(b"".join(handles[r] for r in self.peer_ranks), dtype=np.uint8)
                                     .reshape(len(self.peer_ranks), -1).copy())
            ok = True
            try:
                self.peer_raw = pm.get_raw_peers(table, self.peer_rank, self.raw)
            except Exception:
                if not consensus:
                    raise
                ok = False
            if consensus and not agree(ok, group):
                self._release()
                raise PeerSetupError("PeerMemoryPool: a rank could not map its peers' IPC blocks")
        else:
            self._host = []

    def _release(self):
        pm = _pm()
        if self.peer_raw is not None:
            pm.close_raw_peers([p for i, p in enumerate(self.peer_raw) if i != self.peer_rank])
            self.peer_raw = None
        if self.raw is not None:
            pm.free_raw(self.raw)
            self.raw = None

    def __del__(self):
        try:
            if self.native:
                self._release()
        except Exception:
            pass

    def reset(self):
        self.dynamic_offset = 0

    def _take(self, nbytes, dynamic):
        if dynamic:
            start = (self.dynamic_offset + _ALIGN - 1) // _ALIGN * _ALIGN
            self.dynamic_offset = start + nbytes
            assert self.dynamic_offset <= self.dynamic_size, "Dynamic peer memory pool exhausted"
            return self.static_size + start
        start = (self.static_offset + _ALIGN - 1) // _ALIGN * _ALIGN
        self.static_offset = start + nbytes
        assert self.static_offset <= self.static_size, "Static peer memory pool exhausted"
        return start

    def allocate_peer_tensors(self, shape, dtype, channels_last, dynamic):
        if dtype not in _VIEW:
            raise AssertionError("dtype %s not supported" % (str(dtype),))
        nbytes = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        off = self._take(nbytes, dynamic)
        if self.native:
            view = getattr(_pm(), _VIEW[dtype])
            return [view(p + off, list(shape), bool(channels_last)) for p in self.peer_raw]
        fmt = torch.channels_last if channels_last and len(shape) == 4 else torch.contiguous_format
        ts = [torch.zeros(shape, dtype=dtype).contiguous(memory_format=fmt) for _ in self.peer_ranks]
        self._host.append(ts)
        return ts


class PeerTimeoutError(RuntimeError):
    """A peer did not publish its data within the bounded wait of an IPC exchange kernel."""


class PeerSetupError(RuntimeError):
    """IPC peer memory could not be set up on every rank of a group (raised on all of them)."""


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` is True on every rank of ``group`` (a MIN all-reduce)."""
    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class _ErrorWatch:
    """Host view of a kernel's sticky device ``err`` word without a synchronisation per call: after
    every launch the word is copied (async) into pinned memory, and the next call checks the copy a
    previous, completed call left there -- a timeout raises at most one call late. ``check(sync=True)``
    (a step boundary) waits for the stream first. The kernels also write NaN where data is missing,
    so even the late call's output is visibly invalid, never silently rank-local."""

    def __init__(self, err, what):
        self.err = err
        self.what = what
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=torch.cuda.is_available())

    def after_launch(self):
        self.host.copy_(self.err, non_blocking=True)

    def check(self, sync=False):
        if sync:
            torch.cuda.current_stream(self.err.device).synchronize()
            self.host.copy_(self.err)
        if int(self.host[0]) != 0:
            raise PeerTimeoutError(f"{self.what}: a peer did not publish its data in time (outputs were NaN-poisoned)")


class PeerHaloExchanger1d:
    """In-place halo exchange along H (or W) of a padded activation ``y`` ([N, C, H+2h, W], channels_last
    or not, or explicit NHWC [N, H+2h, W, C]); the first / last rank of the group get zero halos."""

    def __init__(self, ranks, rank_in_group, peer_pool, half_halo, max_spins=1 << 22):
        self.peer_group_size = len(ranks)
        self.ranks = ranks
        self.peer_rank = rank_in_group
        self.low_neighbor = (rank_in_group + self.peer_group_size - 1) % self.peer_group_size
        self.high_neighbor = (rank_in_group + 1) % self.peer_group_size
        self.low_zero = rank_in_group == 0
        self.high_zero = rank_in_group == self.peer_group_size - 1
        self.peer_pool = peer_pool
        self.half_halo = half_halo
        self.max_spins = max_spins
        self.epoch = 0
        self._tx = {}
        self.native = getattr(peer_pool, "native", False)
        if self.native:
            self.signals = peer_pool.allocate_peer_tensors([2, 64], torch.int32, False, False)
            self.err = torch.zeros(1, dtype=torch.int32, device="cuda")
            self._watch = _ErrorWatch(self.err, "PeerHaloExchanger1d")

    def _slots(self, numel, dtype):
        key = (numel, dtype)
        if key not in self._tx:  # same allocation order on every rank -> same pool offsets
            lo = self.peer_pool.allocate_peer_tensors([2, numel], dtype, False, False)
            hi = self.peer_pool.allocate_peer_tensors([2, numel], dtype, False, False)
            self._tx[key] = (lo, hi)
        return self._tx[key]

    def _views(self, y, H_split, explicit_nhwc):
        h = self.half_halo
        dim = (1 if H_split else 2) if explicit_nhwc else (2 if H_split else 3)
        n = y.size(dim)
        return (y.narrow(dim, h, h), y.narrow(dim, n - 2 * h, h), y.narrow(dim, 0, h), y.narrow(dim, n - h, h))

    def __call__(self, y, H_split=True, explicit_nhwc=False, numSM=0, diagnostics=False):
        out_lo, out_hi, in_lo, in_hi = self._views(y, H_split, explicit_nhwc)
        if not (self.native and y.is_cuda):
            left = self.ranks[self.low_neighbor] if not self.low_zero else -1
            right = self.ranks[self.high_neighbor] if not self.high_zero else -1
            li = torch.empty_like(in_lo, memory_format=torch.contiguous_format)
            ri = torch.empty_like(in_hi, memory_format=torch.contiguous_format)
            _exchange(dist.group.WORLD, left, right, out_lo, out_hi, li, ri)
            in_lo.copy_(li)
            in_hi.copy_(ri)
            return
        self.exchange_views(out_lo, out_hi, in_lo, in_hi, diagnostics)

    def exchange_views(self, out_lo, out_hi, in_lo, in_hi, diagnostics=False):
        """Native exchange of explicit 4-D halo views (outgoing low / high, incoming low / high)."""
        self.epoch += 1
        lo_tx, hi_tx = self._slots(out_lo.numel(), out_lo.dtype)
        me, lo_n, hi_n = self.peer_rank, self.low_neighbor, self.high_neighbor
        _pm().push_pull_halos_1d(out_lo, out_hi, in_lo, in_hi, lo_tx[me], hi_tx[me], hi_tx[lo_n], lo_tx[hi_n],
                                 self.signals[me], self.signals[lo_n], self.signals[hi_n], self.low_zero,
                                 self.high_zero, self.epoch, self.err, self.max_spins)
        self._watch.after_launch()
        self._watch.check(sync=diagnostics)

    def check(self):
        """Raise :class:`PeerTimeoutError` if any exchange so far timed out (synchronises)."""
        if getattr(self, "_watch", None) is not None:
            self._watch.check(sync=True)


class PeerAllReduce:
    """SUM all-reduce of small fp32 vectors among the ranks of a :class:`PeerMemoryPool` through
    IPC-mapped peer memory: one single-workgroup kernel pushes the payload into every peer's slot row,
    publishes an epoch flag and sums the rows in rank order once every peer's flag arrived (bounded
    wait; ``err`` is set on a timeout) -- no collective launch, no host synchronisation. This is the
    statistics exchange of group batch norm (reference: apex/contrib/csrc/groupbn/ipc.cu:22-129 and
    the peer-buffer exchange of nhwc_batch_norm_kernel.h). Every rank must issue the same sequence of
    calls with the same payload sizes, like any collective. Without a native pool (CPU / gloo) it
    falls back to ``dist.all_reduce``.

    The exchange epoch lives in device memory (``epoch_dev``): each kernel takes the previous value + 1
    and stores it back, so the exchange can be captured in a HIP graph and every replay publishes and
    waits for a fresh epoch on every rank (a host counter would be frozen into the captured kernel)."""

    def __init__(self, peer_pool, capacity=1 << 14, group=None, max_spins=1 << 22):
        self.pool = peer_pool
        self.group = group
        self.G = len(peer_pool.peer_ranks)
        self.me = peer_pool.peer_rank
        self.capacity = int(capacity)
        self.max_spins = max_spins
        self.epoch = 0
        self.native = getattr(peer_pool, "native", False)
        if self.native:
            assert self.G <= 8, "PeerAllReduce: at most 8 ranks per pool"
            self.slots = peer_pool.allocate_peer_tensors([2, self.G, self.capacity], torch.float32, False, False)
            self.flags = peer_pool.allocate_peer_tensors([self.G], torch.int32, False, False)
            self._slot_ptrs = [t.data_ptr() for t in self.slots]
            self._flag_ptrs = [t.data_ptr() for t in self.flags]
            self.err = torch.zeros(1, dtype=torch.int32, device="cuda")
            self.epoch_dev = torch.zeros(1, dtype=torch.int32, device="cuda")
            self._watch = _ErrorWatch(self.err, "PeerAllReduce")

    @property
    def size(self):
        return self.G

    def all_reduce_(self, t):
        """In-place SUM over the pool's ranks of a contiguous fp32 GPU tensor (numel <= capacity)."""
        if not (self.native and t.is_cuda):
            dist.all_reduce(t, group=self.group)
            return t
        assert t.dtype == torch.float32 and t.is_contiguous(), "PeerAllReduce: contiguous fp32 tensors only"
        self.epoch += 1  # (host count of calls; the kernel's epoch is the device counter)
        self._watch.check()  # an earlier exchange timed out: raise before adding to the damage
        _pm().peer_allreduce(t, t, self._slot_ptrs, self._flag_ptrs, self.capacity, self.me, 1, self.err,
                             self.max_spins, self.epoch_dev)
        self._watch.after_launch()
        return t

    def all_reduce_async(self, t):
        """:meth:`all_reduce_` issued on this reducer's own HIP stream (after the work already queued on
        the current stream): the current stream continues with independent kernels -- e.g. a weight
        gradient -- while the exchange's flag wait runs. Returns a handle whose ``wait()`` makes the
        current stream wait for the result. Every exchange goes through the one side stream, so the
        calls stay in the same order on every rank."""
        if not (self.native and t.is_cuda):
            return _DoneHandle(self.all_reduce_(t))
        side = getattr(self, "_side", None)
        if side is None:
            side = self._side = torch.cuda.Stream(device=t.device)
        side.wait_stream(torch.cuda.current_stream(t.device))
        with torch.cuda.stream(side):
            self.all_reduce_(t)
        t.record_stream(side)
        return _StreamHandle(side, t)

    def check(self):
        """Raise :class:`PeerTimeoutError` if any exchange so far timed out (synchronises; call it at
        a step boundary, e.g. next to the loss read)."""
        if self.native:
            self._watch.check(sync=True)


class _DoneHandle:
    def __init__(self, t):
        self.t = t

    def wait(self):
        return self.t


class _StreamHandle:
    def __init__(self, side, t):
        self.side, self.t = side, t

    def wait(self):
        torch.cuda.current_stream(self.t.device).wait_stream(self.side)
        return self.t


def build_peer_allreduce(capacity=1 << 13, max_spins=1 << 26, group=None):
    """A :class:`PeerAllReduce` over all ranks of ``group`` (default WORLD) when every rank can map
    every peer's IPC block AND a probe exchange returns the exact sum on every rank; otherwise
    ``None`` -- on every rank alike, so a caller can fall back to an RCCL communicator without the ranks
    diverging. Meant for single-node groups (HIP IPC does not cross nodes). ``max_spins`` bounds the
    wait for a peer's flag (2^26 spins is minutes: a rank that is merely slow, e.g. still compiling its
    first step, is waited for; a dead one NaN-poisons the output and raises)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if not (torch.cuda.is_available() and _native.available()) or world > 8:
        agree(False, group)
        return None
    ranks = list(range(world)) if group is None else dist.get_process_group_ranks(group)
    size = 2 * world * capacity * 4 + 4096
    try:
        pool = PeerMemoryPool(size, 0, peer_ranks=ranks, group=group, consensus=True)
    except PeerSetupError:
        return None
    ok = True
    red = None
    try:
        red = PeerAllReduce(pool, capacity=capacity, group=group, max_spins=max_spins)
        t = torch.full((capacity,), float(rank + 1), dtype=torch.float32, device="cuda")
        red.all_reduce_(t)
        red.check()
        ok = bool(torch.all(t == float(world * (world + 1) // 2)).item())
        red.epoch_after_probe = red.epoch
    except Exception:  # noqa: BLE001 - every rank learns of it through agree()
        ok = False
    if not agree(ok, group):
        return None
    return red
