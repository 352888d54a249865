"""DistributedDataParallel and Reducer (reference: apex/parallel/distributed.py:89-640).

Behaviour kept from the reference:
* parameters (and buffers) are broadcast from rank 0 at construction, flattened per dtype;
* gradient buckets are built from the order gradients ARRIVE in the first backward pass (the
  order that gives the best overlap), ``message_size`` elements per bucket, one bucket chain per
  dtype; rank 0's bucket structure is broadcast so every rank issues identical collectives;
* buckets are all-reduced in order while the rest of backward is still running;
* ``delay_allreduce``, ``allreduce_trigger_params``, ``retain_allreduce_buffers``,
  ``allreduce_always_fp32``, ``gradient_predivide_factor``, ``num_allreduce_streams`` (one
  process group per stream, round-robin), ``allreduce_communicators``.

MI355X / RCCL design:
* collectives are issued with ``async_op=True`` on the RCCL backend: RCCL runs them on its own HIP
  stream, so bucket all-reduces overlap the remaining backward kernels without a hand-managed side
  stream; the end-of-backward callback makes the compute stream wait on each work handle.
* buckets can be cut by BYTES (``bucket_cap_mb``, plus a smaller ``first_bucket_mb``) instead of the
  reference's element count, sized per xGMI peer (:func:`xgmi_bucket_mb`).
* averaging uses ``ReduceOp.AVG`` inside the collective when the backend supports it (RCCL), so no
  extra scaling kernel runs per bucket.
* once the bucket structure is known each parameter gets a slot view of its bucket's persistent
  flat buffer (same strides as the parameter; the views live in the bucket, not on the Parameter).
  The per-parameter hook copies a gradient into its slot as it arrives -- overlapped with the rest of
  backward -- and the all-reduce runs on the flat buffer in place. By default the averaged slot is
  copied back into ``param.grad`` afterwards; with ``gradient_as_bucket_view=True`` (torch DDP's
  option of the same name; bench.py uses it) ``param.grad`` BECOMES the slot view and nothing is
  copied back. A gradient-as-bucket-view ``param.grad`` is overwritten by the next backward, so
  code that keeps a gradient across backwards (amp's accumulation stash) must copy it:
  :func:`grad_is_bucket_view` tells it when.
* device-agnostic: the same code runs on CPU tensors over gloo (the reference hard-codes CUDA).
* a single-process world skips every collective.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.distributed as dist
from torch.nn.modules import Module
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from . import comm_stats


def xgmi_bucket_mb(world_size: int, grad_bytes: int, min_per_peer_mb: float = 2.0, max_buckets: int = 8):
    """(bucket_cap_mb, first_bucket_mb) for a fully connected xGMI node.

    A ring all-reduce of B bytes over W ranks moves B/W-byte slices per step on one link, so each
    slice must be >= ~``min_per_peer_mb`` MB to stay bandwidth-bound (~153 GB/s per link) rather
    than latency-bound -> bucket >= W * min_per_peer_mb. At most ``max_buckets`` buckets keep the
    per-collective launch/latency overhead small; the first bucket is 1/4 size so communication
    starts early in backward.
    """
    total_mb = grad_bytes / 2 ** 20
    cap = max(world_size * min_per_peer_mb, total_mb / max_buckets)
    return cap, max(world_size * min_per_peer_mb / 4, cap / 4)


def _raw(t: torch.Tensor) -> torch.Tensor:
    """1-D view of a dense tensor in its storage order (contiguous or channels_last)."""
    if t.is_contiguous():
        return t.view(-1)
    for fmt in (torch.channels_last, torch.channels_last_3d):
        try:
            if t.is_contiguous(memory_format=fmt):
                return t.as_strided((t.numel(),), (1,))
        except RuntimeError:
            pass
    raise RuntimeError("DistributedDataParallel: gradients must be dense (contiguous or channels_last)")


def _fmt(t: torch.Tensor):
    for fmt in (torch.channels_last, torch.channels_last_3d):
        try:
            if t.dim() >= 4 and t.is_contiguous(memory_format=fmt):
                return fmt
        except RuntimeError:
            pass
    return torch.contiguous_format


def flatten(bucket):
    return _flatten_dense_tensors(bucket)


def unflatten(coalesced, bucket):
    return _unflatten_dense_tensors(coalesced, bucket)


def apply_flat_dist_call(bucket, call, extra_args=None):
    coalesced = flatten(bucket)
    if extra_args is not None:
        call(coalesced, *extra_args)
    else:
        call(coalesced)
    if call is dist.all_reduce:
        coalesced /= dist.get_world_size()
    for buf, synced in zip(bucket, unflatten(coalesced, bucket)):
        buf.copy_(synced)


def split_by_type(tensors):
    buckets = {}
    for t in tensors:
        buckets.setdefault(t.dtype, []).append(t)
    return list(buckets.values())


# reference name kept
split_half_float_double_bfloat16 = split_by_type


def flat_dist_call(tensors, call, extra_args=None):
    for bucket in split_by_type(tensors):
        apply_flat_dist_call(bucket, call, extra_args)


def extract_tensors(maybe_tensor, tensor_list):
    if torch.is_tensor(maybe_tensor):
        tensor_list.append(maybe_tensor)
    else:
        try:
            for item in maybe_tensor:
                extract_tensors(item, tensor_list)
        except TypeError:
            return


class Reducer(object):
    """Manual all-reduce (average) of a module's gradients, triggered by ``reduce()``.

    Constructed from a module the parameters are broadcast from rank 0; constructed from a
    gradient list the caller owns parameter synchronisation.
    """

    def __init__(self, module_or_grads_list, process_group=None):
        self.process_group = process_group
        if isinstance(module_or_grads_list, Module):
            self.module = module_or_grads_list
            flat_dist_call([p.data for p in self.module.parameters()], self._broadcast)
        else:
            self.module = None
            self.grads = []
            extract_tensors(module_or_grads_list, self.grads)

    def _broadcast(self, t):
        dist.broadcast(t, _group_rank0(self.process_group), group=self.process_group)

    def _allreduce(self, t):
        dist.all_reduce(t, group=self.process_group)

    def reduce(self):
        grads = ([p.grad.data for p in self.module.parameters() if p.grad is not None] if self.module
                 else self.grads)
        ws = dist.get_world_size(self.process_group)
        for bucket in split_by_type(grads):
            coalesced = flatten(bucket)
            self._allreduce(coalesced)
            coalesced /= ws
            for buf, synced in zip(bucket, unflatten(coalesced, bucket)):
                buf.copy_(synced)


def _group_rank0(pg):
    if pg is None:
        return 0
    try:
        return dist.get_global_rank(pg, 0)
    except Exception:
        return 0


def _supports_avg(pg) -> bool:
    try:
        return dist.get_backend(pg) == "nccl"
    except Exception:
        return False


# parameter -> the data pointer of its bucket slot, for the parameters of gradient-as-bucket-view DDP
# instances. The keys are weak and the values are plain ints, so nothing here keeps a parameter or its
# bucket buffer alive (a stored slot VIEW would pin the whole flat bucket as long as the parameter lives)
_VIEW_SLOTS = None


def _view_slots():
    global _VIEW_SLOTS
    if _VIEW_SLOTS is None:
        from torch.utils.weak import WeakTensorKeyDictionary

        _VIEW_SLOTS = WeakTensorKeyDictionary()
    return _VIEW_SLOTS


def grad_is_bucket_view(p: torch.Tensor) -> bool:
    """True when ``p.grad`` is the gradient-as-bucket-view slot of a DDP bucket: the next backward
    writes into that memory, so a caller that keeps the gradient aside must clone it."""
    g = p.grad
    if g is None or _VIEW_SLOTS is None:
        return False
    ptr = _VIEW_SLOTS.get(p)
    return ptr is not None and g.data_ptr() == ptr


def _slot_view(flat: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
    """View of ``flat[off:off+numel]`` with ``p``'s shape and (dense) strides."""
    n = p.numel()
    if p.is_contiguous():
        return flat[off:off + n].view(p.shape)
    return flat[off:off + n].as_strided(p.size(), p.stride())


class _Bucket:
    __slots__ = ("params", "numel", "dtype", "flat", "work", "launched", "ready", "outputs", "slots", "placed")

    def __init__(self, params, dtype):
        self.params = params  # list of param indices
        self.dtype = dtype
        self.numel = 0
        self.flat = None
        self.work = None
        self.launched = False
        self.ready = 0
        self.outputs = None
        self.slots = None  # per-parameter views of flat
        self.placed = set()  # params whose gradient the hooks already put into their slot this backward


class DistributedDataParallel(Module):
    """Data-parallel wrapper with overlapped, bucketed gradient all-reduce over RCCL / gloo.

    Args mirror the reference (apex/parallel/distributed.py:162-175); ``process_group`` selects the
    data-parallel group (default: WORLD).
    """

    def __init__(self, module, message_size=10000000, delay_allreduce=False, shared_param=None,
                 allreduce_trigger_params=None, retain_allreduce_buffers=False, allreduce_always_fp32=False,
                 num_allreduce_streams=1, allreduce_communicators=None, gradient_average=True,
                 gradient_predivide_factor=1.0, gradient_average_split_factor=None, prof=False,
                 process_group=None, bucket_cap_mb=None, first_bucket_mb=None, gradient_as_bucket_view=False,
                 force_collectives=False):
        super().__init__()
        if shared_param is not None:
            raise ValueError("shared_param is no longer supported as an option.  It was misleadingly named "
                             "from the start.  It turns out overlapping communication with computation should "
                             "work fine with shared parameters.  If you still wish to delay communication to "
                             "the end of the backward pass, use delay_allreduce=True|False instead.")
        if gradient_average_split_factor is not None:
            print("Warning:  gradient_average_split_factor has been renamed to gradient_predivide_factor.  "
                  "For now, gradient_average_split_factor will also work, but please update to "
                  "gradient_predivide_factor instead.")
            gradient_predivide_factor = gradient_average_split_factor
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        # a single-process world skips every collective unless force_collectives (an initialised process
        # group is required then): the bucket / hook / async all-reduce path runs as with several ranks --
        # how a one-GPU box exercises the RCCL code paths (tests/test_rccl_world1.py)
        self._collectives = self.world_size > 1 or (bool(force_collectives) and dist.is_initialized())
        self.message_size = int(message_size)
        # byte-based bucket policy (MI355X): ``bucket_cap_mb`` replaces the element-count
        # ``message_size`` cut; ``first_bucket_mb`` makes the first bucket of each dtype small so its
        # all-reduce starts while most of backward is still ahead. See :func:`xgmi_bucket_mb`.
        self.bucket_cap_bytes = int(float(bucket_cap_mb) * 2 ** 20) if bucket_cap_mb else None
        self.first_bucket_bytes = int(float(first_bucket_mb) * 2 ** 20) if first_bucket_mb else None
        self.delay_allreduce = delay_allreduce
        self.retain_allreduce_buffers = retain_allreduce_buffers
        self.allreduce_always_fp32 = allreduce_always_fp32
        self.gradient_average = gradient_average
        self.gradient_predivide_factor = gradient_predivide_factor
        self.prof = prof
        self.gradient_as_bucket_view = bool(gradient_as_bucket_view)
        self.allreduce_buffers = []
        self.num_allreduce_streams = num_allreduce_streams
        self.custom_allreduce_triggers = False
        self.allreduce_trigger_params = None
        if allreduce_trigger_params is not None:
            if delay_allreduce:
                raise ValueError("Setting allreduce_trigger_params is only valid if delay_allreduce=False.")
            self.custom_allreduce_triggers = True
            self.allreduce_trigger_params = set(id(p) for p in allreduce_trigger_params)
        if allreduce_communicators is not None:
            groups = allreduce_communicators[0] if isinstance(allreduce_communicators, tuple) else allreduce_communicators
            self._groups = list(groups)
            self.num_allreduce_streams = len(self._groups)
        else:
            self._groups = None  # created lazily (collective)
        self._use_avg = (gradient_average and gradient_predivide_factor == 1.0 and not allreduce_always_fp32
                         and _supports_avg(process_group))
        self._sync_enabled = True
        self._callback_queued = False
        self._hooks = []

        # sync parameters and buffers from rank 0
        if self._collectives:
            if self.world_size > 1:  # every rank runs the same kernels / fold modes (beforeholiday_amd.config)
                from .. import config

                config.check_ranks(process_group)
            root = _group_rank0(process_group)
            tensors = [p.data for p in module.parameters()] + [b.data for b in module.buffers()]
            for bucket in split_by_type(tensors):
                coalesced = flatten(bucket)
                dist.broadcast(coalesced, root, group=process_group)
                for buf, synced in zip(bucket, unflatten(coalesced, bucket)):
                    buf.copy_(synced)
        self._refresh_params()

    # ------------------------------------------------------------------ bookkeeping
    def __setstate__(self, state):
        super().__setstate__(state)
        self._hooks = []
        self._refresh_params()

    def __getstate__(self):
        attrs = dict(self.__dict__)
        for k in ("_hooks", "_buckets", "_groups", "_param_to_bucket", "_arrival"):
            attrs.pop(k, None)
        return attrs

    def _refresh_params(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if _VIEW_SLOTS is not None:
            for p in getattr(self, "active_params", []):
                _VIEW_SLOTS.pop(p, None)
        self.active_params = [p for p in self.module.parameters() if p.requires_grad]
        self._param_ids = [id(p) for p in self.active_params]
        self.needs_refresh = True
        self._buckets: List[_Bucket] = []
        self._param_to_bucket = {}
        self._arrival = []
        self._next_bucket = 0
        if self._collectives:
            for idx, p in enumerate(self.active_params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(idx)))

    def _pg_for(self, bucket_idx):
        if self.num_allreduce_streams <= 1:
            return self.process_group
        if self._groups is None:
            ranks = None
            if self.process_group is not None:
                ranks = dist.get_process_group_ranks(self.process_group)
            self._groups = [dist.new_group(ranks=ranks) for _ in range(self.num_allreduce_streams)]
        return self._groups[bucket_idx % len(self._groups)]

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no all-reduce) inside this context."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    # ------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        if self.prof:
            torch.cuda.nvtx.range_push("forward pass DDP logic")
        if self._collectives:
            if [id(p) for p in self.module.parameters() if p.requires_grad] != self._param_ids:
                self._refresh_params()
            self._callback_queued = False
            self._next_bucket = 0
            for b in self._buckets:
                b.work, b.launched, b.ready, b.outputs = None, False, 0, None
            if self.needs_refresh:
                self._arrival = []
            if self.retain_allreduce_buffers:
                self.allreduce_buffers = [None for _ in self._buckets]
        if self.prof:
            torch.cuda.nvtx.range_pop()
        return self.module(*inputs, **kwargs)

    # ------------------------------------------------------------------ backward hooks
    def _make_hook(self, idx):
        def hook(param):
            if not self._sync_enabled:
                return
            if self.prof:
                torch.cuda.nvtx.range_push("allreduce_hook")
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
                self._callback_queued = True
            if self.needs_refresh or self.delay_allreduce:
                if self.needs_refresh:
                    self._arrival.append(idx)
            else:
                b_idx = self._param_to_bucket.get(idx)
                if b_idx is not None:
                    b = self._buckets[b_idx]
                    self._to_slot(b, idx)
                    b.placed.add(idx)
                    b.ready += 1
                    if b.ready == len(b.params):
                        self._launch_ready_in_order()
            if self.prof:
                torch.cuda.nvtx.range_pop()
        return hook

    def _launch_ready_in_order(self):
        while self._next_bucket < len(self._buckets):
            b = self._buckets[self._next_bucket]
            if b.ready < len(b.params):
                break
            self._launch(self._next_bucket)
            self._next_bucket += 1

    def _cut_threshold(self, dtype, n_closed: int) -> int:
        """Bucket size (elements) for the next bucket of ``dtype`` after ``n_closed`` closed ones."""
        esize = torch.empty((), dtype=dtype).element_size()
        if n_closed == 0 and self.first_bucket_bytes:
            return max(1, self.first_bucket_bytes // esize)
        if self.bucket_cap_bytes:
            return max(1, self.bucket_cap_bytes // esize)
        return self.message_size

    def _build_buckets(self, order: List[int]):
        """Cut buckets from an arrival order (per dtype; message_size elements, bucket_cap_mb bytes,
        or trigger params)."""
        seen = set(order)
        order = list(order) + [i for i in range(len(self.active_params)) if i not in seen]
        open_b = {}
        closed = {}
        buckets = []
        for idx in order:
            p = self.active_params[idx]
            b = open_b.get(p.dtype)
            if b is None:
                b = _Bucket([], p.dtype)
                open_b[p.dtype] = b
                buckets.append(b)
            b.params.append(idx)
            b.numel += p.numel()
            cut = (id(p) in self.allreduce_trigger_params) if self.custom_allreduce_triggers else \
                (b.numel >= self._cut_threshold(p.dtype, closed.get(p.dtype, 0)))
            if cut:
                open_b.pop(p.dtype)
                closed[p.dtype] = closed.get(p.dtype, 0) + 1
        return buckets

    def bucket_sizes(self):
        """(dtype, elements) of each bucket, in all-reduce order (empty before the first backward)."""
        return [(b.dtype, b.numel) for b in self._buckets]

    def _sync_bucket_structure(self, buckets):
        """Broadcast rank 0's bucket structure: [nb, sizes(nb), param indices...] padded to 1+2P."""
        P = len(self.active_params)
        dev = self.active_params[0].device if P else torch.device("cpu")
        if dist.get_backend(self.process_group) == "gloo":
            dev = torch.device("cpu")
        info = torch.zeros(1 + 2 * P, dtype=torch.int64, device=dev)
        if self.rank == 0:
            flat = [len(buckets)] + [len(b.params) for b in buckets] + [i for b in buckets for i in b.params]
            info[: len(flat)] = torch.tensor(flat, dtype=torch.int64)
        dist.broadcast(info, _group_rank0(self.process_group), group=self.process_group)
        info = info.cpu().tolist()
        nb = info[0]
        sizes = info[1:1 + nb]
        idxs = info[1 + nb:1 + nb + sum(sizes)]
        out, pos = [], 0
        for s in sizes:
            ps = idxs[pos:pos + s]
            pos += s
            b = _Bucket(ps, self.active_params[ps[0]].dtype)
            b.numel = sum(self.active_params[i].numel() for i in ps)
            out.append(b)
        return out

    def _alloc_slots(self, b: _Bucket):
        """Persistent flat buffer of a bucket and one slot view per parameter (gradient-as-bucket-view)."""
        p0 = self.active_params[b.params[0]]
        if b.flat is None or b.flat.numel() != b.numel or b.flat.device != p0.device or b.flat.dtype != p0.dtype:
            b.flat = torch.empty(b.numel, dtype=p0.dtype, device=p0.device)
        b.slots, off = {}, 0
        for i in b.params:
            p = self.active_params[i]
            b.slots[i] = _slot_view(b.flat, off, p)
            if self.gradient_as_bucket_view:
                _view_slots()[p] = b.slots[i].data_ptr()
            off += p.numel()

    def _to_slot(self, b: _Bucket, i: int):
        """Copy the gradient into its bucket slot (unless it is already there); with
        gradient_as_bucket_view ``param.grad`` then becomes the slot view."""
        if b.slots is None:
            self._alloc_slots(b)
        p, slot = self.active_params[i], b.slots[i]
        g = p.grad
        if g is None:
            slot.zero_()
            if not self.gradient_as_bucket_view:
                p.grad = torch.zeros_like(p)  # receives the average (other ranks may have one)
                return
        elif g.data_ptr() != slot.data_ptr() or g.stride() != slot.stride():
            _raw(slot).copy_(_raw(g if g.stride() == slot.stride() else g.contiguous(memory_format=_fmt(slot))))
        else:
            return
        if self.gradient_as_bucket_view:
            p.grad = slot

    def _launch(self, b_idx):
        b = self._buckets[b_idx]
        if b.launched:
            return
        if b.slots is None:
            self._alloc_slots(b)
        for i in b.params:  # parameters the hooks have not placed yet (first / delayed / unused)
            if i not in b.placed:
                self._to_slot(b, i)
        tensor = b.flat.float() if self.allreduce_always_fp32 and b.flat.dtype != torch.float32 else b.flat
        if self.gradient_predivide_factor != 1.0:
            tensor.mul_(1.0 / self.gradient_predivide_factor)
        op = dist.ReduceOp.AVG if self._use_avg else dist.ReduceOp.SUM
        b.work = dist.all_reduce(tensor, op=op, group=self._pg_for(b_idx), async_op=True)
        b.outputs = tensor
        b.launched = True

    def _finish(self, b_idx):
        b = self._buckets[b_idx]
        if b.work is not None:
            with comm_stats.timed("ddp_wait", b.flat):
                b.work.wait()
            b.work = None
        tensor = b.outputs
        if self.gradient_average and not self._use_avg:
            tensor.mul_(self.gradient_predivide_factor / self.world_size)
        if tensor is not b.flat:
            b.flat.copy_(tensor)
        if not self.gradient_as_bucket_view:  # the averaged slots back into the parameters' own grads
            ps = [self.active_params[i] for i in b.params]
            torch._foreach_copy_([p.grad for p in ps], [b.slots[i] for i in b.params])
        if self.retain_allreduce_buffers:
            self.allreduce_buffers[b_idx] = b.flat
        b.outputs = None

    def _end_of_backward(self):
        if self.prof:
            torch.cuda.nvtx.range_push("allreduce_params")
        if self.needs_refresh:
            buckets = self._build_buckets(self._arrival)
            self._buckets = self._sync_bucket_structure(buckets)
            self._param_to_bucket = {i: bi for bi, b in enumerate(self._buckets) for i in b.params}
            self.needs_refresh = False
            if self.retain_allreduce_buffers:
                self.allreduce_buffers = [None for _ in self._buckets]
        for bi in range(len(self._buckets)):
            self._launch(bi)  # buckets not yet launched (first / delayed / unused-param iterations)
        for bi in range(len(self._buckets)):
            self._finish(bi)
        self._callback_queued = False
        self._next_bucket = 0
        for b in self._buckets:
            b.launched, b.ready = False, 0
            b.placed.clear()
        if self.prof:
            torch.cuda.nvtx.range_pop()
