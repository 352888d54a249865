"""ZeRO-2 AdamW: optimizer state and gradients sharded over data-parallel ranks
(reference: apex/contrib/optimizers/distributed_fused_adam.py:19-1310).

MI355X-first design (288 GB HBM per GPU, RCCL over xGMI):

* Parameters are packed, per dtype, into large flat **buckets** (``bucket_cap_mb``, default 100 MB;
  a parameter never straddles buckets — a bucket grows to hold a larger one). Each parameter's
  ``.data`` and ``.grad`` become *views* into its bucket's parameter / gradient buffers, so
  autograd accumulates gradients straight into the bucket (no per-parameter grad copy) and the
  parameter all-gather writes straight into the model's parameters (no copy back).
* Buckets are ordered by reverse registration order (≈ gradient arrival order); a post-accumulate
  hook launches the bucket's ``reduce_scatter_tensor`` as soon as its last gradient lands, on RCCL's
  stream, overlapped with the rest of backward. One large collective per bucket is what a
  per-link-bound xGMI ring wants. Averaging is folded into the optimizer's unscale factor (SUM
  collective + 1/world inside the Adam kernel: no extra pass, works on every backend).
* The step is sync-free: the gradient norm (for clipping and inf detection) is one fused l2-norm
  over the local shards + one scalar all-reduce; the Adam update runs the capturable multi-tensor
  kernel with device-resident lr / step / inv_scale / found_inf and writes the param-sync-dtype
  copy in the same pass; then one ``all_gather_into_tensor`` per bucket refreshes the parameters.
* ``redundant_process_group`` (HSDP-style replicas of the shards) adds one shard all-reduce.
"""
from __future__ import annotations

import collections
import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C, fused_adam_cuda


def _round_up(n, m):
    return (n + m - 1) // m * m


class _Bucket:
    """One flat bucket: parameter/gradient buffers (full size) + this rank's optimizer shard."""

    def __init__(self, dtype, device, params, dist_size, dist_rank, alignment, state_dtype, grad_sync_dtype,
                 param_sync_dtype):
        self.params = params
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += _round_up(p.numel(), alignment)
        self.size = _round_up(max(off, 1), dist_size * alignment)
        self.shard_size = self.size // dist_size
        self.shard_start = dist_rank * self.shard_size
        self.param_buffer = torch.zeros(self.size, dtype=dtype, device=device)
        self.grad_buffer = torch.zeros(self.size, dtype=dtype, device=device)
        self.sync_grad = (self.grad_buffer if grad_sync_dtype == dtype
                          else torch.zeros(self.size, dtype=grad_sync_dtype, device=device))
        self.grad_shard = torch.zeros(self.shard_size, dtype=grad_sync_dtype, device=device)
        self.param_sync_shard = torch.zeros(self.shard_size, dtype=param_sync_dtype, device=device)
        self.param_sync_full = (self.param_buffer if param_sync_dtype == dtype
                                else torch.zeros(self.size, dtype=param_sync_dtype, device=device))
        # optimizer shard state
        self.master = torch.zeros(self.shard_size, dtype=state_dtype, device=device)
        self.exp_avg = torch.zeros(self.shard_size, dtype=state_dtype, device=device)
        self.exp_avg_sq = torch.zeros(self.shard_size, dtype=state_dtype, device=device)
        self.ready = set()
        self.work = None
        # per-element group id of this shard (for per-group hyper-parameters) is resolved by fragments
        self.fragments = []  # (param_index, param_lo, param_hi, shard_lo, shard_hi)
        for i, (p, o) in enumerate(zip(params, self.offsets)):
            lo = max(o, self.shard_start)
            hi = min(o + p.numel(), self.shard_start + self.shard_size)
            if lo < hi:
                self.fragments.append((i, lo - o, hi - o, lo - self.shard_start, hi - self.shard_start))

    def view(self, buf, i):
        p = self.params[i]
        o = self.offsets[i]
        return buf[o:o + p.numel()].view(p.shape)


class DistributedFusedAdam(torch.optim.Optimizer):
    """AdamW with ZeRO-2 sharding. Arguments follow the reference (``lr``, ``bias_correction``,
    ``betas``, ``eps``, ``weight_decay``, ``dtype`` (state), ``grad_sync_dtype``,
    ``param_sync_dtype``, ``process_group``, ``distributed_process_group``,
    ``redundant_process_group``, ``average_grad_sync``, ``overlap_grad_sync``, ``bucket_cap_mb``,
    ``pipeline_size``, ``contiguous_grad_buffer``). ``adam_w_mode=False`` selects L2 Adam."""

    _step_supports_amp_scaling = True

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, dtype=torch.float32, grad_sync_dtype=None, param_sync_dtype=None, device="cuda",
                 process_group=None, distributed_process_group=None, redundant_process_group=None,
                 average_grad_sync=True, overlap_grad_sync=True, bucket_cap_mb=100, pipeline_size=2,
                 contiguous_grad_buffer=True, adam_w_mode=True):
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if amsgrad:
            raise RuntimeError("DistributedFusedAdam does not support the AMSGrad variant.")
        self.dtype = dtype
        self.grad_sync_dtype = grad_sync_dtype
        self.param_sync_dtype = param_sync_dtype
        self.adam_w_mode = adam_w_mode
        self.process_group = process_group if process_group is not None else dist.group.WORLD
        self.distributed_process_group = distributed_process_group or self.process_group
        self.redundant_process_group = redundant_process_group
        self.distributed_rank = dist.get_rank(self.distributed_process_group)
        self.distributed_size = dist.get_world_size(self.distributed_process_group)
        self.redundant_size = 1 if redundant_process_group is None else dist.get_world_size(redundant_process_group)
        if dist.get_world_size(self.process_group) != self.distributed_size * self.redundant_size:
            raise RuntimeError("Invalid process group configuration (process group size != distributed size x "
                               "redundant size)")
        self.average_grad_sync = average_grad_sync
        self.overlap_grad_sync = overlap_grad_sync
        self.pipeline_size = pipeline_size
        self.contiguous_grad_buffer = contiguous_grad_buffer
        self.bucket_cap_mb = bucket_cap_mb
        self._grad_sync_enabled = True
        self._grad_norm = None
        self._buckets: List[_Bucket] = []
        self._param_loc: Dict[int, tuple] = {}
        self._group_of: Dict[int, int] = {}
        self._hooks = []
        self.state["step"] = 0
        self._build_buckets()

    # ------------------------------------------------------------------ construction
    def _build_buckets(self):
        plist = []
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                if p.requires_grad and id(p) not in self._group_of:
                    self._group_of[id(p)] = gi
                    plist.append(p)
        if not plist:
            return
        self.device = plist[0].device
        by_dtype = collections.OrderedDict()
        for p in reversed(plist):  # gradients arrive roughly in reverse registration order
            by_dtype.setdefault(p.dtype, []).append(p)
        alignment = 16
        for dtype, ps in by_dtype.items():
            cap = max(1, int(self.bucket_cap_mb * 2 ** 20) // torch.tensor([], dtype=dtype).element_size())
            cur, cur_n = [], 0
            groups = []
            for p in ps:
                if cur and cur_n + p.numel() > cap:
                    groups.append(cur)
                    cur, cur_n = [], 0
                cur.append(p)
                cur_n += _round_up(p.numel(), alignment)
            if cur:
                groups.append(cur)
            for members in groups:
                b = _Bucket(dtype, self.device, members, self.distributed_size, self.distributed_rank, alignment,
                            self.dtype, self.grad_sync_dtype or dtype, self.param_sync_dtype or dtype)
                bi = len(self._buckets)
                self._buckets.append(b)
                with torch.no_grad():
                    for i, p in enumerate(members):
                        b.view(b.param_buffer, i).copy_(p.detach())
                        self._param_loc[id(p)] = (bi, i)
                    # parameters become views into the bucket; master shard from the bucket
                    for i, p in enumerate(members):
                        p.data = b.view(b.param_buffer, i)
                        p.grad = b.view(b.grad_buffer, i) if self.contiguous_grad_buffer else None
                    b.master.copy_(b.param_buffer[b.shard_start:b.shard_start + b.shard_size].to(self.dtype))
                    self._pack_sync(b.param_sync_shard, b.param_buffer[b.shard_start:b.shard_start + b.shard_size])
        # broadcast initial parameters so every rank starts identical (reference: init broadcast)
        for b in self._buckets:
            src = dist.get_global_rank(self.process_group, 0) if self.process_group is not dist.group.WORLD else 0
            dist.broadcast(b.param_buffer, src, group=self.process_group)
            b.master.copy_(b.param_buffer[b.shard_start:b.shard_start + b.shard_size].to(self.dtype))
            self._pack_sync(b.param_sync_shard, b.param_buffer[b.shard_start:b.shard_start + b.shard_size])
        self._register_post_backward_hooks()

    @staticmethod
    def _pack_sync(dst, src):
        """src (param / master dtype) -> parameter all-gather dtype (uint8 = e5m2 bytes)."""
        if dst.dtype == torch.uint8:
            fused_adam_cuda.maybe_cast(None, src.contiguous(), dst)
        else:
            dst.copy_(src)

    @staticmethod
    def _unpack_sync(dst, src):
        if src.dtype == torch.uint8:
            fused_adam_cuda.maybe_cast(None, src, dst)
        else:
            dst.copy_(src)

    def _register_post_backward_hooks(self):
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) not in self._param_loc:
                    continue
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _on_grad(self, p):
        bi, i = self._param_loc[id(p)]
        b = self._buckets[bi]
        view = b.view(b.grad_buffer, i)
        if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
            # autograd produced a fresh tensor (.grad was None or had another layout): fold it in
            view.add_(p.grad)
            p.grad = view
        b.ready.add(i)
        if self.overlap_grad_sync and self._grad_sync_enabled and len(b.ready) == len(b.params):
            self._start_bucket_sync(b)

    # ------------------------------------------------------------------ gradient sync
    def _start_bucket_sync(self, b: _Bucket):
        if b.work is not None:
            return
        src = b.grad_buffer
        if b.sync_grad is not b.grad_buffer:
            b.sync_grad.copy_(b.grad_buffer)
            src = b.sync_grad
        if self.distributed_size == 1:
            b.grad_shard.copy_(src)
            b.work = _Done()
        else:
            b.work = dist.reduce_scatter_tensor(b.grad_shard, src, group=self.distributed_process_group,
                                                async_op=True)

    def _finish_grad_sync(self):
        for b in self._buckets:
            if b.work is None:
                self._start_bucket_sync(b)
        for b in self._buckets:
            b.work.wait()
            if self.redundant_size > 1:
                dist.all_reduce(b.grad_shard, group=self.redundant_process_group)
            b.work = None
            b.ready.clear()

    @contextlib.contextmanager
    def no_sync(self, greedy_grad_copy=False):
        """Accumulate gradients locally (e.g. all but the last microbatch)."""
        old = self._grad_sync_enabled
        self._grad_sync_enabled = False
        try:
            yield
        finally:
            self._grad_sync_enabled = old
            for b in self._buckets:
                b.ready.clear()

    def grad_sync(self):
        """Start the reduce-scatter of every bucket that has not started yet (and wait)."""
        self._finish_grad_sync()

    def zero_grad(self, set_to_none=False):
        for b in self._buckets:
            b.grad_buffer.zero_()
            b.ready.clear()
            b.work = None
            for i, p in enumerate(b.params):
                p.grad = b.view(b.grad_buffer, i) if self.contiguous_grad_buffer else None
        self._grad_norm = None

    def grad_buffer_view(self, param):
        bi, i = self._param_loc[id(param)]
        return self._buckets[bi].view(self._buckets[bi].grad_buffer, i)

    # ------------------------------------------------------------------ norms / clipping
    def _grad_scale_divisor(self):
        return float(self.distributed_size * self.redundant_size) if self.average_grad_sync else 1.0

    def _local_grad_norm_sq(self):
        shards = [b.grad_shard for b in self._buckets]
        if not shards:
            return torch.zeros(1, device="cpu")
        flag = torch.zeros(1, dtype=torch.int, device=self.device)
        groups = collections.defaultdict(list)
        for s in shards:
            groups[s.dtype].append(s)
        sq = torch.zeros(1, dtype=torch.float32, device=self.device)
        for gs in groups.values():
            n, _ = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [gs], False)
            sq = sq + n.float().reshape(1) ** 2
        return sq

    def grad_norm(self, parameters=[], norm_type=2.0, force=False):
        """Global L2 norm of the (averaged, still loss-scaled) gradients; device tensor, cached."""
        assert norm_type == 2.0, "only the L2 norm is supported"
        if self._grad_norm is None or force:
            self._finish_grad_sync()
            sq = self._local_grad_norm_sq()
            dist.all_reduce(sq, group=self.distributed_process_group)
            self._grad_norm = sq.sqrt() / self._grad_scale_divisor()
        return self._grad_norm

    def clip_grad_norm(self, max_norm, parameters=[], norm_type=2.0):
        """Clip by the global norm (applied inside the next step's unscale factor). Returns the norm."""
        norm = self.grad_norm(parameters, norm_type)
        self._clip_coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        return norm

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None, *, grad_scaler=None):
        loss = closure() if closure is not None else None
        if not self._buckets:
            return loss
        self._finish_grad_sync()
        inv = torch.full([1], 1.0 / self._grad_scale_divisor(), dtype=torch.float32, device=self.device)
        found_inf = torch.zeros(1, dtype=torch.float32, device=self.device)
        if grad_scaler is not None and getattr(grad_scaler, "_enabled", True):
            scale = grad_scaler._get_scale_async() if hasattr(grad_scaler, "_get_scale_async") else grad_scaler._scale
            inv = inv * scale.double().reciprocal().float().reshape(1)
            norm = self.grad_norm(force=True)
            found_inf = (~torch.isfinite(norm)).float().reshape(1)
            st = grad_scaler._per_optimizer_states[id(self)]
            st["found_inf_per_device"] = {found_inf.device: found_inf}
            from torch.amp.grad_scaler import OptState
            st["stage"] = OptState.STEPPED
        if getattr(self, "_clip_coef", None) is not None:
            inv = inv * self._clip_coef.reshape(1)
            self._clip_coef = None
        self.state["step"] += 1
        step_t = torch.full([1], self.state["step"], dtype=torch.int, device=self.device)
        flag = torch.zeros(1, dtype=torch.int, device=self.device)
        for gi, group in enumerate(self.param_groups):
            lists = [[], [], [], [], []]
            for b in self._buckets:
                for (i, plo, phi, slo, shi) in b.fragments:
                    if self._group_of[id(b.params[i])] != gi:
                        continue
                    lists[0].append(b.grad_shard[slo:shi])
                    lists[1].append(b.master[slo:shi])
                    lists[2].append(b.exp_avg[slo:shi])
                    lists[3].append(b.exp_avg_sq[slo:shi])
                    lists[4].append(b.param_sync_shard[slo:shi])
            if not lists[0]:
                continue
            beta1, beta2 = group["betas"]
            lr_t = torch.full([1], group["lr"], dtype=torch.float32, device=self.device)
            # the kernel requires one dtype per list: split by (grad dtype, sync dtype)
            keyed = collections.defaultdict(lambda: [[], [], [], [], []])
            for k in range(len(lists[0])):
                key = (lists[0][k].dtype, lists[4][k].dtype)
                for j in range(5):
                    keyed[key][j].append(lists[j][k])
            for sub in keyed.values():
                multi_tensor_applier(amp_C.multi_tensor_adam_capturable, flag, sub, lr_t, beta1, beta2,
                                     group["eps"], step_t, 1 if self.adam_w_mode else 0,
                                     1 if group["bias_correction"] else 0, group["weight_decay"], inv, found_inf)
        # refresh parameters: all-gather the param-sync shards straight into the bucket buffers
        works = []
        for b in self._buckets:
            if self.distributed_size == 1:
                b.param_sync_full.copy_(b.param_sync_shard)
            else:
                works.append(dist.all_gather_into_tensor(b.param_sync_full, b.param_sync_shard,
                                                         group=self.distributed_process_group, async_op=True))
        for w in works:
            w.wait()
        for b in self._buckets:
            if b.param_sync_full is not b.param_buffer:
                self._unpack_sync(b.param_buffer, b.param_sync_full)
        self._grad_norm = None
        return loss

    # ------------------------------------------------------------------ checkpointing
    def _global_param_index(self):
        """Global parameter numbering of torch.optim's state_dict (param_groups order)."""
        idx, out = 0, {}
        for g in self.param_groups:
            for p in g["params"]:
                out[id(p)] = idx
                idx += 1
        return out

    def _local_state(self):
        """This rank's shard as layout-free per-parameter fragments (CPU tensors)."""
        pidx = self._global_param_index()
        frags = []
        for b in self._buckets:
            for (i, plo, phi, slo, shi) in b.fragments:
                frags.append({"param": pidx[id(b.params[i])], "lo": plo, "hi": phi,
                              "master": b.master[slo:shi].cpu(), "exp_avg": b.exp_avg[slo:shi].cpu(),
                              "exp_avg_sq": b.exp_avg_sq[slo:shi].cpu()})
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = [pidx[id(p)] for p in g["params"]]
            groups.append(d)
        return {"state": {"step": self.state["step"], "fragments": frags, "distributed_size": self.distributed_size,
                          "distributed_rank": self.distributed_rank},
                "param_groups": groups}

    def state_dict(self, gather_on_root=True):
        """Optimizer state in the reference's layout (``distributed_fused_adam.py:1123-1262``).

        ``gather_on_root=True`` (collective): every rank serialises its local state, root returns
        ``{"gathered_states": [bytes of rank 0, rank 1, ...]}`` and the other ranks ``None``.
        ``gather_on_root=False``: this rank's local state dict. The local state is a list of
        per-parameter fragments (global param index, element range, master / exp_avg /
        exp_avg_sq), so a checkpoint loads back under ANY distributed size or bucket size."""
        local = self._local_state()
        if not gather_on_root:
            return local
        import io

        buf = io.BytesIO()
        torch.save(local, buf)
        blob = buf.getvalue()
        gathered = [None] * self.distributed_size if self.distributed_rank == 0 else None
        if self.distributed_size == 1:
            gathered = [blob]
        else:
            root = dist.get_global_rank(self.distributed_process_group, 0) \
                if self.distributed_process_group is not dist.group.WORLD else 0
            dist.gather_object(blob, gathered, dst=root, group=self.distributed_process_group)
        if self.distributed_rank == 0:
            return {"gathered_states": gathered}
        return None

    def load_state_dict(self, state_dict):
        """Load a ``{"gathered_states": [...]}`` checkpoint (any distributed size) or a local dict."""
        import io

        if "gathered_states" in state_dict:
            locals_ = [torch.load(io.BytesIO(bytes(blob)), weights_only=True) for blob in state_dict["gathered_states"]]
        else:
            locals_ = [state_dict]
        for g, sg in zip(self.param_groups, locals_[0]["param_groups"]):
            g.update({k: v for k, v in sg.items() if k != "params"})
        self.state["step"] = locals_[0]["state"]["step"]
        # reassemble per-parameter state from every rank's fragments, then take this rank's shards
        full: Dict[int, Dict[str, torch.Tensor]] = {}
        pidx = self._global_param_index()
        numel = {pidx[id(p)]: p.numel() for g in self.param_groups for p in g["params"]}
        for loc in locals_:
            for f in loc["state"]["fragments"]:
                ent = full.setdefault(f["param"], {})
                for name in ("master", "exp_avg", "exp_avg_sq"):
                    if name not in ent:
                        ent[name] = torch.zeros(numel[f["param"]], dtype=f[name].dtype)
                    ent[name][f["lo"]:f["hi"]] = f[name]
        for b in self._buckets:
            for (i, plo, phi, slo, shi) in b.fragments:
                ent = full.get(pidx[id(b.params[i])])
                if ent is None:
                    continue
                for name in ("master", "exp_avg", "exp_avg_sq"):
                    getattr(b, name)[slo:shi].copy_(ent[name][plo:phi])
            self._pack_sync(b.param_sync_shard, b.master)
            if self.distributed_size == 1:
                b.param_sync_full.copy_(b.param_sync_shard)
            else:
                dist.all_gather_into_tensor(b.param_sync_full, b.param_sync_shard, group=self.distributed_process_group)
            if b.param_sync_full is not b.param_buffer:
                self._unpack_sync(b.param_buffer, b.param_sync_full)


class _Done:
    def wait(self):
        return True
