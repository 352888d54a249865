"""ZeRO-sharded LAMB (reference: apex/contrib/optimizers/distributed_fused_lamb.py:19-905).

Shares the bucket / shard machinery of :class:`DistributedFusedAdam` (parameters and gradients as
views into flat per-dtype buckets, one reduce-scatter per bucket overlapped with backward, one
all-gather per bucket after the step). LAMB needs per-PARAMETER norms of the weights and of the
update while each rank only holds fragments of parameters, so the step is:

1. global gradient norm of the RAW reduced shards: fused l2-norm + one scalar all-reduce. Overflow
   (non-finite norm) becomes a device ``noop`` flag: every later kernel returns immediately, the
   device step counter does not advance -- no host synchronisation anywhere in the step;
2. update term (``distributed_lamb_cuda.multi_tensor_lamb_compute_update_term``, per fragment):
   unscale by the device ``global_scale`` (world x loss scale x user scale), clip by
   ``max_grad_norm``, Adam moments, ``u`` (+ decoupled weight decay) -- no separate unscale pass;
3. per-fragment ||p||^2 and ||u||^2 (fused per-tensor l2-norm) scattered into per-parameter vectors
   and summed over the shard group with ONE all-reduce of a [2, n_params] tensor;
4. ``multi_tensor_lamb_update_weights``: ``p -= lr * (||p||/||u||) * u`` and, in the same pass, the
   all-gather payload (param dtype, or e5m2 bytes with ``e5m2_allgather=True``: a quarter / half the
   all-gather bytes, decompressed into the parameters after the collective).
Per-fragment hyper-parameter vectors and index maps are built once and cached on the device.
The reference's block/chunk/shard pipelines with separate RS/AR/AG process-group pools (``dwu_*``)
are NCCL-scheduling devices; RCCL here runs one collective per bucket on its own stream, so those
arguments are accepted for API compatibility.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C, distributed_lamb_cuda
from .distributed_fused_adam import DistributedFusedAdam


class DistributedFusedLAMB(DistributedFusedAdam):
    def __init__(self, params, lr=1e-3, bias_correction=True, grad_averaging=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, max_grad_norm=0.0, adam_w_mode=True, use_nvlamb=False,
                 step_supports_amp_scaling=True, overlap_reductions=True, dwu_group_size=0, dwu_num_blocks=4,
                 dwu_num_chunks=4, dwu_num_rs_pg=1, dwu_num_ar_pg=4, dwu_num_ag_pg=0, e5m2_allgather=False,
                 verbose=False, clip_after_ar=True, process_group=None, bucket_cap_mb=100, dtype=torch.float32):
        super().__init__(params, lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                         weight_decay=weight_decay, dtype=dtype, process_group=process_group,
                         overlap_grad_sync=overlap_reductions, bucket_cap_mb=bucket_cap_mb, adam_w_mode=adam_w_mode,
                         param_sync_dtype=torch.uint8 if e5m2_allgather else None)
        for g in self.param_groups:
            g.setdefault("max_grad_norm", max_grad_norm)
            g.setdefault("grad_averaging", grad_averaging)
        self.max_grad_norm = max_grad_norm
        self.use_nvlamb = use_nvlamb
        self.e5m2_allgather = e5m2_allgather
        self._global_scale = 1.0
        self._lamb_param_index = {}
        n = 0
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) in self._param_loc:
                    self._lamb_param_index[id(p)] = n
                    n += 1
        self._n_params = n
        for b in self._buckets:
            b.update = torch.zeros(b.shard_size, dtype=torch.float32, device=b.master.device)
        self._plans = None
        self._step_t = None
        self._noop = None

    # reference API -----------------------------------------------------------------------------
    def set_global_scale(self, global_scale):
        """Loss scale the gradients carry (divided out inside the step)."""
        self._global_scale = global_scale

    @property
    def global_scale(self):
        return self._global_scale

    @property
    def L2_grad_norm(self):
        return self._grad_norm

    @property
    def has_overflow(self):
        """Device int flag of the last step (1: skipped because of a non-finite gradient norm)."""
        return self._noop

    def set_is_accumulation_step(self, is_accumulation_step):
        self._grad_sync_enabled = not is_accumulation_step

    def set_last_step(self, last_step):
        pass

    def complete_reductions(self):
        self._finish_grad_sync()

    # cached per-group fragment plans -----------------------------------------------------------
    def _build_plans(self):
        dev = self.device
        plans = []
        for gi, group in enumerate(self.param_groups):
            frags = [(b, b.params[i], slo, shi) for b in self._buckets for (i, plo, phi, slo, shi) in b.fragments
                     if self._group_of[id(b.params[i])] == gi]
            if not frags:
                continue
            beta1, beta2 = group["betas"]
            T = len(frags)
            full = lambda v, dt=torch.float32: torch.full([T], v, dtype=dt, device=dev)  # noqa: E731
            plans.append(dict(
                group=group,
                g=[b.grad_shard[lo:hi] for b, _, lo, hi in frags],
                p=[b.master[lo:hi] for b, _, lo, hi in frags],
                m=[b.exp_avg[lo:hi] for b, _, lo, hi in frags],
                v=[b.exp_avg_sq[lo:hi] for b, _, lo, hi in frags],
                u=[b.update[lo:hi] for b, _, lo, hi in frags],
                c=[b.param_sync_shard[lo:hi] for b, _, lo, hi in frags],
                beta1=full(beta1), beta2=full(beta2),
                beta3=full(1.0 - beta1 if group.get("grad_averaging", True) else 1.0),
                eps=full(group["eps"]),
                decay=full(group["weight_decay"]),
                bias_correction=full(1 if group["bias_correction"] else 0, torch.int),
                idx=torch.tensor([self._lamb_param_index[id(p)] for _, p, _, _ in frags], dtype=torch.long,
                                 device=dev),
                key=(group["betas"], group["eps"], group["weight_decay"], group["bias_correction"],
                     group.get("grad_averaging", True)),
            ))
        self._plans = plans

    # step --------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None, grad_scaler=None):
        loss = closure() if closure is not None else None
        if not self._buckets:
            return loss
        self._finish_grad_sync()
        dev = self.device
        if self._plans is None or any(pl["key"] != (pl["group"]["betas"], pl["group"]["eps"],
                                                     pl["group"]["weight_decay"], pl["group"]["bias_correction"],
                                                     pl["group"].get("grad_averaging", True))
                                      for pl in self._plans):
            self._build_plans()
        if self._step_t is None:
            self._step_t = torch.full([1], int(self.state["step"]), dtype=torch.int, device=dev)
        # 1. global norm of the raw (summed, loss-scaled) gradient shards; overflow -> device noop flag
        gscale = torch.full([1], self._grad_scale_divisor() * float(self._global_scale), dtype=torch.float32,
                            device=dev)
        if grad_scaler is not None and getattr(grad_scaler, "_enabled", True):
            s = grad_scaler._get_scale_async() if hasattr(grad_scaler, "_get_scale_async") else grad_scaler._scale
            gscale = gscale * s.float().reshape(1)
        sq = self._local_grad_norm_sq()
        dist.all_reduce(sq, group=self.distributed_process_group)
        raw_norm = sq.sqrt().reshape(1)
        noop = (~torch.isfinite(raw_norm)).int()
        self._noop = noop
        self._grad_norm = raw_norm / gscale
        if grad_scaler is not None and getattr(grad_scaler, "_enabled", True):
            st = grad_scaler._per_optimizer_states[id(self)]
            st["found_inf_per_device"] = {dev: noop.float()}
            from torch.amp.grad_scaler import OptState
            st["stage"] = OptState.STEPPED
        self._step_t += 1 - noop
        self.state["step"] += 1  # host counter of attempted steps; state_dict() reads the device one
        for pl in self._plans:
            group = pl["group"]
            max_norm = group.get("max_grad_norm", self.max_grad_norm) or 0.0
            # 2. update term
            distributed_lamb_cuda.multi_tensor_lamb_compute_update_term(
                2048 * 32, noop, [pl["g"], pl["p"], pl["m"], pl["v"], pl["u"]], pl["beta1"], pl["beta2"],
                pl["beta3"], pl["bias_correction"], self._step_t, pl["eps"], 1 if self.adam_w_mode else 0,
                pl["decay"], gscale, raw_norm, max_norm)
            # 3. per-parameter norms across shards: one [2, n_params] all-reduce
            flag = torch.zeros(1, dtype=torch.int, device=dev)
            _, pn = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [pl["p"]], True)
            _, un = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [pl["u"]], True)
            sums = torch.zeros(2, self._n_params, dtype=torch.float32, device=dev)
            sums[0].index_add_(0, pl["idx"], pn.float() ** 2)
            sums[1].index_add_(0, pl["idx"], un.float() ** 2)
            dist.all_reduce(sums, group=self.distributed_process_group)
            norms = sums.sqrt()
            # 4. trust-ratio update + all-gather payload in one pass
            lr_t = torch.full([1], group["lr"], dtype=torch.float32, device=dev)
            distributed_lamb_cuda.multi_tensor_lamb_update_weights(
                2048 * 32, noop, [pl["p"], pl["u"], pl["c"]], norms[0][pl["idx"]], norms[1], pl["idx"], lr_t,
                pl["decay"], raw_norm, self.use_nvlamb)
        # refresh parameters (e5m2 payloads are decompressed into the parameters)
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
        return loss

    def state_dict(self, gather_on_root=True):
        if self._step_t is not None:
            self.state["step"] = int(self._step_t.item())  # checkpoint-time read of the device counter
        return super().state_dict(gather_on_root)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._step_t = None
