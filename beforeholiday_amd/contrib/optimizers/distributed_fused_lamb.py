"""ZeRO-sharded LAMB (reference: apex/contrib/optimizers/distributed_fused_lamb.py:19-905).

Shares the bucket / shard machinery of :class:`DistributedFusedAdam` (parameters and gradients as
views into flat per-dtype buckets, one reduce-scatter per bucket overlapped with backward, one
all-gather per bucket after the step). LAMB needs per-PARAMETER norms of the weights and of the
update while each rank only holds fragments of parameters, so the step is:

1. global gradient norm: fused l2-norm of the local shards + one scalar all-reduce; gradients are
   unscaled / averaged in one multi-tensor scale pass (device scalar, no host sync);
2. stage 1 (fused kernel, per fragment): Adam moments + update ``u`` (+ decoupled weight decay),
   clipping by ``max_grad_norm`` folded in;
3. per-fragment ||p||^2 and ||u||^2 (fused per-tensor l2-norm) scattered into per-parameter vectors
   and summed over the shard group with ONE all-reduce of a [2, n_params] tensor;
4. stage 2 (fused kernel): p -= lr * (||p|| / ||u||) * u using the global per-parameter norms.
The reference's block/chunk/shard pipelines with separate RS/AR/AG process-group pools
(``dwu_*``) are NCCL-scheduling devices; they are accepted for API compatibility and ignored.
``e5m2_allgather`` is accepted and ignored (parameters are all-gathered in their own dtype).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C
from .distributed_fused_adam import DistributedFusedAdam


class DistributedFusedLAMB(DistributedFusedAdam):
    def __init__(self, params, lr=1e-3, bias_correction=True, grad_averaging=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, max_grad_norm=0.0, adam_w_mode=True, use_nvlamb=False,
                 step_supports_amp_scaling=True, overlap_reductions=True, dwu_group_size=0, dwu_num_blocks=4,
                 dwu_num_chunks=4, dwu_num_rs_pg=1, dwu_num_ar_pg=4, dwu_num_ag_pg=0, e5m2_allgather=False,
                 verbose=False, clip_after_ar=True, process_group=None, bucket_cap_mb=100, dtype=torch.float32):
        super().__init__(params, lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                         weight_decay=weight_decay, dtype=dtype, process_group=process_group,
                         overlap_grad_sync=overlap_reductions, bucket_cap_mb=bucket_cap_mb, adam_w_mode=adam_w_mode)
        for g in self.param_groups:
            g.setdefault("max_grad_norm", max_grad_norm)
            g.setdefault("grad_averaging", grad_averaging)
        self.max_grad_norm = max_grad_norm
        self.use_nvlamb = use_nvlamb
        self._global_scale = 1.0
        self._param_index = {}
        n = 0
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) in self._param_loc:
                    self._param_index[id(p)] = n
                    n += 1
        self._n_params = n
        for b in self._buckets:
            b.update = torch.zeros_like(b.master)

    # reference API -----------------------------------------------------------------------------
    def set_global_scale(self, global_scale):
        """Loss scale the gradients carry (divided out inside the step)."""
        self._global_scale = global_scale

    @property
    def global_scale(self):
        return self._global_scale

    @property
    def L2_grad_norm(self):
        return self.grad_norm() / self._global_scale if self._grad_norm is not None else None

    def set_is_accumulation_step(self, is_accumulation_step):
        self._grad_sync_enabled = not is_accumulation_step

    def set_last_step(self, last_step):
        pass

    def complete_reductions(self):
        self._finish_grad_sync()

    # step --------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None, grad_scaler=None):
        loss = closure() if closure is not None else None
        if not self._buckets:
            return loss
        self._finish_grad_sync()
        dev = self.device
        flag = torch.zeros(1, dtype=torch.int, device=dev)
        scale = torch.full([1], 1.0 / (self._grad_scale_divisor() * self._global_scale), dtype=torch.float32,
                           device=dev)
        found_inf = None
        if grad_scaler is not None and getattr(grad_scaler, "_enabled", True):
            s = grad_scaler._get_scale_async() if hasattr(grad_scaler, "_get_scale_async") else grad_scaler._scale
            scale = scale * s.double().reciprocal().float().reshape(1)
        # 1. unscale/average gradients in place, then global norm
        for dt in {b.grad_shard.dtype for b in self._buckets}:
            shards = [b.grad_shard for b in self._buckets if b.grad_shard.dtype == dt]
            multi_tensor_applier(amp_C.multi_tensor_scale, flag, [shards, shards], scale)
        sq = self._local_grad_norm_sq()
        dist.all_reduce(sq, group=self.distributed_process_group)
        gnorm = sq.sqrt()
        self._grad_norm = gnorm
        if grad_scaler is not None and getattr(grad_scaler, "_enabled", True):
            found_inf = (~torch.isfinite(gnorm)).float().reshape(1)
            st = grad_scaler._per_optimizer_states[id(self)]
            st["found_inf_per_device"] = {found_inf.device: found_inf}
            from torch.amp.grad_scaler import OptState
            st["stage"] = OptState.STEPPED
            if found_inf.item() != 0.0:  # one host read per step, only under a GradScaler
                self._grad_norm = None
                return loss
        self.state["step"] += 1
        step = self.state["step"]
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            max_norm = group.get("max_grad_norm", self.max_grad_norm) or 0.0
            frags = []  # (bucket, param, slo, shi)
            for b in self._buckets:
                for (i, plo, phi, slo, shi) in b.fragments:
                    if self._group_of[id(b.params[i])] == gi:
                        frags.append((b, b.params[i], slo, shi))
            if not frags:
                continue
            g_l = [b.grad_shard[lo:hi] for b, _, lo, hi in frags]
            p_l = [b.master[lo:hi] for b, _, lo, hi in frags]
            m_l = [b.exp_avg[lo:hi] for b, _, lo, hi in frags]
            v_l = [b.exp_avg_sq[lo:hi] for b, _, lo, hi in frags]
            u_l = [b.update[lo:hi] for b, _, lo, hi in frags]
            decay = torch.full([len(frags)], group["weight_decay"] if self.adam_w_mode else 0.0,
                               dtype=torch.float32, device=dev)
            # 2. stage 1: moments + update (clipping by max_grad_norm inside)
            multi_tensor_applier(amp_C.multi_tensor_lamb_stage1_cuda, flag, [g_l, p_l, m_l, v_l, u_l], decay,
                                 step, beta1, beta2, group["eps"], gnorm,
                                 max_norm if max_norm > 0 else float("inf"))
            # 3. per-parameter norms across shards
            _, pn = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [p_l], True)
            _, un = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [u_l], True)
            idx = torch.tensor([self._param_index[id(p)] for _, p, _, _ in frags], dtype=torch.long, device=dev)
            sums = torch.zeros(2, self._n_params, dtype=torch.float32, device=dev)
            sums[0].index_add_(0, idx, pn.float() ** 2)
            sums[1].index_add_(0, idx, un.float() ** 2)
            dist.all_reduce(sums, group=self.distributed_process_group)
            norms = sums.sqrt()
            # 4. stage 2 with the global per-parameter norms expanded per fragment
            multi_tensor_applier(amp_C.multi_tensor_lamb_stage2_cuda, flag, [p_l, u_l], norms[0][idx],
                                 norms[1][idx], group["lr"], group["weight_decay"], self.use_nvlamb)
        # refresh parameters
        works = []
        for b in self._buckets:
            b.param_sync_shard.copy_(b.master)
            if self.distributed_size == 1:
                b.param_sync_full.copy_(b.param_sync_shard)
            else:
                works.append(dist.all_gather_into_tensor(b.param_sync_full, b.param_sync_shard,
                                                         group=self.distributed_process_group, async_op=True))
        for w in works:
            w.wait()
        for b in self._buckets:
            if b.param_sync_full is not b.param_buffer:
                b.param_buffer.copy_(b.param_sync_full)
        self._grad_norm = None
        return loss
