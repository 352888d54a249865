"""Model-parallel-aware GradScaler (reference: apex/transformer/amp/grad_scaler.py:21-119).

A rank that sees inf/nan in its shard of the gradients must make every TP/PP rank skip the step and
back off the scale together, so ``found_inf`` is MAX-all-reduced over the model-parallel group. All
per-device flags are stacked into ONE tensor and reduced with ONE collective (the reference issues one
all-reduce per flag) and the step decision costs a single host sync.
"""
from collections import defaultdict

import torch

from .. import parallel_state


class GradScaler(torch.amp.GradScaler):
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True, device="cuda"):
        super().__init__(device, init_scale=init_scale, growth_factor=growth_factor, backoff_factor=backoff_factor,
                         growth_interval=growth_interval, enabled=enabled)

    @staticmethod
    def _mp_max(flags):
        found = torch.stack([f.reshape(()).float() for f in flags]).amax().reshape(1)
        torch.distributed.all_reduce(found, op=torch.distributed.ReduceOp.MAX,
                                     group=parallel_state.get_model_parallel_group())
        return found

    def _maybe_opt_step(self, optimizer, optimizer_state, *args, **kwargs):
        found = self._mp_max(list(optimizer_state["found_inf_per_device"].values()))
        if found.item() == 0:
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale=None):
        if not self._enabled:
            return
        _scale, _growth_tracker = self._check_scale_growth_tracker("update")
        if new_scale is not None:
            if isinstance(new_scale, float):
                self._scale.fill_(new_scale)
            else:
                reason = "new_scale should be a float or a 1-element tensor with requires_grad=False."
                assert isinstance(new_scale, torch.Tensor) and new_scale.numel() == 1, reason
                assert new_scale.requires_grad is False, reason
                self._scale.copy_(new_scale)
        else:
            found_infs = [f.to(device=_scale.device, non_blocking=True)
                          for state in self._per_optimizer_states.values()
                          for f in state["found_inf_per_device"].values()]
            assert len(found_infs) > 0, "No inf checks were recorded prior to update."
            found = self._mp_max(found_infs)
            torch._amp_update_scale_(_scale, _growth_tracker, found, self._growth_factor, self._backoff_factor,
                                     self._growth_interval)
        self._per_optimizer_states = defaultdict(torch.amp.grad_scaler._refresh_per_optimizer_state)
