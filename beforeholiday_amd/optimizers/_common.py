"""Shared plumbing for the fused optimizers."""
from __future__ import annotations

import torch


def noop_buffer(device) -> torch.Tensor:
    return torch.zeros(1, dtype=torch.int, device=device)


def first_device(param_groups):
    for g in param_groups:
        for p in g["params"]:
            return p.device
    return torch.device("cpu")


def grad_like_param(p: torch.Tensor) -> torch.Tensor:
    """The gradient laid out exactly like its parameter (the kernels walk raw memory).

    Reference: the channels_last handling in apex/optimizers/fused_sgd.py:166-199.
    """
    g = p.grad
    if g.stride() == p.stride() or p.numel() <= 1:
        return g
    for fmt in (torch.contiguous_format, torch.channels_last, torch.channels_last_3d):
        try:
            if p.is_contiguous(memory_format=fmt):
                return g.contiguous(memory_format=fmt)
        except RuntimeError:
            continue
    raise RuntimeError("fused optimizers support contiguous / channels_last parameters only")


def zero_param_grads(params, set_to_none: bool):
    """``p.grad = None`` or zero-fill (one foreach launch), the torch.optim way: ``detach_()`` only a
    gradient that has a ``grad_fn``. A gradient that is a VIEW (DDP's gradient-as-bucket-view slots)
    cannot be detached in place, and does not need it: ``requires_grad_(False)`` is enough."""
    grads = []
    for p in params:
        if p.grad is None:
            continue
        if set_to_none:
            p.grad = None
            continue
        if p.grad.grad_fn is not None:
            p.grad.detach_()
        else:
            p.grad.requires_grad_(False)
        grads.append(p.grad)
    if grads:
        torch._foreach_zero_(grads)


def zero_grad(opt, set_grad_none: bool, set_to_none=None):
    none = set_grad_none if set_to_none is None else set_to_none
    zero_param_grads([p for group in opt.param_groups for p in group["params"]], none)


class ParamTableMixin:
    """Host fast path of the fused optimizers: the parameters and their state tensors are registered
    once in a native ``amp_C.ParamTable`` and a step is ONE call that reads the gradients in C++
    (see csrc/bindings/mta.cpp). The table is rebuilt when the param groups change, after
    ``load_state_dict`` / ``add_param_group``, and when a parameter gets its first gradient (the step
    returns False before launching anything, the optimizer creates that state and retries).

    Under amp O2 / O5 a second table (``_amp_native_table``) pairs every fp32 master (the optimizer's
    parameter, owner of the state) with its 16-bit model parameter: the step reads the model
    parameter's (still loss-scaled) gradient and writes the model parameter back in the same launch
    (amp/_process_optimizer.py, ``_MasterPlan`` fused path)."""

    _table = None
    _table_sig = None
    _amp_table = None
    _amp_table_sig = None
    native_table = True  # False: always the per-step tensor-list path (kept for A/B tests)

    def _table_signature(self):
        return tuple((id(g["params"]), len(g["params"])) for g in self.param_groups)

    def _native_table(self, state_keys, master=None):
        sig = self._table_signature()
        if self._table is not None and self._table_sig == sig:
            return self._table
        from .._native import submodule

        table = submodule("amp_C").ParamTable()
        for g in self.param_groups:
            sts = [self.state.get(p) or {} for p in g["params"]]
            s0 = [st.get(state_keys[0]) for st in sts]
            s1 = [st.get(state_keys[1]) for st in sts]
            m = [st.get(master) for st in sts] if master else []
            table.add_group(list(g["params"]), s0, s1, m)
        self._table, self._table_sig = table, sig
        return table

    def _amp_native_table(self, state_keys, models):
        """``models``: {id(fp32 master): 16-bit model parameter}. Entries whose parameter is not a
        master (amp's fp32-from-fp32 parameters) are plain entries."""
        sig = (self._table_signature(), len(models))
        if self._amp_table is not None and self._amp_table_sig == sig:
            return self._amp_table
        from .._native import submodule

        table = submodule("amp_C").ParamTable()
        for g in self.param_groups:
            sts = [self.state.get(p) or {} for p in g["params"]]
            table.add_group([models.get(id(p), p) for p in g["params"]],
                            [st.get(state_keys[0]) for st in sts], [st.get(state_keys[1]) for st in sts],
                            [p if id(p) in models else None for p in g["params"]])
        self._amp_table, self._amp_table_sig = table, sig
        return table

    def _reset_tables(self):
        self._table = None
        self._amp_table = None

    def _device_step_counters(self):
        """amp's device-resident loss scale: the noop flag may skip a step on the device, so the step
        counters the bias corrections use advance on the device only when it does not (None when the
        host counters are exact)."""
        if not getattr(self, "_device_step", False):
            return None
        steps = getattr(self, "_device_steps", None)
        if steps is None or steps.numel() != len(self.param_groups):
            steps = self._device_steps = torch.tensor([g["step"] - 1 for g in self.param_groups], dtype=torch.int32,
                                                      device=self._dummy_overflow_buf.device)
        steps.add_((self._dummy_overflow_buf == 0).to(torch.int32))
        return steps

    def _fast_path_ok(self):
        if not self.native_table:
            return False
        buf = getattr(self, "_dummy_overflow_buf", None)
        if buf is None or not buf.is_cuda:
            return False
        from .._native import available

        return available()

    def state_dict(self):
        steps = getattr(self, "_device_steps", None)
        if steps is not None:  # the device counters are the real step counts (skipped steps excluded)
            for g, st in zip(self.param_groups, steps.tolist()):
                g["step"] = int(st)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._reset_tables()
        self._device_steps = None  # re-seeded from the loaded host counters

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._reset_tables()
