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
    returns False before launching anything, the optimizer creates that state and retries)."""

    _table = None
    _table_sig = None
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

    def _fast_path_ok(self):
        if not self.native_table:
            return False
        buf = getattr(self, "_dummy_overflow_buf", None)
        if buf is None or not buf.is_cuda:
            return False
        from .._native import available

        return available()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._table = None

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._table = None
