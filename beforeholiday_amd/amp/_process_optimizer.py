"""How ``amp.initialize`` rewires an optimizer (behaviour: apex/amp/_process_optimizer.py:28-489).

The optimizer gets an ``_amp_stash`` (the state the rest of amp and the fused optimizers read:
``fp16_groups`` / ``fp32_from_fp16_groups`` / ``all_fp32_from_fp16_params`` / ``params_have_scaled_gradients``)
and a :class:`_GradPlan` that implements the three moments of a mixed-precision step:

* ``prepare`` (entering ``scale_loss``): gradients already sitting on the parameters are moved aside
  (stashed) so this backward writes fresh, scaled ones;
* ``finish`` (leaving ``scale_loss``): the fresh gradients are unscaled -- 16-bit model gradients
  straight into the fp32 master gradients, one multi-tensor launch per dtype pair -- and added to
  the stashed ones where a previous micro-batch left some (gradient accumulation);
* after ``optimizer.step()`` the fp32 masters are copied back into the 16-bit model parameters (one
  launch per dtype; FusedSGD writes them inside its own kernel).

Fused mixed-precision step (O2 / O5 with FusedLAMB or FusedAdam on the GPU): ``finish`` leaves the
scaled 16-bit gradients where they are -- under a dynamic scale it only runs the norm of them, which
sets the overflow flag and is the scaled global norm LAMB needs -- and ``optimizer.step()`` runs ONE
native call whose kernels read those gradients times the device inverse scale, update the fp32
masters and write the 16-bit model parameters (the reference's mixed-precision LAMB,
csrc/multi_tensor_lamb_mp.cu:41,248,367; FusedSGD's 4-list copy, apex/optimizers/fused_sgd.py:245-252).
Neither the fp32 master gradients nor the separate master-to-model pass exist on that path. Anything
that needs the master gradients before the step (``amp.master_params``, a second ``scale_loss``
accumulating into the same step) materialises them first, so the unfused semantics are kept. The
path is OPT-IN (``Config.amp_fused_master_step``; the benchmarks turn it on): while a fused step is
pending the masters reachable through ``optimizer.param_groups`` have ``.grad is None``, so gradient
clipping or inspection must go through ``amp.master_params(optimizer)``, which materialises them.

Three plans: :class:`_MasterPlan` (O2 / O5: fp32 master copies replace the 16-bit parameters inside
the optimizer), :class:`_FusedSGDMasterPlan` (FusedSGD folds the unscale into its kernel unless
``materialize_master_grads``) and :class:`_ModelPlan` (O1 / O4 / O0: the model parameters are the
masters).
"""
from __future__ import annotations

import types

import torch

from .. import config as _config
from ..multi_tensor_apply import multi_tensor_applier, multi_tensor_applier_l2norm
from ..ops import amp_C

_LOW = (torch.float16, torch.bfloat16)

# the fused mixed-precision step (module docstring; Config.amp_fused_master_step, opt-in); False (the
# default) keeps the reference's unscale + step + copy sequence, so the fp32 master gradients are
# populated in optimizer.param_groups after scale_loss exits
fused_master_step = False


def _apply_config(c):
    global fused_master_step
    fused_master_step = c.amp_fused_master_step


_config.on_change(_apply_config)


class AmpOptimizerState(object):
    pass


def _check_param_type(param):
    if param.dtype in _LOW or param.dtype == torch.float32:
        return
    raise TypeError("Optimizer's parameters must be one of float32, float16, bfloat16. Received {}"
                    .format(param.type()))


def _by_dtype(pairs):
    """{(dtype_a, dtype_b): ([a...], [b...])} so every multi-tensor launch sees one dtype per list."""
    out = {}
    for a, b in pairs:
        lists = out.setdefault((a.dtype, b.dtype), ([], []))
        lists[0].append(a)
        lists[1].append(b)
    return out


def _unscale_into_models(scaler, params, stash, scale_override=None):
    """Unscale the gradients of ``params`` in place (the parameters are their own masters) and fold
    in the stashed gradients of an earlier micro-batch; clears ``stash``."""
    fresh, accum, old = [], [], []
    for i, p in enumerate(params):
        s = stash[i]
        if p.grad is None:
            if s is not None:
                p.grad = s  # no new gradient this pass: keep the accumulated one
        elif s is None:
            fresh.append(p.grad)
        else:
            accum.append(p.grad)
            old.append(s)
        stash[i] = None
    if getattr(scaler, "device_mode", False) and scale_override is None:
        # device-resident scale: unscale and accumulate on the device reciprocal (no host read)
        if fresh:
            scaler.unscale(fresh, fresh, None, models_are_masters=True)
        if accum:
            scaler.unscale_with_stashed(accum, old, accum)
        return
    if scale_override is None:
        if scaler.loss_scale() == 1.0 and not scaler.dynamic:
            if accum:  # static scale 1: plain accumulation
                torch._foreach_add_(accum, old)
            return
        grads_have, stashed_have, out_scale = scaler.loss_scale(), 1.0, 1.0
    else:
        grads_have, stashed_have, out_scale = scale_override
    if fresh:
        scaler.unscale(fresh, fresh, None, models_are_masters=True, scale_override=grads_have / out_scale)
    if accum:
        scaler.unscale_with_stashed(accum, old, accum, scale_override=(grads_have, stashed_have, out_scale))


def _keep(p):
    """``p.grad`` to set aside across the next backward. A DDP gradient-as-bucket-view gradient lives in
    the bucket buffer that the next backward overwrites (parallel/distributed.py), so it is cloned."""
    from ..parallel.distributed import grad_is_bucket_view

    return p.grad.clone() if grad_is_bucket_view(p) else p.grad


class _GradPlan(object):
    def __init__(self, opt):
        self.opt = opt
        self.stash = opt._amp_stash
        self.ready = False

    def ensure(self):
        if not self.ready:
            self.setup()
            self.ready = True
            self.stash.lazy_init_called = True

    def setup(self):
        raise NotImplementedError

    def prepare(self):
        raise NotImplementedError

    def finish(self, scaler):
        raise NotImplementedError

    def add_group(self, group):
        raise NotImplementedError


class _ModelPlan(_GradPlan):
    """The model parameters are the masters (no fp32 copies)."""

    def setup(self):
        st = self.stash
        st.all_fp16_params, st.all_fp32_params = [], []
        for group in self.opt.param_groups:
            for p in group["params"]:
                self.add_param(p)

    def add_param(self, p):
        st = self.stash
        _check_param_type(p)
        (st.all_fp16_params if p.dtype in _LOW else st.all_fp32_params).append(p)

    def _lists(self):
        st = self.stash
        st.all_fp16_grad_stash = getattr(st, "all_fp16_grad_stash", [])
        st.all_fp32_grad_stash = getattr(st, "all_fp32_grad_stash", [])
        for name, params in (("all_fp16_grad_stash", st.all_fp16_params), ("all_fp32_grad_stash", st.all_fp32_params)):
            lst = getattr(st, name)
            lst.extend([None] * (len(params) - len(lst)))
        return ((st.all_fp16_params, st.all_fp16_grad_stash), (st.all_fp32_params, st.all_fp32_grad_stash))

    def prepare(self):
        self.ensure()
        for params, stash in self._lists():
            for i, p in enumerate(params):
                stash[i], p.grad = _keep(p), None

    def finish(self, scaler):
        self.ensure()
        for params, stash in self._lists():
            _unscale_into_models(scaler, params, stash)

    def add_group(self, group):
        self.ensure()
        for p in group["params"]:
            self.add_param(p)
        self._lists()


class _MasterPlan(_GradPlan):
    """16-bit model parameters train through fp32 master copies that replace them in the optimizer."""

    def setup(self):
        st = self.stash
        st.fp16_groups, st.fp32_from_fp16_groups, st.fp32_from_fp32_groups = [], [], []
        st.all_fp16_params, st.all_fp32_from_fp16_params, st.all_fp32_from_fp32_params = [], [], []
        st.all_fp32_from_fp32_grad_stash = []
        for group in self.opt.param_groups:
            self._split(group, move_state=True)
        # optimizer state (e.g. torch.optim momentum) is re-keyed to the masters
        self.opt.load_state_dict(self.opt.state_dict())

    def _split(self, group, move_state=False):
        """Swap the 16-bit parameters of ``group`` for fp32 masters and record both sides."""
        st = self.stash
        low, masters, fp32 = [], [], []
        params = group["params"]
        for i, p in enumerate(params):
            if not p.requires_grad:
                continue
            _check_param_type(p)
            if p.dtype in _LOW:
                master = p.detach().clone().float()
                master.requires_grad = True
                params[i] = master
                if move_state and p in self.opt.state:
                    self.opt.state[master] = self.opt.state.pop(p)
                low.append(p)
                masters.append(master)
            else:
                fp32.append(p)
        st.fp16_groups.append(low)
        st.fp32_from_fp16_groups.append(masters)
        st.fp32_from_fp32_groups.append(fp32)
        st.all_fp16_params += low
        st.all_fp32_from_fp16_params += masters
        st.all_fp32_from_fp32_params += fp32
        st.all_fp32_from_fp32_grad_stash += [None] * len(fp32)
        for p in masters + fp32:
            p.grad = None

    _fused = None  # (inverse scale tensor or None, scaled norm or None) while a fused step is pending
    _inv = None
    _inv_of = None
    _models = None

    def prepare(self):
        self.ensure()
        st = self.stash
        if self._fused is not None:  # a second backward before the step: accumulate the unfused way
            self.materialize()
        for p in st.all_fp16_params:  # 16-bit grads are folded into the fp32 master grads: drop them
            p.grad = None
        for i, p in enumerate(st.all_fp32_from_fp32_params):
            st.all_fp32_from_fp32_grad_stash[i], p.grad = _keep(p), None

    # ---- fused mixed-precision step
    def _fused_wanted(self, scaler):
        from .scaler import LossScaler

        ok = getattr(self.opt, "_amp_fused_ok", None)
        return (fused_master_step and ok is not None and LossScaler.has_fused_kernel and ok()
                and all(m.grad is None for m in self.stash.all_fp32_from_fp16_params))

    def _inverse_scale(self, scaler, dev):
        """A one-element device tensor holding 1/scale of this backward (None for a static scale of 1).
        Plan-owned, so the scale update between ``finish`` and the step cannot change it."""
        if scaler.device_mode:
            if self._inv is None or self._inv.device != dev:
                self._inv = torch.empty(1, dtype=torch.float32, device=dev)
            torch.reciprocal(scaler._scale_dev, out=self._inv)
            self._inv_of = None
            return self._inv
        scale = float(scaler.loss_scale())
        if scale == 1.0:
            return None
        if self._inv is None or self._inv.device != dev or self._inv_of != scale:
            self._inv = torch.full((1,), 1.0 / scale, dtype=torch.float32, device=dev)
            self._inv_of = scale
        return self._inv

    def _start_fused(self, scaler, grads):
        inv = self._inverse_scale(scaler, grads[0].device)
        norm = None
        if scaler.dynamic:
            # the overflow check: a non-finite partial sum sets the flag update_scale reads; the value
            # is the norm of the scaled gradients, which LAMB's global norm reuses
            flag = scaler._overflow_buf if scaler.device_mode else scaler._flag_for(grads)
            by_dt = {}
            for g in grads:
                by_dt.setdefault(g.dtype, []).append(g)
            norms = [multi_tensor_applier_l2norm(amp_C.multi_tensor_l2norm, flag, [gl], False)[0]
                     for gl in by_dt.values()]
            norm = norms[0] if len(norms) == 1 else multi_tensor_applier_l2norm(
                amp_C.multi_tensor_l2norm, flag, [norms], False)[0]
        self._fused = (inv, norm)

    def fused_pending(self):
        return self._fused is not None

    def discard(self):
        """The pending fused step is dropped (skipped overflow step, zero_grad)."""
        self._fused = None

    def materialize(self):
        """Turn a pending fused step back into fp32 master gradients (the unfused state)."""
        if self._fused is None:
            return
        inv, _ = self._fused
        self._fused = None
        st = self.stash
        pairs = []
        for low, master in zip(st.all_fp16_params, st.all_fp32_from_fp16_params):
            if low.grad is not None:
                master.grad = torch.empty_like(master)
                pairs.append((low.grad, master.grad))
        for ins, outs in _by_dtype(pairs).values():
            multi_tensor_applier(amp_C.multi_tensor_scale, st.dummy_overflow_buf, [ins, outs],
                                 inv if inv is not None else 1.0)

    def fused_step(self):
        inv, norm = self._fused
        self._fused = None
        st = self.stash
        if self._models is None or len(self._models) != len(st.all_fp16_params):
            self._models = {id(m): p for m, p in zip(st.all_fp32_from_fp16_params, st.all_fp16_params)}
        with torch.no_grad():
            self.opt._amp_fused_step(self._models, inv, norm)

    def finish(self, scaler):
        self.ensure()
        st = self.stash
        if self._fused is None and self._fused_wanted(scaler):
            grads = [p.grad for p in st.all_fp16_params if p.grad is not None]
            if grads:
                self._start_fused(scaler, grads)
                _unscale_into_models(scaler, st.all_fp32_from_fp32_params, st.all_fp32_from_fp32_grad_stash)
                return
        self.materialize()
        new_pairs, acc_pairs = [], []
        for low, master in zip(st.all_fp16_params, st.all_fp32_from_fp16_params):
            if low.grad is None:
                continue  # nothing new; a master grad from an earlier micro-batch stays as it is
            if master.grad is None:
                master.grad = torch.empty_like(master)
                new_pairs.append((low.grad, master.grad))
            else:
                acc_pairs.append((low.grad, master.grad))
        if new_pairs:
            scaler.unscale([a for a, _ in new_pairs], [b for _, b in new_pairs], None, models_are_masters=False)
        if acc_pairs:
            acc = [b for _, b in acc_pairs]
            scaler.unscale_with_stashed([a for a, _ in acc_pairs], acc, acc)
        _unscale_into_models(scaler, st.all_fp32_from_fp32_params, st.all_fp32_from_fp32_grad_stash)

    def masters_to_model(self):
        st = self.stash
        if not st.all_fp16_params:
            return
        for masters, models in _by_dtype(zip((m.data for m in st.all_fp32_from_fp16_params),
                                             (p.data for p in st.all_fp16_params))).values():
            multi_tensor_applier(amp_C.multi_tensor_scale, st.dummy_overflow_buf, [masters, models], 1.0)

    def zero_grad(self, set_to_none=True):
        # set_to_none=True by default (PyTorch >= 2.0 semantics): the next prepare() drops / stashes these
        # grads anyway, so zero-filling them would only add one fill kernel per parameter plus a
        # stashed-gradient axpby pass after backward. set_to_none=False keeps the reference's zeroing.
        from ..optimizers._common import zero_param_grads

        self.ensure()
        st = self.stash
        self.discard()
        zero_param_grads(st.all_fp16_params + st.all_fp32_from_fp32_params, set_to_none)
        for p in st.all_fp32_from_fp16_params:
            p.grad = None

    def add_group(self, group):
        self.ensure()
        self._split(group)


class _FusedSGDMasterPlan(_MasterPlan):
    """FusedSGD reads the scaled 16-bit gradients itself (``materialize_master_grads=False``): they are
    stashed and unscaled in place with the scale bookkeeping FusedSGD expects (``most_recent_scale``)."""

    def prepare(self):
        if self.opt.materialize_master_grads:
            return super().prepare()
        self.ensure()
        st = self.stash
        st.all_fp16_grad_stash = getattr(st, "all_fp16_grad_stash", [])
        st.all_fp16_grad_stash.extend([None] * (len(st.all_fp16_params) - len(st.all_fp16_grad_stash)))
        for i, p in enumerate(st.all_fp16_params):
            st.all_fp16_grad_stash[i], p.grad = _keep(p), None
        for i, p in enumerate(st.all_fp32_from_fp32_params):
            st.all_fp32_from_fp32_grad_stash[i], p.grad = _keep(p), None

    def finish(self, scaler):
        opt = self.opt
        if opt.materialize_master_grads:
            return super().finish(scaler)
        self.ensure()
        st = self.stash
        now = scaler.loss_scale()
        out_scale = min(now, opt.most_recent_scale) if opt.scale_set_by_backward else now
        override = (now, opt.most_recent_scale, out_scale)
        _unscale_into_models(scaler, st.all_fp16_params, st.all_fp16_grad_stash, override)
        _unscale_into_models(scaler, st.all_fp32_from_fp32_params, st.all_fp32_from_fp32_grad_stash, override)
        opt.most_recent_scale = out_scale
        opt.scale_set_by_backward = True


def _process_optimizer(optimizer, properties):
    from ..optimizers import FusedSGD

    if hasattr(optimizer, "_amp_stash"):
        raise RuntimeError("A given optimizer should only be passed through amp.initialize once.")
    for name in ("_lazy_init_maybe_master_weights", "_master_params_to_model_params", "_prepare_amp_backward",
                 "_post_amp_backward", "_amp_lazy_init"):
        if hasattr(optimizer, name):
            raise RuntimeError("Incoming optimizer already has {} defined.".format(name))
    st = optimizer._amp_stash = AmpOptimizerState()
    st.lazy_init_called = False
    st.params_have_scaled_gradients = False
    st.multi_tensor_scale = amp_C.multi_tensor_scale
    st.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
    dev = next((p.device for g in optimizer.param_groups for p in g["params"]), None)
    st.dummy_overflow_buf = torch.zeros(1, dtype=torch.int, device=dev or "cpu")

    fused_sgd = isinstance(optimizer, FusedSGD)
    if properties.master_weights:
        plan = (_FusedSGDMasterPlan if fused_sgd else _MasterPlan)(optimizer)
        inner_step = optimizer.step

        def step(self, closure=None):
            if closure is not None:
                raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
            if plan.fused_pending():  # one native call: unscale + update + 16-bit write
                out = plan.fused_step()
            else:
                out = inner_step()
                if not fused_sgd:  # FusedSGD writes the 16-bit params inside its kernel
                    plan.masters_to_model()
            for p in self._amp_stash.all_fp32_from_fp16_params:
                p.grad = None
            return out

        optimizer.step = types.MethodType(step, optimizer)
        optimizer.zero_grad = types.MethodType(lambda self, set_to_none=True: plan.zero_grad(set_to_none), optimizer)
        optimizer._master_params_to_model_params = types.MethodType(lambda self: plan.masters_to_model(), optimizer)
    else:
        plan = _ModelPlan(optimizer)
    st.plan = plan
    optimizer._lazy_init_maybe_master_weights = types.MethodType(lambda self: plan.setup(), optimizer)
    optimizer._amp_lazy_init = types.MethodType(lambda self: plan.ensure(), optimizer)
    optimizer._prepare_amp_backward = types.MethodType(lambda self: plan.prepare(), optimizer)
    optimizer._post_amp_backward = types.MethodType(lambda self, scaler: plan.finish(scaler), optimizer)

    inner_add = optimizer.add_param_group

    def add_param_group(self, new_group):
        assert isinstance(new_group, dict), "param group must be a dict"
        params = new_group["params"]
        if isinstance(params, torch.Tensor):
            new_group["params"] = [params]
        elif isinstance(params, set):
            raise TypeError("optimizer parameters need to be organized in ordered collections, but the ordering "
                            "of tensors in sets will change between runs. Please use a list instead.")
        else:
            new_group["params"] = list(params)
        plan.add_group(new_group)
        inner_add(new_group)

    optimizer.add_param_group = types.MethodType(add_param_group, optimizer)
    return optimizer
