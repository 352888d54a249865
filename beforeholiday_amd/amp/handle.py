"""scale_loss / disable_casts / AmpHandle (reference: apex/amp/handle.py:16-281)."""
from __future__ import annotations

import contextlib

import torch

from ._amp_state import _amp_state, maybe_print
from .scaler import LossScaler


def _device_scaler_wanted(loss_scaler, optimizers):
    """Config.amp_device_scaler (BH_AMP_DEVICE_SCALER=1), dynamic scaling, the fused unscale kernel, a CUDA loss, and only fused
    optimizers whose kernels return early on a set noop flag (``_dummy_overflow_buf``): FusedLAMB
    (both stages), FusedSGD and FusedAdam (table path)."""
    from .. import config
    from ..optimizers import FusedAdam, FusedLAMB, FusedSGD

    def flag_aware(o):
        if isinstance(o, FusedAdam):  # the native table path reads the flag; capturable has its own scaler API
            return not o.capturable and not o.master_weights
        return isinstance(o, (FusedLAMB, FusedSGD))

    return (config.get().amp_device_scaler and loss_scaler.dynamic
            and LossScaler.has_fused_kernel and torch.cuda.is_available()
            and all(flag_aware(o) and hasattr(o, "_dummy_overflow_buf") for o in optimizers))


class _StepGate(object):
    """Installed once per optimizer as ``optimizer.step`` by :func:`scale_loss` (reference behaviour:
    apex/amp/handle.py:128-154, which re-patches ``step`` on every overflow instead).

    * host-scaled: an overflowing backward sets ``pending_skip`` (the message to print); the next call
      then drops the step -- fp32 master grads are released and FusedSGD's scale bookkeeping reset --
      and clears the mark;
    * device-scaled: the step always runs (its fused kernels read the step-level overflow flag and
      return early on their own), then that flag is cleared for the next accumulation window.
    """

    def __init__(self, optimizer, inner):
        self.optimizer = optimizer
        self.inner = inner
        self.pending_skip = None
        self.device_flag = None

    def __call__(self, closure=None):
        if closure is not None:
            raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
        if self.pending_skip is not None:
            maybe_print(self.pending_skip)
            self.pending_skip = None
            opt = self.optimizer
            for p in getattr(opt._amp_stash, "all_fp32_from_fp16_params", ()):
                p.grad = None
            plan = getattr(opt._amp_stash, "plan", None)
            if plan is not None and hasattr(plan, "discard"):
                plan.discard()
            if hasattr(opt, "most_recent_scale"):
                opt.most_recent_scale = 1.0
                opt.scale_set_by_backward = False
            return None
        out = self.inner()
        if self.device_flag is not None:
            self.device_flag.zero_()
        return out


def _gated_step(self, closure=None):
    return self._amp_stash.step_gate(closure)


def _gate(optimizer):
    """The optimizer's :class:`_StepGate`, installed on first use. ``optimizer.step`` becomes a bound
    method (``types.MethodType``), not the gate object itself: torch's LR schedulers wrap
    ``optimizer.step`` through its ``__func__`` (``patch_track_step_called``), so a scheduler built
    after the first ``scale_loss`` still works."""
    import types

    stash = optimizer._amp_stash
    gate = getattr(stash, "step_gate", None)
    if gate is None:
        gate = stash.step_gate = _StepGate(optimizer, optimizer.step)
        optimizer.step = types.MethodType(_gated_step, optimizer)
    return gate


@contextlib.contextmanager
def scale_loss(loss, optimizers, loss_id=0, model=None, delay_unscale=False, delay_overflow_check=False):
    """Yields ``loss.float() * loss_scale``; on exit unscales gradients (fp16 -> fp32 master grads
    under master weights), checks for Inf/NaN and, on overflow, lowers the scale and makes the next
    ``optimizer.step()`` a no-op (host scale: skipped by the step gate; device scale: the fused
    kernels see the step-level flag)."""
    from ..parallel.LARC import LARC

    props = getattr(_amp_state, "opt_properties", None)
    if props is None or not props.enabled:
        yield loss
        return
    if isinstance(optimizers, (torch.optim.Optimizer, LARC)):
        optimizers = [optimizers]
    scaler = _amp_state.loss_scalers[loss_id]
    if not scaler.device_mode and _device_scaler_wanted(scaler, optimizers):
        scaler.enable_device_mode(loss.device)
    if scaler.device_mode:
        for opt in optimizers:
            opt._dummy_overflow_buf = scaler._step_flag
            opt._device_step = True  # FusedLAMB: step counters advance on the device, unless skipped
            _gate(opt).device_flag = scaler._step_flag
    factor = scaler.scale_for_loss()

    trivial = not props.master_weights and not scaler.dynamic and not scaler.device_mode and factor == 1.0
    if not trivial and not delay_unscale:
        for opt in optimizers:
            if not opt._amp_stash.params_have_scaled_gradients:
                opt._prepare_amp_backward()

    yield loss.float() if trivial else loss.float() * factor

    if not trivial:
        if delay_unscale:
            for opt in optimizers:
                opt._amp_stash.params_have_scaled_gradients = True
        else:
            scaler.clear_overflow_state()  # this pass's flag only
            for opt in optimizers:
                opt._post_amp_backward(scaler)
                opt._amp_stash.params_have_scaled_gradients = False
            if scaler.device_mode and not delay_overflow_check:
                should_skip = scaler.fold_and_update_device()
            else:
                if scaler.device_mode:
                    scaler.fold_pass_into_step()
                should_skip = not delay_overflow_check and scaler.update_scale()
            if should_skip:
                msg = "Gradient overflow.  Skipping step, loss scaler {} reducing loss scale to {}".format(
                    loss_id, scaler.loss_scale())
                for opt in optimizers:
                    _gate(opt).pending_skip = msg
    if props.patch_torch_functions and _amp_state.handle is not None:
        _amp_state.handle._clear_cache()


@contextlib.contextmanager
def disable_casts():
    """Temporarily turn the O1/O4 cast wrappers off (e.g. around the optimizer step)."""
    h = _amp_state.handle
    if h is None:
        yield
        return
    prev = h._is_active
    h._is_active = False
    try:
        yield
    finally:
        h._is_active = prev


class _Handle(object):
    """State of the O1 / O4 function patching that the cast wrappers (amp/wrap.py) consult on every
    call: whether casting is on, the per-iteration cache of 16-bit weight copies, and the list of
    (module, name, original) patches needed to undo it.

    :class:`AmpHandle` is the live one ``amp.init()`` returns; :class:`NoOpHandle` backs the
    ``amp.half_function``-style decorators while amp is off (never casts). The old per-optimizer
    ``scale_loss`` API of these handles is gone (as in the reference): it raises, pointing to
    ``amp.initialize`` / ``amp.scale_loss``."""

    casting = False
    caching = False

    def __init__(self, verbose=False):
        self._verbose = bool(verbose)
        self._cache = {}
        self._patches = []
        self._is_active = self.casting

    # -- queried by the cast wrappers
    def is_active(self):
        return self._is_active

    @property
    def verbose(self):
        return self._verbose

    @property
    def has_cache(self):
        return self.caching

    @property
    def cache(self):
        return self._cache

    def remove_cache(self, param):
        self._cache.pop(param, None)

    def _clear_cache(self):
        self._cache.clear()

    @contextlib.contextmanager
    def _disable_casts(self):
        prev, self._is_active = self._is_active, False
        try:
            yield
        finally:
            self._is_active = prev

    # -- patch bookkeeping (amp/utils.py records every replaced function here)
    def _save_func(self, mod, fn, func):
        self._patches.append((mod, fn, func))

    def _deactivate(self):
        while self._patches:  # newest first: nested patches of one attribute unwind correctly
            mod, fn, func = self._patches.pop()
            setattr(mod, fn, func)

    # -- legacy optimizer API
    def wrap_optimizer(self, optimizer, num_loss=1):
        from .opt import OptimWrapper

        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        if not self.casting:
            yield loss
            return
        raise RuntimeError("handle.scale_loss (the pre-amp.initialize API) is not supported: use "
                           "amp.initialize(model, optimizer, opt_level=...) and amp.scale_loss(loss, optimizer)")


class AmpHandle(_Handle):
    """Returned by ``amp.init()``: casting on, weight-cast cache on unless ``enable_caching=False``."""

    casting = True

    def __init__(self, loss_scale="dynamic", enable_caching=True, verbose=False):
        self.caching = bool(enable_caching)
        super().__init__(verbose)
        self.loss_scale = loss_scale


class NoOpHandle(_Handle):
    """Handle of the decorators while amp is not initialised: never casts, nothing to undo."""
