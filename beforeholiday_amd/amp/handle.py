"""scale_loss / disable_casts / AmpHandle (reference: apex/amp/handle.py:16-281)."""
from __future__ import annotations

import contextlib

import torch

from ._amp_state import _amp_state, maybe_print
from .scaler import LossScaler


def _device_scaler_wanted(loss_scaler, optimizers):
    """BH_AMP_DEVICE_SCALER=1, dynamic scaling, the fused unscale kernel, a CUDA loss, and only fused
    optimizers whose kernels return early on a set noop flag (``_dummy_overflow_buf``): FusedLAMB
    (both stages) and FusedSGD."""
    import os

    from ..optimizers import FusedLAMB, FusedSGD

    return (os.environ.get("BH_AMP_DEVICE_SCALER", "0") == "1" and loss_scaler.dynamic
            and LossScaler.has_fused_kernel and torch.cuda.is_available()
            and all(isinstance(o, (FusedLAMB, FusedSGD)) and hasattr(o, "_dummy_overflow_buf")
                    for o in optimizers))


@contextlib.contextmanager
def scale_loss(loss, optimizers, loss_id=0, model=None, delay_unscale=False, delay_overflow_check=False):
    """Yields ``loss.float() * loss_scale``; on exit unscales gradients (fp16 -> fp32 master grads
    under master weights), checks for Inf/NaN and, on overflow, reduces the scale and arms a
    one-shot skip of ``optimizer.step()``."""
    from ..parallel.LARC import LARC

    if not hasattr(_amp_state, "opt_properties") or _amp_state.opt_properties is None or \
            not _amp_state.opt_properties.enabled:
        yield loss
        return
    if isinstance(optimizers, (torch.optim.Optimizer, LARC)):
        optimizers = [optimizers]
    loss_scaler = _amp_state.loss_scalers[loss_id]
    if not loss_scaler.device_mode and _device_scaler_wanted(loss_scaler, optimizers):
        loss_scaler.enable_device_mode(loss.device)
    if loss_scaler.device_mode:
        for optimizer in optimizers:  # an overflowing step: the fused kernels see the flag and no-op
            optimizer._dummy_overflow_buf = loss_scaler._overflow_buf
            optimizer._device_step = True  # FusedLAMB: step counters advance on the device, unless skipped
    loss_scale = loss_scaler.scale_for_loss()

    if (not _amp_state.opt_properties.master_weights) and (not loss_scaler.dynamic) and \
            not loss_scaler.device_mode and loss_scale == 1.0:
        yield loss.float()
        if _amp_state.opt_properties.patch_torch_functions and _amp_state.handle is not None:
            _amp_state.handle._clear_cache()
        return

    if not delay_unscale:
        for optimizer in optimizers:
            if not optimizer._amp_stash.params_have_scaled_gradients:
                optimizer._prepare_amp_backward()

    yield loss.float() * loss_scale

    if delay_unscale:
        for optimizer in optimizers:
            optimizer._amp_stash.params_have_scaled_gradients = True
    else:
        loss_scaler.clear_overflow_state()
        for optimizer in optimizers:
            optimizer._post_amp_backward(loss_scaler)
            optimizer._amp_stash.params_have_scaled_gradients = False
        should_skip = False if delay_overflow_check else loss_scaler.update_scale()
        if should_skip:
            for optimizer in optimizers:
                if not optimizer._amp_stash.already_patched:
                    def patch_step(opt, loss_scaler, loss_id):
                        opt_step = opt.step

                        def skip_step(closure=None):
                            if closure is not None:
                                raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
                            maybe_print(("Gradient overflow.  Skipping step, loss scaler {} reducing loss scale to {}")
                                        .format(loss_id, loss_scaler.loss_scale()))
                            if hasattr(opt._amp_stash, "all_fp32_from_fp16_params"):
                                for param in opt._amp_stash.all_fp32_from_fp16_params:
                                    param.grad = None
                            if hasattr(opt, "most_recent_scale"):
                                opt.most_recent_scale = 1.0
                                opt.scale_set_by_backward = False
                            opt.step = opt_step
                            opt._amp_stash.already_patched = False
                        return skip_step

                    optimizer.step = patch_step(optimizer, loss_scaler, loss_id)
                    optimizer._amp_stash.already_patched = True

    if _amp_state.opt_properties.patch_torch_functions and _amp_state.handle is not None:
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


class AmpHandle(object):
    """Legacy (pre-``amp.initialize``) handle returned by ``amp.init()``."""

    def __init__(self, loss_scale="dynamic", enable_caching=True, verbose=False):
        self._enable_caching = enable_caching
        self._verbose = verbose
        self._cache = dict()
        self._default_scaler = LossScaler(loss_scale)
        self._is_active = True
        self._all_wrappers = []

    def is_active(self):
        return self._is_active

    @contextlib.contextmanager
    def _disable_casts(self):
        self._is_active = False
        yield
        self._is_active = True

    def wrap_optimizer(self, optimizer, num_loss=1):
        from .opt import OptimWrapper

        self._default_scaler = None
        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        raise RuntimeError("The old Amp API is no longer supported.  Please move to the new API, documented "
                           "here:  https://nvidia.github.io/apex/amp.html.  Transition guide:  "
                           "https://nvidia.github.io/apex/amp.html#transition-guide-for-old-api-users")

    def _clear_cache(self):
        self._cache.clear()

    # Experimental support for saving / restoring uncasted versions of functions
    def _save_func(self, mod, fn, func):
        self._all_wrappers.append((mod, fn, func))

    def _deactivate(self):
        for mod, fn, func in self._all_wrappers:
            setattr(mod, fn, func)
        self._all_wrappers = []

    @property
    def has_cache(self):
        return self._enable_caching

    @property
    def cache(self):
        return self._cache

    def remove_cache(self, param):
        if self.has_cache and param in self.cache:
            del self.cache[param]

    @property
    def verbose(self):
        return self._verbose


class NoOpHandle(object):
    def is_active(self):
        return False

    @contextlib.contextmanager
    def _disable_casts(self):
        yield

    def wrap_optimizer(self, optimizer, num_loss=1):
        from .opt import OptimWrapper

        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        yield loss

    @property
    def has_cache(self):
        return False

    @property
    def verbose(self):
        return False

    def _clear_cache(self):
        pass

    def _deactivate(self):
        pass
