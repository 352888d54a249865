"""Optimizer wrapper of the legacy ``handle.wrap_optimizer`` API (reference: apex/amp/opt.py:9-103):
one dynamic loss scaler per loss of a multi-loss step, and the step skipped when any of them saw an
overflow.

Design here: the wrapper is a thin proxy (``__getattr__`` forwards everything it does not define) that
keeps, per step, a cursor over the losses. Because the gradients of several losses accumulate into
the same ``.grad`` tensors, loss ``i > 0`` is unscaled on its own: the gradients accumulated so far
are moved aside before its backward and added back after it has been unscaled with ITS scale."""
import contextlib

from ._amp_state import maybe_print
from .scaler import LossScaler


class OptimWrapper(object):
    def __init__(self, optimizer, amp_handle, num_loss):
        self._optimizer = optimizer
        self._amp_handle = amp_handle
        self._num_loss = num_loss
        self._scalers = [LossScaler("dynamic") for _ in range(num_loss)]
        self._overflowed = [False] * num_loss
        self._cursor = 0  # index of the next loss of this step

    def _all_params(self):
        return [p for g in self._optimizer.param_groups for p in g["params"]]

    @contextlib.contextmanager
    def scale_loss(self, loss):
        if not self._amp_handle.is_active():
            yield loss
            return
        if not 0 <= self._cursor < self._num_loss:
            raise RuntimeError(f"scale_loss called for more than num_loss={self._num_loss} losses in one step")
        scaler = self._scalers[self._cursor]
        params = self._all_params()
        # gradients of the previous losses of this step, set aside (they carry other scales)
        earlier = [p.grad.detach().clone() if (self._cursor > 0 and p.grad is not None) else None for p in params]
        if self._cursor > 0:
            self._optimizer.zero_grad()
        scale = scaler.loss_scale()
        yield loss * scale
        scaler.clear_overflow_state()
        fresh = [p.grad for p in params if p.grad is not None]
        scaler.unscale(fresh, fresh, scale)
        self._overflowed[self._cursor] = scaler.update_scale()
        self._cursor += 1
        for p, g in zip(params, earlier):
            if g is None:
                continue
            if p.grad is None:  # this loss did not reach p (zero_grad set its grad to None)
                p.grad = g
            else:
                p.grad.data.add_(g)

    def step(self, closure=None):
        if not self._amp_handle.is_active():
            return self._optimizer.step(closure=closure)
        if closure is not None:
            raise NotImplementedError("The `closure` argument is unsupported by the amp optimizer wrapper.")
        self._cursor = 0
        for p in self._all_params():
            self._amp_handle.remove_cache(p)
        if any(self._overflowed):
            self._overflowed = [False] * self._num_loss
            maybe_print("Gradient overflow, skipping update")
            return None
        return self._optimizer.step()

    # everything else is the wrapped optimizer's
    def __getattr__(self, name):
        return getattr(self._optimizer, name)

    def __repr__(self):
        return repr(self._optimizer)

    def state_dict(self):
        return self._optimizer.state_dict()

    def load_state_dict(self, state_dict):
        return self._optimizer.load_state_dict(state_dict)

    def zero_grad(self, *args, **kwargs):
        return self._optimizer.zero_grad(*args, **kwargs)

    def add_param_group(self, param_group):
        return self._optimizer.add_param_group(param_group)
