"""O1 / O4 casting for ``torch.nn`` recurrent layers.

``torch.nn.modules.rnn`` calls its kernels through a module-level ``_VF`` reference
(``_VF.lstm(...)``, ``_VF.gru_cell(...)``, ...), which is a read-only extension module, so the
generic function patching of ``amp.init`` cannot reach them. Behaviour of the reference
(``apex/amp/amp.py:172-183``, ``apex/amp/rnn_compat.py:17-53``, ``apex/amp/wrap.py:226-275``):
under O1 an ``nn.LSTM`` / ``nn.GRU`` / ``nn.RNN`` (packed or padded, any depth / direction) and the
``*Cell`` modules run in the low-precision type while the parameters stay fp32.

Design here:

* :class:`VFShim` is a mutable stand-in for ``_VF``: attribute lookups fall through to the real
  ``torch._VF`` unless amp installed a wrapper on the shim. It is swapped into
  ``torch.nn.modules.rnn._VF`` through the handle's save list, so ``amp`` deactivation restores the
  original reference.
* full-sequence functions (``lstm``, ``gru``, ``rnn_tanh``, ``rnn_relu``): every floating tensor
  argument (input, hidden state(s)) is cast, and the flat weight list is re-synthesised as views of
  ONE low-precision buffer (an autograd-tracked ``cat`` of the casts), so the MIOpen RNN path sees
  packed contiguous weights and gradients flow back into the fp32 parameters. Packed sequences keep
  their int64 ``batch_sizes`` untouched.
* cell functions (``*_cell``): plain argument casts with the per-iteration weight-cast cache.
"""
from __future__ import annotations

import functools

import torch

from . import utils

RNN_NAMES = ("rnn_relu", "rnn_tanh", "gru", "lstm")


class VFShim:
    """Mutable proxy of ``torch._VF``: explicit attributes override, everything else delegates."""

    def __init__(self, target=None):
        object.__setattr__(self, "_target", target if target is not None else torch._VF)

    def __getattr__(self, name):
        return getattr(object.__getattribute__(self, "_target"), name)


def _flat_low_precision(weights, dtype):
    """Views of one contiguous ``dtype`` buffer holding every weight of ``weights`` (differentiable)."""
    if not weights:
        return weights
    flat = torch.cat([w.reshape(-1).to(dtype) for w in weights])
    out, off = [], 0
    for w in weights:
        n = w.numel()
        out.append(flat[off:off + n].view(w.shape))
        off += n
    return out


def _is_weight_list(x):
    return isinstance(x, (list, tuple)) and len(x) > 0 and all(isinstance(w, torch.Tensor) for w in x) \
        and any(isinstance(w, torch.nn.Parameter) or w.requires_grad for w in x)


def make_rnn_wrapper(orig_fn, cast_fn, handle):
    dtype = cast_fn.dtype

    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if not handle.is_active():
            return orig_fn(*args, **kwargs)
        new_args = []
        for a in args:
            if _is_weight_list(a):
                new_args.append(_flat_low_precision(list(a), dtype))
            elif isinstance(a, tuple):  # LSTM (h, c)
                new_args.append(tuple(cast_fn(t) for t in a))
            else:
                new_args.append(cast_fn(a))
        return orig_fn(*new_args, **kwargs)

    return wrapper


def _make_check_input(orig_check, handle):
    """``RNNBase.check_input`` rejects an input whose dtype differs from the (fp32) weights unless
    torch autocast is on; under amp the casts happen one level down, so validate the shape against a
    zero-storage stand-in of the weight dtype instead."""

    @functools.wraps(orig_check)
    def check_input(self, input, batch_sizes):
        w = self._flat_weights[0] if getattr(self, "_flat_weights", None) else None
        if handle.is_active() and w is not None and input.is_floating_point() and input.dtype != w.dtype:
            input = input.new_empty((), dtype=w.dtype).expand(input.shape)
        return orig_check(self, input, batch_sizes)

    return check_input


def install(handle, cast_fn, verbose=False):
    """Patch ``torch.nn.modules.rnn._VF`` with a shim carrying the cast wrappers (saved on ``handle``)."""
    rnn_mod = torch.nn.modules.rnn
    shim = VFShim(torch._VF)
    utils.set_func_save(handle, rnn_mod, "_VF", shim)
    base = rnn_mod.RNNBase
    utils.set_func_save(handle, base, "check_input", _make_check_input(base.check_input, handle))
    vcast = utils.verbosify(cast_fn, "rnn", verbose)
    for name in RNN_NAMES:
        if hasattr(torch._VF, name):
            object.__setattr__(shim, name, make_rnn_wrapper(getattr(torch._VF, name), vcast, handle))
    from . import wrap

    for name in RNN_NAMES:
        cell = name + "_cell"
        if hasattr(torch._VF, cell):
            object.__setattr__(shim, cell, getattr(torch._VF, cell))  # make it patchable on the shim
            wrap.cached_cast(shim, cell, cast_fn, handle, try_caching=True, verbose=verbose)
    return shim


def has_old_rnns():
    """The pre-1.0 THNN RNN backend never exists on supported torch versions."""
    return False
