"""O1/O4 function patching and the user decorator / registry API.

Behaviour of /root/reference/apex/amp/amp.py:29-198 (which functions get which wrapper, and in what
order), organised differently: the whole patch set is a list of :class:`_Rule` entries produced by
:func:`_rules`, and :func:`init` just installs them. Registering a user function appends a rule that
the next :func:`init` installs first.
"""
from __future__ import annotations

import functools
import itertools
from typing import Callable, Iterator, List, NamedTuple

import torch

from . import rnn_compat, utils, wrap
from ._amp_state import _amp_state
from .handle import AmpHandle, NoOpHandle
from .lists import functional_overrides, tensor_overrides, torch_overrides

_DECORATOR_HANDLE = None


class _Rule(NamedTuple):
    """Install ``apply(module, name, handle, verbose)`` on ``module.name``."""
    module: object
    name: str
    apply: Callable


def _cast(cast_fn, cache):
    return lambda mod, fn, handle, verbose: wrap.cached_cast(mod, fn, cast_fn, handle, cache, verbose)


def _plain(installer):
    return lambda mod, fn, handle, verbose: installer(mod, fn, handle, verbose)


def _error(msg=None):
    return lambda mod, fn, handle, verbose: wrap.err_if_any_half(mod, fn, handle, msg)


# user registrations, consumed by the next init()
_USER_RULES: List[_Rule] = []

# the low-precision cast per patch type: (override-list attribute, cast function)
_LOW = {torch.float16: ("FP16_FUNCS", utils.maybe_half), torch.bfloat16: ("BFLOAT16_FUNCS", utils.maybe_bfloat16)}


def _rules(low_list: str, low_cast, allow_banned: bool) -> Iterator[_Rule]:
    """Every wrapper O1 / O4 installs, in installation order."""
    yield from _USER_RULES
    tables = (functional_overrides, torch_overrides, tensor_overrides)
    # forced casts: whitelist -> low precision (cached casts of parameters), blacklist -> fp32
    for t in tables:
        yield from (_Rule(t.MODULE, fn, _cast(low_cast, True)) for fn in getattr(t, low_list))
        yield from (_Rule(t.MODULE, fn, _cast(utils.maybe_float, False)) for fn in t.FP32_FUNCS)
    # type promotion on multi-argument functions / methods (sequence variants for torch.cat & co)
    for t in (torch_overrides, tensor_overrides):
        yield from (_Rule(t.MODULE, fn, _plain(wrap.promote)) for fn in t.CASTS)
        yield from (_Rule(t.MODULE, fn, _plain(wrap.sequence_promote)) for fn in t.SEQUENCE_CASTS)
    # in-place blacklist functions refuse low-precision inputs; other in-place methods match self
    yield from (_Rule(torch_overrides.MODULE, fn, _error()) for fn in utils.as_inplace(torch_overrides.FP32_FUNCS))
    tm = tensor_overrides.MODULE
    yield from (_Rule(tm, fn, _plain(wrap.err_if_arg0_half)) for fn in utils.as_inplace(tensor_overrides.FP32_FUNCS))
    matched = itertools.chain(getattr(tensor_overrides, low_list), tensor_overrides.CASTS)
    yield from (_Rule(tm, fn, _plain(wrap.promote_match_arg0)) for fn in utils.as_inplace(matched))
    # banned functions (e.g. binary_cross_entropy): error, or fp32 when explicitly allowed
    for fn, msg in functional_overrides.BANNED_FUNCS:
        yield _Rule(functional_overrides.MODULE, fn, _cast(utils.maybe_float, True) if allow_banned else _error(msg))


# ---- decorators / registration -------------------------------------------------------------------

def _decorated(orig_fn, cast_fn, make_wrapper):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        handle = _DECORATOR_HANDLE
        if handle is None or not handle.is_active():
            return orig_fn(*args, **kwargs)
        return make_wrapper(orig_fn, utils.verbosify(cast_fn, orig_fn.__name__, handle.verbose), handle)(*args,
                                                                                                           **kwargs)

    return wrapper


def half_function(fn):
    return _decorated(fn, utils.maybe_half, functools.partial(wrap.make_cast_wrapper, try_caching=True))


def bfloat16_function(fn):
    return _decorated(fn, utils.maybe_bfloat16, functools.partial(wrap.make_cast_wrapper, try_caching=True))


def float_function(fn):
    return _decorated(fn, utils.maybe_float, functools.partial(wrap.make_cast_wrapper, try_caching=False))


def promote_function(fn):
    return _decorated(fn, utils.maybe_float, wrap.make_promote_wrapper)


def _register(module, name, apply):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_RULES.append(_Rule(module, name, apply))


def register_half_function(module, name):
    _register(module, name, _cast(utils.maybe_half, True))


def register_bfloat16_function(module, name):
    _register(module, name, _cast(utils.maybe_bfloat16, True))


def register_float_function(module, name):
    _register(module, name, _cast(utils.maybe_float, False))


def register_promote_function(module, name):
    _register(module, name, _plain(wrap.promote))


# ---- install / remove ----------------------------------------------------------------------------

def deactivate():
    """Remove every installed wrapper (restores the original torch functions)."""
    global _DECORATOR_HANDLE
    if _amp_state.handle is not None:
        _amp_state.handle._deactivate()
    _amp_state.handle = None
    _DECORATOR_HANDLE = None


def init(enabled=True, loss_scale="dynamic", patch_type=torch.float16, enable_caching=True, verbose=False,
         allow_banned=False):
    """Install the O1 (fp16) / O4 (bf16) cast wrappers on torch, torch.Tensor and F."""
    global _DECORATOR_HANDLE
    if isinstance(_amp_state.handle, AmpHandle):  # re-initialisation: do not stack wrappers
        _amp_state.handle._deactivate()
    if not enabled:
        _DECORATOR_HANDLE = NoOpHandle()
        _amp_state.handle = None
        return _DECORATOR_HANDLE
    if patch_type not in _LOW:
        raise RuntimeError("Unsupported patch_torch_functions_type passed to initialize. Supported types are: "
                           "torch.float16 and torch.bfloat16.")
    low_list, low_cast = _LOW[patch_type]
    handle = AmpHandle(loss_scale, enable_caching, verbose)
    handle.cast_dtype = patch_type
    for rule in list(_rules(low_list, low_cast, allow_banned)):
        rule.apply(rule.module, rule.name, handle, verbose)
    _USER_RULES.clear()
    # recurrent layers (nn.RNN/GRU/LSTM, packed sequences, *Cell modules) run in the low-precision
    # type through a mutable stand-in for torch.nn.modules.rnn._VF
    rnn_compat.install(handle, low_cast, verbose)
    _DECORATOR_HANDLE = handle
    _amp_state.handle = handle
    return handle


def kernel_cast_dtype():
    """The 16-bit dtype amp's O1 / O4 function patching casts matmul-class ops to (None when that
    patching is off or disabled, e.g. inside the optimizer step). Modules that call the own MFMA
    kernels directly -- which the patched torch functions never see -- use it to run those kernels in
    the same precision the cast lists give ``conv2d`` / ``linear`` (reference:
    apex/amp/lists/functional_overrides.py:18-32)."""
    h = _amp_state.handle
    if h is None or not h.is_active():
        return None
    return getattr(h, "cast_dtype", None)


def kernel_cast(t):
    """``t`` in :func:`kernel_cast_dtype` through amp's per-iteration weight-cast cache (a leaf fp32
    parameter is cast once per iteration; the cast is differentiable, so the parameter still gets an
    fp32 gradient). Returns ``t`` unchanged when no cast applies."""
    dt = kernel_cast_dtype()
    if dt is None or not t.is_floating_point() or t.dtype == dt:
        return t
    fn = utils.maybe_half if dt == torch.float16 else utils.maybe_bfloat16
    return utils.cached_cast(fn, t, _amp_state.handle.cache)
