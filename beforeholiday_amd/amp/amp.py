"""O1/O4 function patching and the user decorator/registry API (reference: apex/amp/amp.py:29-198)."""
from __future__ import annotations

import functools
import itertools

import torch

from . import rnn_compat, utils, wrap
from ._amp_state import _amp_state
from .handle import AmpHandle, NoOpHandle
from .lists import functional_overrides, tensor_overrides, torch_overrides

_DECORATOR_HANDLE = None
_USER_CAST_REGISTRY = set()
_USER_PROMOTE_REGISTRY = set()


def _decorator_helper(orig_fn, cast_fn, wrap_fn):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        handle = _DECORATOR_HANDLE
        if handle is None or not handle.is_active():
            return orig_fn(*args, **kwargs)
        inner_cast_fn = utils.verbosify(cast_fn, orig_fn.__name__, handle.verbose)
        return wrap_fn(orig_fn, inner_cast_fn, handle)(*args, **kwargs)

    return wrapper


def half_function(fn):
    return _decorator_helper(fn, utils.maybe_half, functools.partial(wrap.make_cast_wrapper, try_caching=True))


def bfloat16_function(fn):
    return _decorator_helper(fn, utils.maybe_bfloat16, functools.partial(wrap.make_cast_wrapper, try_caching=True))


def float_function(fn):
    return _decorator_helper(fn, utils.maybe_float, functools.partial(wrap.make_cast_wrapper, try_caching=False))


def promote_function(fn):
    return _decorator_helper(fn, utils.maybe_float, wrap.make_promote_wrapper)


def _register(module, name, entry, registry):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    registry.add(entry)


def register_half_function(module, name):
    _register(module, name, (module, name, utils.maybe_half), _USER_CAST_REGISTRY)


def register_bfloat16_function(module, name):
    _register(module, name, (module, name, utils.maybe_bfloat16), _USER_CAST_REGISTRY)


def register_float_function(module, name):
    _register(module, name, (module, name, utils.maybe_float), _USER_CAST_REGISTRY)


def register_promote_function(module, name):
    _register(module, name, (module, name), _USER_PROMOTE_REGISTRY)


def deactivate():
    """Remove every installed wrapper (restores the original torch functions)."""
    global _DECORATOR_HANDLE
    h = _amp_state.handle
    if h is not None:
        h._deactivate()
    _amp_state.handle = None
    _DECORATOR_HANDLE = None


def init(enabled=True, loss_scale="dynamic", patch_type=torch.float16, enable_caching=True, verbose=False,
         allow_banned=False):
    """Install the O1 (fp16) / O4 (bf16) cast wrappers on torch, torch.Tensor and F."""
    global _DECORATOR_HANDLE
    if _amp_state.handle is not None and isinstance(_amp_state.handle, AmpHandle):
        # re-initialisation: drop the previous wrappers first so they don't stack
        _amp_state.handle._deactivate()
    if not enabled:
        handle = NoOpHandle()
        _DECORATOR_HANDLE = handle
        _amp_state.handle = None
        return handle

    handle = AmpHandle(loss_scale, enable_caching, verbose)
    for mod, fn, cast_fn in _USER_CAST_REGISTRY:
        wrap.cached_cast(mod, fn, cast_fn, handle, cast_fn is not utils.maybe_float, verbose)
    _USER_CAST_REGISTRY.clear()
    for mod, fn in _USER_PROMOTE_REGISTRY:
        wrap.promote(mod, fn, handle, verbose)
    _USER_PROMOTE_REGISTRY.clear()

    if patch_type == torch.float16:
        low_prec_funcs, maybe_low = "FP16_FUNCS", utils.maybe_half
    elif patch_type == torch.bfloat16:
        low_prec_funcs, maybe_low = "BFLOAT16_FUNCS", utils.maybe_bfloat16
    else:
        raise RuntimeError("Unsupported patch_torch_functions_type passed to initialize. Supported types are: "
                           "torch.float16 and torch.bfloat16.")

    override_modules = [functional_overrides, torch_overrides, tensor_overrides]
    cast_table = [(low_prec_funcs, maybe_low), ("FP32_FUNCS", utils.maybe_float)]
    for module, (list_name, cast_fn) in itertools.product(override_modules, cast_table):
        for fn in getattr(module, list_name):
            wrap.cached_cast(module.MODULE, fn, cast_fn, handle, cast_fn is maybe_low, verbose)

    for promote_mod, (list_name, promote_fn) in itertools.product(
            [torch_overrides, tensor_overrides], [("CASTS", wrap.promote), ("SEQUENCE_CASTS", wrap.sequence_promote)]):
        for fn in getattr(promote_mod, list_name):
            promote_fn(promote_mod.MODULE, fn, handle, verbose)

    for fn in utils.as_inplace(torch_overrides.FP32_FUNCS):
        wrap.err_if_any_half(torch_overrides.MODULE, fn, handle)
    for fn in utils.as_inplace(tensor_overrides.FP32_FUNCS):
        wrap.err_if_arg0_half(tensor_overrides.MODULE, fn, handle, verbose)
    for fn in utils.as_inplace(itertools.chain(getattr(tensor_overrides, low_prec_funcs), tensor_overrides.CASTS)):
        wrap.promote_match_arg0(tensor_overrides.MODULE, fn, handle, verbose)

    # recurrent layers: nn.RNN/GRU/LSTM (+ packed sequences) and the *Cell modules run in the low
    # precision type through a mutable stand-in for torch.nn.modules.rnn._VF
    rnn_compat.install(handle, maybe_low, verbose)

    for fn, err_msg in functional_overrides.BANNED_FUNCS:
        if allow_banned:
            wrap.cached_cast(functional_overrides.MODULE, fn, utils.maybe_float, handle, True, verbose)
        else:
            wrap.err_if_any_half(functional_overrides.MODULE, fn, handle, err_msg)

    _DECORATOR_HANDLE = handle
    _amp_state.handle = handle
    return handle
