"""Function wrappers installed by ``amp.init`` (reference: apex/amp/wrap.py:10-275)."""
from __future__ import annotations

import functools

import torch

from . import utils

_LOW = (torch.float16, torch.bfloat16)


def make_cast_wrapper(orig_fn, cast_fn, handle, try_caching=False):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if not handle.is_active():
            return orig_fn(*args, **kwargs)
        if try_caching and handle.has_cache:
            args = [utils.cached_cast(cast_fn, a, handle.cache) for a in args]
            kwargs = {k: utils.cached_cast(cast_fn, v, handle.cache) for k, v in kwargs.items()}
            return orig_fn(*args, **kwargs)
        new_args, new_kwargs = utils.casted_args(cast_fn, args, kwargs)
        return orig_fn(*new_args, **new_kwargs)

    return wrapper


def cached_cast(mod, fn, cast_fn, handle, try_caching=False, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)
    cast_fn = utils.verbosify(cast_fn, fn, verbose)
    utils.set_func_save(handle, mod, fn, make_cast_wrapper(orig_fn, cast_fn, handle, try_caching))


def make_promote_wrapper(orig_fn, cast_fn, handle=None):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if handle is not None and not handle.is_active():
            return orig_fn(*args, **kwargs)
        types = utils.collect_fp_tensor_types(args, kwargs)
        if len(types) <= 1:
            return orig_fn(*args, **kwargs)
        if types <= {torch.float16, torch.float32} or types <= {torch.bfloat16, torch.float32} or \
                torch.float32 in types:
            new_args, new_kwargs = utils.casted_args(utils.maybe_float, args, kwargs)
            return orig_fn(*new_args, **new_kwargs)
        raise NotImplementedError("Do not know how to handle these types to promote: {}".format(types))

    return wrapper


def promote(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)
    utils.set_func_save(handle, mod, fn, make_promote_wrapper(orig_fn, utils.maybe_float, handle))


def sequence_promote(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(seq, *args, **kwargs):
        if not handle.is_active():
            return orig_fn(seq, *args, **kwargs)
        types = set(x.dtype for x in seq if utils.is_fp_tensor(x))
        if len(types) <= 1:
            return orig_fn(seq, *args, **kwargs)
        if torch.float32 in types or len(types & set(_LOW)) > 1:
            cast_seq = utils.casted_args(utils.maybe_float, seq, {})[0]
            return orig_fn(cast_seq, *args, **kwargs)
        return orig_fn(seq, *args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def promote_match_arg0(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(arg0, *args, **kwargs):
        assert utils.is_fp_tensor(arg0) or True
        if not handle.is_active() or not utils.is_fp_tensor(arg0):
            return orig_fn(arg0, *args, **kwargs)
        cast_fn = utils._caster(arg0.dtype, "match_arg0")
        new_args, new_kwargs = utils.casted_args(cast_fn, args, kwargs)
        return orig_fn(arg0, *new_args, **new_kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def err_if_any_half(mod, fn, handle, custom_err_msg=None):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if handle.is_active():
            types = utils.collect_fp_tensor_types(args, kwargs)
            if types & set(_LOW):
                if custom_err_msg:
                    raise NotImplementedError(custom_err_msg)
                raise NotImplementedError("Cannot call in-place function {} with fp16 arguments.".format(fn))
        return orig_fn(*args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def err_if_arg0_half(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(arg0, *args, **kwargs):
        if handle.is_active() and utils.is_fp_tensor(arg0) and arg0.dtype in _LOW:
            raise NotImplementedError("Cannot call in-place method {} on fp16 Tensors.".format(fn))
        if handle.is_active():
            new_args, new_kwargs = utils.casted_args(utils.maybe_float, args, kwargs)
            return orig_fn(arg0, *new_args, **new_kwargs)
        return orig_fn(arg0, *args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)
