"""Cast helpers for the O1/O4 function patching (reference: apex/amp/utils.py)."""
from __future__ import annotations

import functools
import itertools

import torch

_LOW = (torch.float16, torch.bfloat16)


def is_fp_tensor(x):
    return isinstance(x, torch.Tensor) and x.is_floating_point()


def is_nested(x):
    return isinstance(x, (tuple, list))


def should_cache(x):
    # only leaf parameters are cached (weights re-used across calls within an iteration)
    return isinstance(x, torch.nn.Parameter) or (isinstance(x, torch.Tensor) and x.is_leaf and x.requires_grad)


def collect_fp_tensor_types(args, kwargs):
    def collect(x, out):
        if is_fp_tensor(x):
            out.add(x.dtype)
        elif is_nested(x):
            for y in x:
                collect(y, out)

    types = set()
    for a in itertools.chain(args, kwargs.values()):
        collect(a, types)
    return types


def _caster(dtype, name):
    def cast(x):
        if is_nested(x):
            return type(x)(cast(y) for y in x)
        if not is_fp_tensor(x) or x.dtype == torch.float64 or x.dtype == dtype:
            return x
        return x.to(dtype)

    cast.__name__ = name
    cast.dtype = dtype
    return cast


maybe_half = _caster(torch.float16, "maybe_half")
maybe_bfloat16 = _caster(torch.bfloat16, "maybe_bfloat16")
maybe_float = _caster(torch.float32, "maybe_float")


def type_string(x):
    return x.type() if isinstance(x, torch.Tensor) else type(x).__name__


def verbosify(cast_fn, fn_name, verbose):
    if not verbose:
        return cast_fn

    def wrapper(x):
        if is_fp_tensor(x) and x.dtype != cast_fn.dtype:
            print("Float->{} ({})".format(cast_fn.dtype, fn_name))
        return cast_fn(x)

    wrapper.dtype = cast_fn.dtype
    return wrapper


def cached_cast(cast_fn, x, cache):
    """Cast with a per-iteration cache for leaf params (invalidated on in-place updates)."""
    if is_nested(x):
        return type(x)(cached_cast(cast_fn, y, cache) for y in x)
    if not is_fp_tensor(x) or x.dtype == cast_fn.dtype:
        return cast_fn(x)
    if should_cache(x):
        key = (id(x), cast_fn.dtype)
        hit = cache.get(key)
        grad_on = torch.is_grad_enabled()
        if hit is not None and hit[0] is x and hit[1] == x._version and hit[2] == grad_on:
            return hit[3]
        y = cast_fn(x)
        cache[key] = (x, x._version, grad_on, y)
        return y
    return cast_fn(x)


def casted_args(cast_fn, args, kwargs):
    new_args = [cast_fn(a) for a in args]
    new_kwargs = {k: cast_fn(v) for k, v in kwargs.items()}
    return new_args, new_kwargs


def as_inplace(fns):
    for x in fns:
        yield x + "_"


def has_func(mod, fn):
    if isinstance(mod, dict):
        return fn in mod
    return hasattr(mod, fn)


def get_func(mod, fn):
    return mod[fn] if isinstance(mod, dict) else getattr(mod, fn)


def set_func(mod, fn, new_fn):
    if isinstance(mod, dict):
        mod[fn] = new_fn
    else:
        setattr(mod, fn, new_fn)


def set_func_save(handle, mod, fn, new_fn):
    cur_fn = get_func(mod, fn)
    handle._save_func(mod, fn, cur_fn)
    set_func(mod, fn, new_fn)
