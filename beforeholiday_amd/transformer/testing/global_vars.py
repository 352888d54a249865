"""Global argument / timer / microbatch state for the standalone test models
(reference: apex/transformer/testing/global_vars.py:26-270)."""
import torch

from ..microbatches import build_num_microbatches_calculator
from ..pipeline_parallel._timers import _Timers as Timers
from .arguments import parse_args

_GLOBAL_ARGS = None
_GLOBAL_NUM_MICROBATCHES_CALCULATOR = None
_GLOBAL_TOKENIZER = None
_GLOBAL_TENSORBOARD_WRITER = None
_GLOBAL_ADLR_AUTORESUME = None
_GLOBAL_TIMERS = None


def get_args():
    _ensure_var_is_initialized(_GLOBAL_ARGS, "args")
    return _GLOBAL_ARGS


def get_num_microbatches() -> int:
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get()


def get_current_global_batch_size() -> int:
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get_current_global_batch_size()


def update_num_microbatches(consumed_samples: int, *, consistency_check: bool = True) -> None:
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR.update(consumed_samples, consistency_check)


def get_tensorboard_writer():
    return _GLOBAL_TENSORBOARD_WRITER


def get_adlr_autoresume():
    return _GLOBAL_ADLR_AUTORESUME


def get_timers():
    _ensure_var_is_initialized(_GLOBAL_TIMERS, "timers")
    return _GLOBAL_TIMERS


def set_global_variables(extra_args_provider=None, args_defaults={}, override_args={}, ignore_unknown_args=False):
    """Parse args (with defaults / overrides), build the microbatch calculator and timers."""
    global _GLOBAL_ARGS, _GLOBAL_NUM_MICROBATCHES_CALCULATOR, _GLOBAL_TIMERS
    _GLOBAL_ARGS = parse_args(extra_args_provider=extra_args_provider, defaults=args_defaults,
                              override_args=override_args, ignore_unknown_args=ignore_unknown_args)
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        _GLOBAL_ARGS.rank, _GLOBAL_ARGS.rampup_batch_size, _GLOBAL_ARGS.global_batch_size,
        _GLOBAL_ARGS.micro_batch_size, _GLOBAL_ARGS.data_parallel_size)
    _GLOBAL_TIMERS = Timers()
    return _GLOBAL_ARGS


def destroy_global_vars():
    global _GLOBAL_ARGS, _GLOBAL_NUM_MICROBATCHES_CALCULATOR, _GLOBAL_TIMERS
    _GLOBAL_ARGS = None
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = None
    _GLOBAL_TIMERS = None


def _ensure_var_is_initialized(var, name):
    assert var is not None, f"{name} is not initialized."


def _ensure_var_is_not_initialized(var, name):
    assert var is None, f"{name} is already initialized."
