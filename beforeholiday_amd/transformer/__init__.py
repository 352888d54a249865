"""Megatron-style model parallelism (reference: apex/transformer): parallel_state, tensor_parallel
(TP + sequence parallel), pipeline_parallel (1F1B / interleaved / no-pipelining schedules + p2p),
amp.GradScaler, microbatches, fused softmax, layers, testing harness."""
import importlib

from .enums import AttnMaskType, AttnType, LayerType, ModelType

_LAZY = ["amp", "functional", "parallel_state", "pipeline_parallel", "tensor_parallel", "utils", "layers",
         "microbatches", "testing", "log_util"]

__all__ = _LAZY + ["LayerType", "AttnType", "AttnMaskType", "ModelType"]


def __getattr__(name):
    if name in _LAZY:
        mod = importlib.import_module(f".{name}", __name__)
        globals()[name] = mod
        return mod
    raise AttributeError(name)
