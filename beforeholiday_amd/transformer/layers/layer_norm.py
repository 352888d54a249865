"""LayerNorms that tag their parameters for sequence parallelism
(reference: apex/transformer/layers/layer_norm.py:26-99).

With sequence parallelism each TP rank normalises a different sequence slice, so the LN weight/bias
gradients are partial and must be all-reduced over the TP group; the ``sequence_parallel_enabled``
attribute marks them for that reduction (see ``allreduce_sequence_parallel_grads``).
"""
import torch

from ...normalization.fused_layer_norm import FusedLayerNorm as _FusedLayerNorm
from ...normalization.fused_layer_norm import MixedFusedLayerNorm as _MixedFusedLayerNorm

__all__ = ["FusedLayerNorm", "FastLayerNorm", "MixedFusedLayerNorm", "allreduce_sequence_parallel_grads"]


def _set_sequence_parallel_enabled(param: torch.Tensor, sequence_parallel_enabled: bool) -> None:
    setattr(param, "sequence_parallel_enabled", sequence_parallel_enabled)


class FusedLayerNorm(_FusedLayerNorm):
    def __init__(self, normalized_shape, eps: float = 1e-5, elementwise_affine: bool = True, *,
                 sequence_parallel_enabled: bool = False):
        super().__init__(normalized_shape=normalized_shape, eps=eps, elementwise_affine=elementwise_affine)
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if self.elementwise_affine:
            _set_sequence_parallel_enabled(self.weight, sequence_parallel_enabled)
            _set_sequence_parallel_enabled(self.bias, sequence_parallel_enabled)


class MixedFusedLayerNorm(_MixedFusedLayerNorm):
    def __init__(self, normalized_shape, eps: float = 1e-5, **kwargs) -> None:
        self.sequence_parallel_enabled = kwargs.pop("sequence_parallel_enabled", False)
        super().__init__(normalized_shape=normalized_shape, eps=eps, **kwargs)
        if self.sequence_parallel_enabled:
            _set_sequence_parallel_enabled(self.weight, True)
            _set_sequence_parallel_enabled(self.bias, True)


class FastLayerNorm(FusedLayerNorm):
    """Hidden-size LayerNorm. The generic wave-per-row LN kernel already covers every hidden size the
    reference's size-specialised fast LN registers, so this is the fused LN with its signature."""

    def __init__(self, hidden_size, eps: float = 1e-5, *, sequence_parallel_enabled: bool = False):
        super().__init__(normalized_shape=hidden_size, eps=eps, elementwise_affine=True,
                         sequence_parallel_enabled=sequence_parallel_enabled)


def allreduce_sequence_parallel_grads(model: torch.nn.Module) -> None:
    """Sum the partial grads of all parameters tagged ``sequence_parallel_enabled`` over the TP group
    with one flat all-reduce."""
    from .. import parallel_state
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
    grads = [p.grad for p in model.parameters()
             if getattr(p, "sequence_parallel_enabled", False) and p.grad is not None]
    if not grads or parallel_state.get_tensor_model_parallel_world_size() == 1:
        return
    flat = _flatten_dense_tensors(grads)
    torch.distributed.all_reduce(flat, group=parallel_state.get_tensor_model_parallel_group())
    for g, s in zip(grads, _unflatten_dense_tensors(flat, grads)):
        g.copy_(s)
