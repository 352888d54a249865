from .layer_norm import FastLayerNorm, FusedLayerNorm, MixedFusedLayerNorm, allreduce_sequence_parallel_grads

__all__ = ["FastLayerNorm", "FusedLayerNorm", "MixedFusedLayerNorm", "allreduce_sequence_parallel_grads"]
