from .layer_norm import FastLayerNorm, FastLayerNormFN, fast_layer_norm

__all__ = ["FastLayerNorm", "FastLayerNormFN", "fast_layer_norm"]
