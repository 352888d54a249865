from .fused_softmax import FusedScaleMaskSoftmax, GenericFusedScaleMaskSoftmax

__all__ = ["FusedScaleMaskSoftmax", "GenericFusedScaleMaskSoftmax"]
