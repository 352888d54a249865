"""Fused optimizers (reference: apex/optimizers/__init__.py:1-7)."""
from .fused_sgd import FusedSGD
from .fused_adam import FusedAdam
from .fused_novograd import FusedNovoGrad
from .fused_lamb import FusedLAMB
from .fused_adagrad import FusedAdagrad
from .fused_mixed_precision_lamb import FusedMixedPrecisionLamb
from .fused_lars import FusedLARS

__all__ = ["FusedSGD", "FusedAdam", "FusedNovoGrad", "FusedLAMB", "FusedAdagrad",
           "FusedMixedPrecisionLamb", "FusedLARS"]
