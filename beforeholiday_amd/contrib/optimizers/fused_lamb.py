"""contrib FusedLAMB (reference: apex/contrib/optimizers/fused_lamb.py:6-208): the same algorithm as
:class:`beforeholiday_amd.optimizers.FusedLAMB` (fused stage-1/stage-2 kernels, global grad-norm
clipping), re-exported under the contrib path."""
from ...optimizers.fused_lamb import FusedLAMB

__all__ = ["FusedLAMB"]
