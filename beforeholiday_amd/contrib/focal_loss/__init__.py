from . import focal_loss
from .focal_loss import FocalLoss

__all__ = ["focal_loss", "FocalLoss"]
