from .asp import ASP
from .sparse_masklib import create_mask

__all__ = ["ASP", "create_mask"]
