from .grad_scaler import GradScaler

__all__ = ["GradScaler"]
