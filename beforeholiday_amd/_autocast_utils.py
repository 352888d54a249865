"""Autocast helpers for fused functional ops (reference: apex/_autocast_utils.py:1-23)."""
from typing import Optional, Sequence

import torch


def _get_autocast_dtypes() -> Sequence[torch.dtype]:
    return [torch.half, torch.bfloat16]


def _get_current_dtype(dtype: Optional[torch.dtype] = None) -> torch.dtype:
    if not torch.is_autocast_enabled("cuda"):
        return dtype or torch.get_default_dtype()
    return torch.get_autocast_dtype("cuda")


def _cast_if_autocast_enabled(*args):
    if not torch.is_autocast_enabled("cuda"):
        return args
    return torch.amp.autocast_mode._cast(args, "cuda", torch.get_autocast_dtype("cuda"))
