"""Library logger with a rank-aware formatter (reference: apex/__init__.py:27-39 — records carry
``rank:(tp,pp,dp)``; apex/transformer/log_util.py)."""
import logging
import os

import torch

_LOGGER_NAME = "beforeholiday_amd"


class RankInfoFormatter(logging.Formatter):
    """Adds ``rank_info`` = (tensor, pipeline, data) parallel ranks (or global rank) to records."""

    def format(self, record):
        try:
            from ..transformer.parallel_state import get_rank_info
            record.rank_info = get_rank_info()
        except Exception:  # noqa: BLE001 - formatting must never raise
            record.rank_info = (0, 0, 0)
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            record.global_rank = torch.distributed.get_rank()
        else:
            record.global_rank = int(os.environ.get("RANK", 0))
        return super().format(record)


def get_logger(name: str = _LOGGER_NAME) -> logging.Logger:
    logger = logging.getLogger(name)
    root = logging.getLogger(_LOGGER_NAME)
    if not root.handlers:
        h = logging.StreamHandler()
        h.setFormatter(RankInfoFormatter(
            "%(asctime)s - PID:%(process)d - rank:%(global_rank)s %(rank_info)s - %(filename)s:%(lineno)d - "
            "%(levelname)s - %(message)s", "%Y-%m-%d %H:%M:%S"))
        root.addHandler(h)
        root.setLevel(logging.WARNING)
        root.propagate = False
    return logger


def set_logging_level(verbosity) -> None:
    get_logger().setLevel(verbosity)
