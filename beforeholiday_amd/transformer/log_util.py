"""Logger helpers (reference: apex/transformer/log_util.py:5-18)."""
import logging
import os


def get_transformer_logger(name: str) -> logging.Logger:
    return logging.getLogger(os.path.splitext(name)[0])


def set_logging_level(verbosity) -> None:
    logging.getLogger("beforeholiday_amd").setLevel(verbosity)
