"""Utilities: rank-aware logging, tracing ranges / timers, checkpoint save & resume."""
from .checkpoint import load_checkpoint, save_checkpoint
from . import graph_rng
from .graphs import GraphedStep, capture_checked, training_state
from .logging import RankInfoFormatter, get_logger, set_logging_level
from .profiling import (EventTimer, annotate, profile_range, profiler_start, profiler_stop, range_pop, range_push,
                        report_memory)

__all__ = ["graph_rng", "get_logger", "set_logging_level", "RankInfoFormatter", "range_push", "range_pop", "profile_range",
           "annotate", "profiler_start", "profiler_stop", "EventTimer", "report_memory", "save_checkpoint",
           "load_checkpoint", "GraphedStep", "capture_checked", "training_state"]
