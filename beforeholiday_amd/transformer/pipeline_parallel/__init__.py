"""Pipeline model parallelism: p2p stage exchange + 1F1B / interleaved / no-pipelining schedules
(reference: apex/transformer/pipeline_parallel/__init__.py)."""
from .schedules import get_forward_backward_func
from .schedules.common import build_model

__all__ = ["get_forward_backward_func", "build_model"]
