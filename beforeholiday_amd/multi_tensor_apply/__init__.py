"""``multi_tensor_applier`` (reference: apex/multi_tensor_apply/__init__.py:3-4).

``multi_tensor_applier(op, noop_flag, tensor_lists, *args)`` calls
``op(chunk_size, noop_flag, tensor_lists, *args)``. Chunk sizes are the scheduling granule of the
gfx950 kernels: 16 K elements (64 KB fp32 per list) for elementwise ops and 64 K elements for
norms, i.e. enough chunks to fill 256 CUs for any realistic parameter set while keeping each
workgroup's loop long enough to hide HBM latency.
"""
from .multi_tensor_apply import MultiTensorApply

multi_tensor_applier = MultiTensorApply(16384)
multi_tensor_applier_l2norm = MultiTensorApply(65536)

__all__ = ["MultiTensorApply", "multi_tensor_applier", "multi_tensor_applier_l2norm"]
