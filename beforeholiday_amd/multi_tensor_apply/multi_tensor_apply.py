"""MultiTensorApply (reference: apex/multi_tensor_apply/multi_tensor_apply.py:3-30)."""
from __future__ import annotations


class MultiTensorApply(object):
    # The pure-PyTorch path always exists (CPU lists); GPU lists require the native extension and
    # raise from the op itself if it is missing, so ``available`` is always True here.
    available = True
    warned = False

    def __init__(self, chunk_size: int):
        if chunk_size <= 0 or chunk_size % 8:
            raise ValueError("chunk_size must be a positive multiple of 8")
        self.chunk_size = chunk_size

    def check_avail(self):
        return True

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)
