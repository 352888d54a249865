"""Tensor-parallel helpers (reference: apex/transformer/tensor_parallel/utils.py:22-64)."""
from typing import List, Sequence

import torch

from ..utils import divide


def split_tensor_along_last_dim(tensor: torch.Tensor, num_partitions: int,
                                contiguous_split_chunks: bool = False) -> List[torch.Tensor]:
    last_dim = tensor.dim() - 1
    chunks = torch.split(tensor, divide(tensor.size(last_dim), num_partitions), dim=last_dim)
    if contiguous_split_chunks:
        return tuple(c.contiguous() for c in chunks)
    return chunks


class VocabUtility:
    """Vocab range [first, last) owned by a TP rank."""

    @staticmethod
    def vocab_range_from_per_partition_vocab_size(per_partition_vocab_size: int, rank, world_size: int) -> Sequence[int]:
        first = rank * per_partition_vocab_size
        return first, first + per_partition_vocab_size

    @staticmethod
    def vocab_range_from_global_vocab_size(global_vocab_size: int, rank: int, world_size: int) -> Sequence[int]:
        return VocabUtility.vocab_range_from_per_partition_vocab_size(divide(global_vocab_size, world_size), rank,
                                                                      world_size)
