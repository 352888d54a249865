"""Megatron-style batch samplers yielding LOCAL minibatches (global batch / dp)
(reference: apex/transformer/_data/_batchsampler.py:16-180).

Note: the reference's sequential sampler accumulates only ``local_minibatch_size`` indices before
slicing out this rank's part, which yields empty batches on data-parallel ranks > 0; here each
step accumulates ``local_minibatch_size * data_parallel_size`` indices (Megatron-LM semantics), so
every rank gets its own disjoint slice.
"""
import abc

import torch


class _Base:
    @abc.abstractmethod
    def __len__(self) -> int:
        ...

    @abc.abstractmethod
    def __iter__(self):
        ...


class MegatronPretrainingSampler(_Base):
    def __init__(self, total_samples: int, consumed_samples: int, local_minibatch_size: int, data_parallel_rank: int,
                 data_parallel_size: int, drop_last: bool = True):
        if total_samples <= 0:
            raise RuntimeError(f"no sample to consume: {total_samples}")
        if consumed_samples >= total_samples:
            raise RuntimeError(f"no samples left to consume: {consumed_samples}, {total_samples}")
        if local_minibatch_size <= 0:
            raise RuntimeError(f"local minibatch size must be greater than 0: {local_minibatch_size}")
        if data_parallel_size <= 0:
            raise RuntimeError(f"data parallel size must be greater than 0: {data_parallel_size}")
        if data_parallel_rank >= data_parallel_size:
            raise RuntimeError(f"data_parallel_rank should be smaller than data size: {data_parallel_rank}, "
                               f"{data_parallel_size}")
        self.total_samples = total_samples
        self.consumed_samples = consumed_samples
        self._local_minibatch_size = local_minibatch_size
        self.data_parallel_rank = data_parallel_rank
        self.data_parallel_size = data_parallel_size
        self.local_minibatch_times_data_parallel_size = local_minibatch_size * data_parallel_size
        self.drop_last = drop_last

    def __len__(self):
        return self.total_samples

    def get_start_end_idx(self):
        start = self.data_parallel_rank * self.local_minibatch_size
        return start, start + self.local_minibatch_size

    @property
    def local_minibatch_size(self) -> int:
        return self._local_minibatch_size

    @local_minibatch_size.setter
    def local_minibatch_size(self, new_local_minibatch_size) -> None:
        self._local_minibatch_size = new_local_minibatch_size
        self.local_minibatch_times_data_parallel_size = new_local_minibatch_size * self.data_parallel_size

    def __iter__(self):
        batch = []
        for idx in range(self.consumed_samples, self.total_samples):
            batch.append(idx)
            if len(batch) == self.local_minibatch_times_data_parallel_size:
                s, e = self.get_start_end_idx()
                yield batch[s:e]
                batch = []
        if batch and not self.drop_last:
            s, e = self.get_start_end_idx()
            yield batch[s:e]


class MegatronPretrainingRandomSampler(_Base):
    """Each DP rank owns a contiguous bucket of the dataset and draws a per-epoch permutation of it
    (seeded by the epoch, so resuming from ``consumed_samples`` reproduces the order)."""

    def __init__(self, total_samples: int, consumed_samples: int, local_minibatch_size: int, data_parallel_rank: int,
                 data_parallel_size: int) -> None:
        if total_samples <= 0:
            raise ValueError(f"no sample to consume: total_samples of {total_samples}")
        if local_minibatch_size <= 0:
            raise ValueError(f"Invalid local_minibatch_size: {local_minibatch_size}")
        if data_parallel_size <= 0:
            raise ValueError(f"Invalid data_parallel_size: {data_parallel_size}")
        if data_parallel_rank >= data_parallel_size:
            raise ValueError(f"data_parallel_rank should be smaller than data parallel size: {data_parallel_rank} < "
                             f"{data_parallel_size}")
        self.total_samples = total_samples
        self.consumed_samples = consumed_samples
        self._local_minibatch_size = local_minibatch_size
        self.data_parallel_rank = data_parallel_rank
        self.data_parallel_size = data_parallel_size
        self.local_minibatch_times_data_parallel_size = local_minibatch_size * data_parallel_size
        self.last_batch_size = total_samples % self.local_minibatch_times_data_parallel_size

    def __len__(self) -> int:
        return self.total_samples

    @property
    def local_minibatch_size(self) -> int:
        return self._local_minibatch_size

    @local_minibatch_size.setter
    def local_minibatch_size(self, new_local_minibatch_size) -> None:
        self._local_minibatch_size = new_local_minibatch_size
        self.local_minibatch_times_data_parallel_size = new_local_minibatch_size * self.data_parallel_size

    def __iter__(self):
        active = self.total_samples - self.last_batch_size
        self.epoch = self.consumed_samples // active
        current_epoch_samples = self.consumed_samples % active
        bucket_size = (self.total_samples // self.local_minibatch_times_data_parallel_size) * self.local_minibatch_size
        bucket_offset = current_epoch_samples // self.data_parallel_size
        start = self.data_parallel_rank * bucket_size
        g = torch.Generator()
        g.manual_seed(self.epoch)
        order = torch.randperm(bucket_size, generator=g).tolist()
        batch = []
        for x in order[bucket_offset:]:
            batch.append(start + x)
            if len(batch) == self.local_minibatch_size:
                self.consumed_samples += self.local_minibatch_times_data_parallel_size
                yield batch
                batch = []
