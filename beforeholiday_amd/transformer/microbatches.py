"""Number-of-microbatches calculators (reference: apex/transformer/microbatches.py:26-195)."""
import logging
from abc import ABC, abstractmethod
from typing import List, Optional

_logger = logging.getLogger(__name__)


def build_num_microbatches_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                      micro_batch_size: int, data_parallel_size: int):
    if rampup_batch_size is None:
        calc = ConstantNumMicroBatches(global_batch_size, micro_batch_size, data_parallel_size)
        if rank == 0:
            _logger.info("setting number of micro-batches to constant %d", calc.get())
        return calc
    assert len(rampup_batch_size) == 3, \
        "expected the following format: --rampup-batch-size <start batch size> <batch size increment> <ramp-up samples>"
    start_batch_size, batch_size_increment, ramup_samples = (int(v) for v in rampup_batch_size)
    if rank == 0:
        _logger.info("will use batch size rampup starting from global batch size %d to global batch size %d with "
                     "batch size increments %d over %d samples.", start_batch_size, global_batch_size,
                     batch_size_increment, ramup_samples)
    return RampupBatchsizeNumMicroBatches(start_batch_size, batch_size_increment, ramup_samples, global_batch_size,
                                          micro_batch_size, data_parallel_size)


class NumMicroBatchesCalculator(ABC):
    def __init__(self):
        self.num_micro_batches = None
        self.current_global_batch_size = None

    def get(self):
        return self.num_micro_batches

    def get_current_global_batch_size(self):
        return self.current_global_batch_size

    @abstractmethod
    def update(self, consumed_samples, consistency_check):
        pass


class ConstantNumMicroBatches(NumMicroBatchesCalculator):
    def __init__(self, global_batch_size, micro_batch_size, data_parallel_size):
        super().__init__()
        per_step = micro_batch_size * data_parallel_size
        assert global_batch_size % per_step == 0, (
            f"global batch size ({global_batch_size}) is not divisible by micro batch size ({micro_batch_size}) "
            f"times data parallel size ({data_parallel_size})")
        self.num_micro_batches = global_batch_size // per_step
        assert self.num_micro_batches >= 1, \
            f"number of micro-batches should be at least 1, got {self.num_micro_batches}."
        self.current_global_batch_size = global_batch_size
        self.micro_batch_size = micro_batch_size

    def update(self, consumed_samples, consistency_check):
        pass


class RampupBatchsizeNumMicroBatches(NumMicroBatchesCalculator):
    """Global batch grows linearly from ``start_batch_size`` by ``batch_size_increment`` steps spread
    evenly over ``ramup_samples`` consumed samples."""

    def __init__(self, start_batch_size, batch_size_increment, ramup_samples, global_batch_size, micro_batch_size,
                 data_parallel_size):
        super().__init__()
        self.micro_batch_size = micro_batch_size
        self.data_parallel_size = data_parallel_size
        self.micro_batch_times_data_parallel_size = micro_batch_size * data_parallel_size
        assert self.micro_batch_times_data_parallel_size > 0
        assert start_batch_size > 0
        self.start_batch_size = start_batch_size
        assert global_batch_size > 0
        self.global_batch_size = global_batch_size
        diff = global_batch_size - start_batch_size
        assert diff >= 0
        assert batch_size_increment > 0
        self.batch_size_increment = batch_size_increment
        assert diff % batch_size_increment == 0, (
            f"expected global batch size interval ({diff}) to be divisible by global batch size increment "
            f"({batch_size_increment})")
        num_increments = diff // batch_size_increment
        self.ramup_samples = ramup_samples
        assert self.ramup_samples >= 0
        self.rampup_samples_per_increment = self.ramup_samples / num_increments if num_increments else 0
        self.update(0, False)

    def update(self, consumed_samples, consistency_check):
        if consumed_samples > self.ramup_samples or self.rampup_samples_per_increment == 0:
            self.current_global_batch_size = self.global_batch_size
        else:
            steps = int(consumed_samples / self.rampup_samples_per_increment)
            self.current_global_batch_size = self.start_batch_size + steps * self.batch_size_increment
            assert self.current_global_batch_size <= self.global_batch_size
        if consistency_check:
            assert self.current_global_batch_size % self.micro_batch_times_data_parallel_size == 0, (
                f"current global batch size ({self.current_global_batch_size}) is not divisible by micro-batch-size "
                f"({self.micro_batch_size}) times data parallel size ({self.data_parallel_size})")
        self.num_micro_batches = self.current_global_batch_size // self.micro_batch_times_data_parallel_size
