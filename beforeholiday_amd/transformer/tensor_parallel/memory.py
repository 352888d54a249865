"""Named preallocated activation buffers (reference: apex/transformer/tensor_parallel/memory.py:25-151).

A ``MemoryBuffer`` is one flat allocation handed out as views in FIFO order and reset wholesale, so
checkpointed activations live in a single HBM region instead of many caching-allocator blocks.
"""
import torch

_MEM_BUFFS = {}


def allocate_mem_buff(name, numel, dtype, track_usage):
    assert name not in _MEM_BUFFS, f"memory buffer {name} already allocated."
    _MEM_BUFFS[name] = MemoryBuffer(name, numel, dtype, track_usage)
    return _MEM_BUFFS[name]


def get_mem_buff(name):
    return _MEM_BUFFS[name]


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class MemoryBuffer:
    def __init__(self, name, numel, dtype, track_usage):
        if torch.distributed.is_initialized() and torch.distributed.get_rank() == 0:
            elsize = torch.tensor([], dtype=dtype).element_size()
            print(f"> building the {name} memory buffer with {numel} num elements and {dtype} dtype "
                  f"({numel * elsize / 2**20:.1f} MB)...", flush=True)
        self.name = name
        self.numel = numel
        self.dtype = dtype
        self.data = torch.empty(numel, dtype=dtype, device=_device(), requires_grad=False)
        self._start = 0
        self.track_usage = track_usage
        if track_usage:
            self.in_use_value = 0.0
            self.total_value = 0.0

    def reset(self):
        self._start = 0

    def is_in_use(self):
        return self._start > 0

    def numel_in_use(self):
        return self._start

    def add(self, tensor):
        assert tensor.dtype == self.dtype, f"Input tensor type {tensor.dtype} different from buffer type {self.dtype}"
        n = tensor.numel()
        end = self._start + n
        assert end <= self.numel, f"Not enough memory left in the buffer ({n} > {self.numel - self._start})"
        view = self.data[self._start:end].view_as(tensor)
        self._start = end
        view.copy_(tensor)
        return view

    def get_data(self):
        if self.track_usage:
            self.in_use_value += float(self._start)
            self.total_value += float(self.numel)
        return self.data[:self._start]

    def print_average_usage(self):
        assert self.track_usage, "You need to enable track usage."
        if torch.distributed.is_initialized() and torch.distributed.get_rank() == 0:
            print(f" > usage of {self.name} memory buffer: {self.in_use_value * 100.0 / self.total_value:.2f} %",
                  flush=True)


class RingMemBuffer:
    """A ring of memory buffers."""

    def __init__(self, name, num_buffers, numel, dtype, track_usage):
        self.num_buffers = num_buffers
        self.buffers = [allocate_mem_buff(f"{name} {i}", numel, dtype, track_usage) for i in range(num_buffers)]
        self._index = -1

    def get_next_buffer(self):
        self._index = (self._index + 1) % self.num_buffers
        buff = self.buffers[self._index]
        assert not buff.is_in_use(), "buffer is already in use."
        return buff
