"""Broadcast a batch dict from TP rank 0 to its TP group (reference: apex/transformer/tensor_parallel/data.py:25-122).

Two broadcasts per call: a fixed-width int64 shape table (``_MAX_DATA_DIM`` slots per key, zero
terminated) and one flattened payload of every key, placed on the current device.
"""
import torch

from ..parallel_state import (get_tensor_model_parallel_group, get_tensor_model_parallel_rank,
                              get_tensor_model_parallel_src_rank)

_MAX_DATA_DIM = 5


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _check_data_types(keys, data, target_dtype):
    for key in keys:
        assert data[key].dtype == target_dtype, \
            f"{key} has data type {data[key].dtype} which is different than {target_dtype}"


def _build_key_size_numel_dictionaries(keys, data):
    table = torch.zeros(len(keys) * _MAX_DATA_DIM, dtype=torch.int64)
    if get_tensor_model_parallel_rank() == 0:
        for k, key in enumerate(keys):
            assert data[key].dim() < _MAX_DATA_DIM, "you should increase MAX_DATA_DIM"
            for i, s in enumerate(data[key].size()):
                table[k * _MAX_DATA_DIM + i] = s
    table_dev = table.to(_device())
    torch.distributed.broadcast(table_dev, get_tensor_model_parallel_src_rank(), group=get_tensor_model_parallel_group())
    table = table_dev.cpu().tolist()
    key_size, key_numel, total = {}, {}, 0
    for k, key in enumerate(keys):
        size = []
        for s in table[k * _MAX_DATA_DIM:(k + 1) * _MAX_DATA_DIM]:
            if s <= 0:
                break
            size.append(s)
        numel = 1
        for s in size:
            numel *= s
        key_size[key], key_numel[key] = size, numel
        total += numel
    return key_size, key_numel, total


def broadcast_data(keys, data, datatype):
    """Returns ``{key: tensor}`` on the current device, identical on every rank of the TP group."""
    key_size, key_numel, total = _build_key_size_numel_dictionaries(keys, data)
    if get_tensor_model_parallel_rank() == 0:
        _check_data_types(keys, data, datatype)
        flat = torch.cat([data[key].contiguous().view(-1) for key in keys], dim=0).to(_device())
    else:
        flat = torch.empty(total, device=_device(), dtype=datatype)
    torch.distributed.broadcast(flat, get_tensor_model_parallel_src_rank(), group=get_tensor_model_parallel_group())
    out, off = {}, 0
    for key in keys:
        out[key] = flat.narrow(0, off, key_numel[key]).view(key_size[key])
        off += key_numel[key]
    return out
