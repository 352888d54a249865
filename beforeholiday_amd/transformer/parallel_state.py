"""Model-parallel topology: tensor (TP), pipeline (PP), data (DP) parallel process groups.

Reference: apex/transformer/parallel_state.py:81-682. Rank layout is the Megatron one: TP groups are
blocks of consecutive ranks (on one MI355X node those are GPUs that share direct xGMI links),
PP groups are strided by ``world_size / pp``, DP groups combine the remaining dimension. Also builds
the embedding / position-embedding / relative-position-embedding groups used for tied weights.

On ROCm the "nccl" backend is RCCL; ``default_backend`` / ``p2p_backend`` may be "nccl" or "gloo"
(gloo lets the whole topology run on CPU for tests).
"""
from __future__ import annotations

import logging
from typing import List, Optional, Sequence, Tuple

import torch

_logger = logging.getLogger(__name__)

_TENSOR_MODEL_PARALLEL_GROUP = None
_PIPELINE_MODEL_PARALLEL_GROUP = None
_MODEL_PARALLEL_GROUP = None
_EMBEDDING_GROUP = None
_POSITION_EMBEDDING_GROUP = None
_ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP = None
_DECODER_RELATIVE_POSITION_EMBEDDING_GROUP = None
_DATA_PARALLEL_GROUP = None

_VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = None
_VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_PIPELINE_MODEL_PARALLEL_SPLIT_RANK = None

_MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_TENSOR_MODEL_PARALLEL_RANK = None
_MPU_PIPELINE_MODEL_PARALLEL_RANK = None

_EMBEDDING_GLOBAL_RANKS = None
_POSITION_EMBEDDING_GLOBAL_RANKS = None
_ENCODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS = None
_DECODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS = None
_PIPELINE_GLOBAL_RANKS = None
_DATA_PARALLEL_GLOBAL_RANKS = None


def is_unitialized() -> bool:
    return _DATA_PARALLEL_GROUP is None


def _new_group(ranks, backend):
    return torch.distributed.new_group(list(ranks), backend=backend)


def initialize_model_parallel(tensor_model_parallel_size_: int = 1, pipeline_model_parallel_size_: int = 1,
                              virtual_pipeline_model_parallel_size_: Optional[int] = None,
                              pipeline_model_parallel_split_rank_: Optional[int] = None, *,
                              default_backend: Optional[str] = None, p2p_backend: Optional[str] = None) -> None:
    """Create TP/PP/DP (and embedding) groups. ``world_size`` must be divisible by tp * pp.

    Example, 16 ranks, tp=2, pp=4: TP groups [0,1],[2,3],...; PP groups [0,4,8,12],[1,5,9,13],...;
    DP groups [0,2],[1,3],[4,6],...
    """
    global _DATA_PARALLEL_GROUP, _MODEL_PARALLEL_GROUP, _TENSOR_MODEL_PARALLEL_GROUP
    global _PIPELINE_MODEL_PARALLEL_GROUP, _PIPELINE_GLOBAL_RANKS, _EMBEDDING_GROUP, _EMBEDDING_GLOBAL_RANKS
    global _POSITION_EMBEDDING_GROUP, _POSITION_EMBEDDING_GLOBAL_RANKS
    global _ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP, _DECODER_RELATIVE_POSITION_EMBEDDING_GROUP
    global _ENCODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS, _DECODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK, _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK, _DATA_PARALLEL_GLOBAL_RANKS

    assert torch.distributed.is_initialized()
    assert default_backend is None or default_backend in ("nccl", "ucc", "gloo")
    assert p2p_backend is None or p2p_backend in ("nccl", "ucc", "gloo")
    if "ucc" in (default_backend, p2p_backend):
        check_torch_ucc_availability()
    world_size = torch.distributed.get_world_size()
    tp = min(tensor_model_parallel_size_, world_size)
    pp = min(pipeline_model_parallel_size_, world_size)
    if world_size % (tp * pp) != 0:
        raise RuntimeError(f"`world_size` ({world_size}) is not divisible by tensor_model_parallel_size ({tp}) x "
                           f"pipeline_model_parallel_size ({pp})")
    dp = world_size // (tp * pp)
    if torch.distributed.get_rank() == 0:
        _logger.info("> initializing tensor model parallel with size %d", tp)
        _logger.info("> initializing pipeline model parallel with size %d", pp)
        _logger.info("> initializing data parallel with size %d", dp)
    num_tp_groups = world_size // tp
    num_pp_groups = world_size // pp

    if virtual_pipeline_model_parallel_size_ is not None:
        assert pipeline_model_parallel_size_ > 2, \
            "pipeline-model-parallel size should be greater than 2 with interleaved schedule"
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = 0
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = virtual_pipeline_model_parallel_size_
    if pipeline_model_parallel_split_rank_ is not None:
        _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = pipeline_model_parallel_split_rank_

    rank = torch.distributed.get_rank()

    assert _DATA_PARALLEL_GROUP is None, "data parallel group is already initialized"
    all_dp_ranks = []
    for i in range(pp):
        start, end = i * num_pp_groups, (i + 1) * num_pp_groups
        for j in range(tp):
            ranks = list(range(start + j, end, tp))
            all_dp_ranks.append(ranks)
            group = _new_group(ranks, default_backend)
            if rank in ranks:
                _DATA_PARALLEL_GROUP = group
                _DATA_PARALLEL_GLOBAL_RANKS = ranks

    assert _MODEL_PARALLEL_GROUP is None, "model parallel group is already initialized"
    for i in range(dp):
        ranks = [r[i] for r in all_dp_ranks]
        group = _new_group(ranks, default_backend)
        if rank in ranks:
            _MODEL_PARALLEL_GROUP = group

    assert _TENSOR_MODEL_PARALLEL_GROUP is None, "tensor model parallel group is already initialized"
    for i in range(num_tp_groups):
        ranks = list(range(i * tp, (i + 1) * tp))
        group = _new_group(ranks, default_backend)
        if rank in ranks:
            _TENSOR_MODEL_PARALLEL_GROUP = group

    assert _PIPELINE_MODEL_PARALLEL_GROUP is None, "pipeline model parallel group is already initialized"
    assert _EMBEDDING_GROUP is None, "embedding group is already initialized"
    assert _POSITION_EMBEDDING_GROUP is None, "position embedding group is already initialized"
    split = pipeline_model_parallel_split_rank_
    for i in range(num_pp_groups):
        ranks = list(range(i, world_size, num_pp_groups))
        group = _new_group(ranks, p2p_backend)
        if rank in ranks:
            _PIPELINE_MODEL_PARALLEL_GROUP = group
            _PIPELINE_GLOBAL_RANKS = ranks
        if len(ranks) > 1:
            embedding_ranks = [ranks[0], ranks[-1]]
            position_embedding_ranks = [ranks[0]]
            enc_rel = [ranks[0]]
            dec_rel = [ranks[0]]
            if split is not None:
                enc_rel = ranks[:split]
                dec_rel = ranks[split:]
                if ranks[split] not in embedding_ranks:
                    embedding_ranks = [ranks[0], ranks[split], ranks[-1]]
                if ranks[split] not in position_embedding_ranks:
                    position_embedding_ranks = [ranks[0], ranks[split]]
        else:
            embedding_ranks = ranks
            position_embedding_ranks = ranks
            enc_rel = ranks
            dec_rel = ranks
        g = _new_group(embedding_ranks, default_backend)
        if rank in embedding_ranks:
            _EMBEDDING_GROUP = g
        if rank in ranks:
            _EMBEDDING_GLOBAL_RANKS = embedding_ranks
        g = _new_group(position_embedding_ranks, default_backend)
        if rank in position_embedding_ranks:
            _POSITION_EMBEDDING_GROUP = g
        if rank in ranks:
            _POSITION_EMBEDDING_GLOBAL_RANKS = position_embedding_ranks
        g = _new_group(enc_rel, default_backend)
        if rank in enc_rel:
            _ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP = g
        if rank in ranks:
            _ENCODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS = enc_rel
        g = _new_group(dec_rel, default_backend)
        if rank in dec_rel:
            _DECODER_RELATIVE_POSITION_EMBEDDING_GROUP = g
        if rank in ranks:
            _DECODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS = dec_rel


def get_rank_info() -> Tuple[int, int, int]:
    """(tensor rank, pipeline rank, data rank) or (0,0,0) when uninitialised (log formatter)."""
    if model_parallel_is_initialized():
        return (get_tensor_model_parallel_rank(), get_pipeline_model_parallel_rank(), get_data_parallel_rank())
    return (0, 0, 0)


def model_parallel_is_initialized():
    return not (_TENSOR_MODEL_PARALLEL_GROUP is None or _PIPELINE_MODEL_PARALLEL_GROUP is None or
                _DATA_PARALLEL_GROUP is None)


def get_model_parallel_group():
    assert _MODEL_PARALLEL_GROUP is not None, "model parallel group is not initialized"
    return _MODEL_PARALLEL_GROUP


def get_tensor_model_parallel_group():
    assert _TENSOR_MODEL_PARALLEL_GROUP is not None, "intra_layer_model parallel group is not initialized"
    return _TENSOR_MODEL_PARALLEL_GROUP


def get_pipeline_model_parallel_group():
    assert _PIPELINE_MODEL_PARALLEL_GROUP is not None, "pipeline_model parallel group is not initialized"
    return _PIPELINE_MODEL_PARALLEL_GROUP


def get_data_parallel_group():
    assert _DATA_PARALLEL_GROUP is not None, "data parallel group is not initialized"
    return _DATA_PARALLEL_GROUP


def get_embedding_group():
    assert _EMBEDDING_GROUP is not None, "embedding group is not initialized"
    return _EMBEDDING_GROUP


def get_position_embedding_group():
    assert _POSITION_EMBEDDING_GROUP is not None, "position embedding group is not initialized"
    return _POSITION_EMBEDDING_GROUP


def get_encoder_relative_position_embedding_group():
    assert _ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP is not None, \
        "encoder relative position embedding group is not initialized"
    return _ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP


def get_decoder_relative_position_embedding_group():
    assert _DECODER_RELATIVE_POSITION_EMBEDDING_GROUP is not None, \
        "decoder relative position embedding group is not initialized"
    return _DECODER_RELATIVE_POSITION_EMBEDDING_GROUP


def is_rank_in_embedding_group(ignore_virtual=False):
    rank = torch.distributed.get_rank()
    if ignore_virtual:
        return rank in _EMBEDDING_GLOBAL_RANKS
    if rank in _EMBEDDING_GLOBAL_RANKS:
        if rank == _EMBEDDING_GLOBAL_RANKS[0]:
            return is_pipeline_first_stage(ignore_virtual=False)
        elif rank == _EMBEDDING_GLOBAL_RANKS[-1]:
            return is_pipeline_last_stage(ignore_virtual=False)
        return True
    return False


def is_rank_in_position_embedding_group():
    return torch.distributed.get_rank() in _POSITION_EMBEDDING_GLOBAL_RANKS


def is_rank_in_encoder_relative_position_embedding_group():
    return torch.distributed.get_rank() in _ENCODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS


def is_rank_in_decoder_relative_position_embedding_group():
    return torch.distributed.get_rank() in _DECODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS


def is_pipeline_stage_before_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    if rank is None:
        rank = get_pipeline_model_parallel_rank()
    if _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None:
        return True
    return rank < _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def is_pipeline_stage_after_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    if rank is None:
        rank = get_pipeline_model_parallel_rank()
    if _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None:
        return True
    return rank >= _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def is_pipeline_stage_at_split():
    rank = get_pipeline_model_parallel_rank()
    return is_pipeline_stage_before_split(rank) and is_pipeline_stage_after_split(rank + 1)


def set_tensor_model_parallel_world_size(world_size):
    global _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = world_size


def set_pipeline_model_parallel_world_size(world_size):
    global _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = world_size


def get_tensor_model_parallel_world_size():
    if _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    return torch.distributed.get_world_size(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_world_size():
    if _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    return torch.distributed.get_world_size(group=get_pipeline_model_parallel_group())


def set_tensor_model_parallel_rank(rank):
    global _MPU_TENSOR_MODEL_PARALLEL_RANK
    _MPU_TENSOR_MODEL_PARALLEL_RANK = rank


def set_pipeline_model_parallel_rank(rank):
    global _MPU_PIPELINE_MODEL_PARALLEL_RANK
    _MPU_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_tensor_model_parallel_rank():
    if _MPU_TENSOR_MODEL_PARALLEL_RANK is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_RANK
    return torch.distributed.get_rank(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_rank():
    if _MPU_PIPELINE_MODEL_PARALLEL_RANK is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_RANK
    return torch.distributed.get_rank(group=get_pipeline_model_parallel_group())


def get_pipeline_model_parallel_split_rank():
    return _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def set_pipeline_model_parallel_split_rank(pipeline_model_parallel_split_rank: int):
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK
    _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = pipeline_model_parallel_split_rank


def is_pipeline_first_stage(ignore_virtual=False):
    if not ignore_virtual:
        if get_virtual_pipeline_model_parallel_world_size() is not None and \
                get_virtual_pipeline_model_parallel_rank() != 0:
            return False
    return get_pipeline_model_parallel_rank() == 0


def is_pipeline_last_stage(ignore_virtual=False):
    if not ignore_virtual:
        vws = get_virtual_pipeline_model_parallel_world_size()
        if vws is not None and get_virtual_pipeline_model_parallel_rank() != (vws - 1):
            return False
    return get_pipeline_model_parallel_rank() == (get_pipeline_model_parallel_world_size() - 1)


def get_virtual_pipeline_model_parallel_rank():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK


def set_virtual_pipeline_model_parallel_rank(rank):
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_virtual_pipeline_model_parallel_world_size():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE


def set_virtual_pipeline_model_parallel_world_size(size):
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = size


def get_tensor_model_parallel_src_rank():
    """Global rank of local rank 0 of this rank's TP group."""
    global_rank = torch.distributed.get_rank()
    local_world_size = get_tensor_model_parallel_world_size()
    return (global_rank // local_world_size) * local_world_size


def get_data_parallel_src_rank():
    assert _DATA_PARALLEL_GLOBAL_RANKS is not None, "data parallel group is not initialized"
    return _DATA_PARALLEL_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_first_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    return _PIPELINE_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_last_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    return _PIPELINE_GLOBAL_RANKS[get_pipeline_model_parallel_world_size() - 1]


def get_pipeline_model_parallel_next_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    rank_in_pipeline = get_pipeline_model_parallel_rank()
    world_size = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(rank_in_pipeline + 1) % world_size]


def get_pipeline_model_parallel_prev_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    rank_in_pipeline = get_pipeline_model_parallel_rank()
    world_size = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(rank_in_pipeline - 1) % world_size]


def get_data_parallel_world_size():
    return torch.distributed.get_world_size(group=get_data_parallel_group())


def get_data_parallel_rank():
    return torch.distributed.get_rank(group=get_data_parallel_group())


def destroy_model_parallel():
    """Forget every group (the process groups themselves are destroyed with the default group)."""
    g = globals()
    for name in ("_MODEL_PARALLEL_GROUP", "_TENSOR_MODEL_PARALLEL_GROUP", "_PIPELINE_MODEL_PARALLEL_GROUP",
                 "_DATA_PARALLEL_GROUP", "_EMBEDDING_GROUP", "_POSITION_EMBEDDING_GROUP",
                 "_ENCODER_RELATIVE_POSITION_EMBEDDING_GROUP", "_DECODER_RELATIVE_POSITION_EMBEDDING_GROUP",
                 "_VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK", "_VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE",
                 "_PIPELINE_MODEL_PARALLEL_SPLIT_RANK", "_MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE",
                 "_MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE", "_MPU_TENSOR_MODEL_PARALLEL_RANK",
                 "_MPU_PIPELINE_MODEL_PARALLEL_RANK", "_EMBEDDING_GLOBAL_RANKS", "_POSITION_EMBEDDING_GLOBAL_RANKS",
                 "_ENCODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS",
                 "_DECODER_RELATIVE_POSITION_EMBEDDING_GLOBAL_RANKS", "_PIPELINE_GLOBAL_RANKS",
                 "_DATA_PARALLEL_GLOBAL_RANKS"):
        g[name] = None


def check_torch_ucc_availability() -> None:
    try:
        import torch_ucc  # noqa: F401
    except ImportError:
        raise ImportError("UCC backend requires [torch_ucc](https://github.com/facebookresearch/torch_ucc) but "
                          "not found")
