"""Model-parallel RNG state tracking + activation checkpointing
(reference: apex/transformer/tensor_parallel/random.py:48-311).

Two RNG streams: the default device generator (same across a TP group, differs across DP replicas —
dropout outside TP regions) and a named "model-parallel-rng" state that differs per TP rank (dropout
inside TP regions). ``fork()`` swaps the named state in and out of the device generator. When no GPU
is present the CPU default generator plays the device role so the same code runs in gloo tests.
"""
import contextlib

import torch
from torch.utils.checkpoint import detach_variable

from .. import parallel_state
from ..utils import gather_split_1d_tensor, split_tensor_into_1d_equal_chunks
from .memory import allocate_mem_buff

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"

_CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER = None


def _get_device_rng_state():
    return torch.cuda.get_rng_state() if torch.cuda.is_available() else torch.get_rng_state()


def _set_cuda_rng_state(new_state, device=-1):
    """Restore the device generator state (CPU generator when no GPU)."""
    if not torch.cuda.is_available():
        torch.set_rng_state(new_state)
        return
    if device == -1:
        device = torch.device("cuda")
    elif isinstance(device, str):
        device = torch.device(device)
    elif isinstance(device, int):
        device = torch.device("cuda", device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    torch.cuda.default_generators[idx].set_state(new_state)


def _device_manual_seed(seed):
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
    else:
        torch.manual_seed(seed)


def init_checkpointed_activations_memory_buffer(micro_batch_size, max_position_embeddings, hidden_size,
                                                num_layers, tensor_model_parallel_size,
                                                checkpoint_num_layers, fp16):
    """Preallocate one flat buffer holding the (TP-split) checkpointed layer inputs."""
    global _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER
    per_layer = micro_batch_size * max_position_embeddings * hidden_size // tensor_model_parallel_size
    assert num_layers % checkpoint_num_layers == 0, "number of layers is not divisible by checkpoint-num-layers"
    numel = per_layer * (num_layers // checkpoint_num_layers)
    dtype = torch.half if fp16 else torch.float
    assert _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is None, "checkpointed activations memory buffer is already allocated."
    _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER = allocate_mem_buff("checkpointed activations", numel, dtype,
                                                                track_usage=False)


def reset_checkpointed_activations_memory_buffer():
    if _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is not None:
        _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER.reset()


class CudaRNGStatesTracker:
    """Named device-RNG states; ``fork(name)`` runs a block under that state and saves its advance."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception(f"cuda rng state {name} already exists")
        orig = _get_device_rng_state()
        _device_manual_seed(seed)
        self.states_[name] = _get_device_rng_state()
        _set_cuda_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception(f"cuda rng state {name} is not added")
        orig = _get_device_rng_state()
        _set_cuda_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _get_device_rng_state()
            _set_cuda_rng_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()

# Host-side seed streams for the fused dropout kernels (bias-dropout-add): each call draws a 31-bit
# kernel seed on the CPU (no device sync). "replicated" is seeded identically on every TP rank (TP
# replicas hold the same activations and must drop the same elements); "model-parallel" is seeded per
# TP rank (sequence-parallel shards need independent masks) -- the two roles the device generator and
# the tracker's "model-parallel-rng" state play for torch dropout (reference: random.py:124-311,
# standalone_transformer_lm.py:1009-1014). Saved/restored by CheckpointFunction like the device states.
_DROPOUT_SEED_GENS = {}


def _seed_dropout_streams(seed, tp_seed):
    for name, s in (("replicated", seed), ("model-parallel", tp_seed)):
        g = torch.Generator()
        g.manual_seed(int(s))
        _DROPOUT_SEED_GENS[name] = g


def dropout_seed(model_parallel: bool = False) -> int:
    """Next fused-dropout kernel seed from the replicated or the per-TP-rank stream (falls back to
    the default CPU generator before :func:`model_parallel_cuda_manual_seed` was called)."""
    g = _DROPOUT_SEED_GENS.get("model-parallel" if model_parallel else "replicated")
    return int(torch.randint(0, 2 ** 31 - 1, (1,), generator=g).item())


_GRAPH_RNG_CALLS = "graph_rng.calls"


def get_dropout_seed_states():
    """The fused-dropout seed streams, and (device step seeds, utils/graph_rng.py) the per-step call
    counter that picks the next salt, so a checkpoint recompute redraws the forward's masks."""
    from ...utils import graph_rng

    states = {k: g.get_state() for k, g in _DROPOUT_SEED_GENS.items()}
    if graph_rng.active():
        states[_GRAPH_RNG_CALLS] = graph_rng._calls
    return states


def set_dropout_seed_states(states):
    from ...utils import graph_rng

    for k, st in states.items():
        if k == _GRAPH_RNG_CALLS:
            graph_rng._calls = st
        else:
            _DROPOUT_SEED_GENS.setdefault(k, torch.Generator()).set_state(st)


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    """Seed the DP stream with ``seed`` and the TP stream with ``seed + 2718 + tp_rank``."""
    tp_seed = seed + 2718 + parallel_state.get_tensor_model_parallel_rank()
    _CUDA_RNG_STATE_TRACKER.reset()
    _device_manual_seed(seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, tp_seed)
    _seed_dropout_streams(seed, tp_seed)


class CheckpointFunction(torch.autograd.Function):
    """Activation checkpoint that replays CPU, device and tracker RNG states in the recompute
    (so dropout masks match), optionally keeping only this TP rank's slice of the first input."""

    @staticmethod
    def forward(ctx, run_function, distribute_saved_activations, *args):
        ctx.run_function = run_function
        ctx.distribute_saved_activations = distribute_saved_activations
        ctx.fwd_cpu_rng_state = torch.get_rng_state()
        ctx.fwd_cuda_rng_state = _get_device_rng_state()
        ctx.fwd_cuda_rng_state_tracker = get_cuda_rng_tracker().get_states()
        ctx.fwd_dropout_seed_states = get_dropout_seed_states()
        with torch.no_grad():
            outputs = run_function(*args)
        if distribute_saved_activations:
            ctx.input_0_shape = args[0].shape
            first = split_tensor_into_1d_equal_chunks(args[0].data).clone()
            args = (first,) + tuple(args[1:])
        ctx.save_for_backward(*args)
        return outputs

    @staticmethod
    def backward(ctx, *grads):
        if not torch.autograd._is_checkpoint_valid():
            raise RuntimeError("Checkpointing is not compatible with .grad(), please use .backward() if possible")
        inputs = list(ctx.saved_tensors)
        if ctx.distribute_saved_activations:
            inputs[0] = gather_split_1d_tensor(inputs[0]).view(ctx.input_0_shape)
        bwd_cpu = torch.get_rng_state()
        bwd_dev = _get_device_rng_state()
        bwd_tracker = get_cuda_rng_tracker().get_states()
        bwd_seeds = get_dropout_seed_states()
        torch.set_rng_state(ctx.fwd_cpu_rng_state)
        _set_cuda_rng_state(ctx.fwd_cuda_rng_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_cuda_rng_state_tracker)
        set_dropout_seed_states(ctx.fwd_dropout_seed_states)
        detached = detach_variable(tuple(inputs))
        with torch.enable_grad():
            outputs = ctx.run_function(*detached)
        torch.set_rng_state(bwd_cpu)
        _set_cuda_rng_state(bwd_dev)
        get_cuda_rng_tracker().set_states(bwd_tracker)
        set_dropout_seed_states(bwd_seeds)
        if isinstance(outputs, torch.Tensor):
            outputs = (outputs,)
        pairs = [(o, g) for o, g in zip(outputs, grads) if isinstance(o, torch.Tensor) and o.requires_grad]
        torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None) + tuple(x.grad if isinstance(x, torch.Tensor) else x for x in detached)


def checkpoint(function, distribute_saved_activations, *args):
    """Checkpoint ``function(*args)``: forward without saving activations, recompute in backward."""
    return CheckpointFunction.apply(function, distribute_saved_activations, *args)
