"""Vocab-parallel cross-entropy (reference: apex/transformer/tensor_parallel/cross_entropy.py:23-103).

The reference runs three full-size passes and three all-reduces ([s,b] MAX, SUM, SUM) and stores a
softmax copy of the logits. Here each rank makes ONE pass over its vocab shard (HIP kernel
``xentropy_cuda.vocab_parallel_stats``: online max / sum-exp + target logit per row), the ranks
exchange 16 bytes per row in ONE all-gather, and a combine kernel produces the loss and the global
log-sum-exp. Backward recomputes ``softmax - onehot`` from the saved logits and lse
(``xentropy_cuda.backward`` with shard-local labels) — no softmax tensor is kept.
"""
import torch

from ..._native import submodule
from ..parallel_state import (get_tensor_model_parallel_group, get_tensor_model_parallel_rank,
                              get_tensor_model_parallel_world_size)
from .utils import VocabUtility


def _stats_ref(logits2d, target1d, start):
    x = logits2d.float()
    m = x.max(dim=-1).values
    s = torch.exp(x - m.unsqueeze(-1)).sum(dim=-1)
    t = target1d - start
    inside = (t >= 0) & (t < x.size(-1))
    xt = x.gather(1, t.clamp(0, x.size(-1) - 1).unsqueeze(1)).squeeze(1) * inside
    return torch.stack([m, s, xt, torch.zeros_like(m)], dim=1)


def _combine_ref(gathered, out_dtype):
    m, s, xt = gathered[..., 0], gathered[..., 1], gathered[..., 2]
    M = m.max(dim=0).values
    S = (s * torch.exp(m - M)).sum(dim=0)
    lse = M + torch.log(S)
    return (lse - xt.sum(dim=0)).to(out_dtype), lse


class _VocabParallelCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vocab_parallel_logits, target, loss_dtype=None):
        V = vocab_parallel_logits.size(-1)
        rank = get_tensor_model_parallel_rank()
        world = get_tensor_model_parallel_world_size()
        start, _ = VocabUtility.vocab_range_from_per_partition_vocab_size(V, rank, world)
        logits2d = vocab_parallel_logits.contiguous().view(-1, V)
        target1d = target.contiguous().view(-1).long()
        native = vocab_parallel_logits.is_cuda
        if native:
            xent = submodule("xentropy_cuda")
            stats = xent.vocab_parallel_stats(logits2d, target1d, start)
        else:
            stats = _stats_ref(logits2d, target1d, start)
        if world > 1:
            gathered = torch.empty((world,) + tuple(stats.shape), dtype=stats.dtype, device=stats.device)
            torch.distributed.all_gather_into_tensor(gathered.view(-1), stats.view(-1),
                                                     group=get_tensor_model_parallel_group())
        else:
            gathered = stats.unsqueeze(0)
        out_dtype = loss_dtype or vocab_parallel_logits.dtype
        if native:
            loss, lse = xent.vocab_parallel_combine(gathered, out_dtype)
        else:
            loss, lse = _combine_ref(gathered, out_dtype)
        ctx.start = start
        ctx.save_for_backward(logits2d, lse, target1d)
        ctx.shape = vocab_parallel_logits.shape
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, grad_output):
        logits2d, lse, target1d = ctx.saved_tensors
        local = target1d - ctx.start  # out-of-shard labels never match a column
        g = grad_output.contiguous().view(-1)
        if logits2d.is_cuda:
            dx = submodule("xentropy_cuda").backward(g, logits2d, lse, local, 0.0)
        else:
            V = logits2d.size(-1)
            p = torch.exp(logits2d.float() - lse.unsqueeze(-1))
            inside = (local >= 0) & (local < V)
            p[torch.arange(p.size(0))[inside], local[inside]] -= 1.0
            dx = (p * g.float().unsqueeze(-1)).to(logits2d.dtype)
        return dx.view(ctx.shape), None, None


def vocab_parallel_cross_entropy(vocab_parallel_logits, target, loss_dtype=None):
    """Per-token loss of logits sharded along the vocab over the TP group. Shapes [..., V/tp], [...].
    The kernels accumulate in fp32 whatever the logits dtype; ``loss_dtype`` (default: the logits
    dtype) only sets the dtype of the returned loss, so 16-bit logits need no fp32 copy (the
    gradient comes back in the logits dtype)."""
    return _VocabParallelCrossEntropy.apply(vocab_parallel_logits, target, loss_dtype)
