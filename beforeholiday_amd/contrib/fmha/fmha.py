"""Fused multi-head attention over variable-length packed sequences
(reference: apex/contrib/fmha/fmha.py:34-76, ``fmhalib`` fwd / bwd taking ``cu_seqlens``,
apex/contrib/csrc/fmha/fmha_api.cpp:358-360; sm80-only kernels for seq <= 512, head 64).

Input ``qkv`` [total_tokens, 3, heads, head_dim] with ``cu_seqlens`` int32 [batch + 1] and the
caller's bound ``max_s`` on the lengths. Head size 64 on the GPU runs the MFMA flash kernels
(kernels/attn.hip, 32x32x16 tiles, online softmax, Philox dropout regenerated in backward) straight
on the packed tokens: every (sequence, head) problem rebases its q / k / v / o pointers by
``cu_seqlens[b]`` on the device and bounds its rows by the sequence length (``varlen_rebase``), so
there is no padding copy, no host read of the lengths, and the call is capturable in a HIP graph.
The backward writes d(qkv) in the packed layout. Other head sizes / CPU: padded batched GEMMs around
the fused mask + softmax + dropout kernel of ``contrib.multihead_attn`` (that path reads the lengths on
the host).
"""
import torch

from ..._native import submodule
from ..multihead_attn._core import MASK_PAD, MaskSoftmaxDropoutFn, _fused_ok, _seed


class FlashVarlenFn(torch.autograd.Function):
    """qkv [total, 3, heads, 64] (packed) -> context [total, heads, 64]."""

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, max_s, p_dropout, is_training, causal=False):
        fa = submodule("fused_attention")
        seed = _seed()
        scale = qkv.size(-1) ** -0.5
        cu = cu_seqlens.to(device=qkv.device, dtype=torch.int32).contiguous()
        out, lse = fa.flash_varlen_forward(qkv[:, 0], qkv[:, 1], qkv[:, 2], cu, int(max_s), causal, scale,
                                           float(p_dropout), bool(is_training), seed)
        ctx.save_for_backward(qkv, cu, out, lse)
        ctx.args = (int(max_s), causal, scale, float(p_dropout), bool(is_training), seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, cu, out, lse = ctx.saved_tensors
        max_s, causal, scale, p, training, seed = ctx.args
        dqkv = torch.empty_like(qkv)
        submodule("fused_attention").flash_varlen_backward(
            dout.contiguous(), qkv[:, 0], qkv[:, 1], qkv[:, 2], out, lse, cu, max_s, causal, scale, p, training, seed,
            dqkv[:, 0], dqkv[:, 1], dqkv[:, 2])
        return dqkv, None, None, None, None, None


def _aligned(qkv):
    return qkv.stride(-1) == 1 and qkv.stride(0) % 8 == 0 and qkv.stride(1) % 8 == 0 and qkv.stride(2) % 8 == 0 \
        and qkv.data_ptr() % 16 == 0


def fmha_varlen(qkv, cu_seqlens, p_dropout, max_s, is_training, causal=False):
    total, three, h, d = qkv.shape
    assert three == 3
    if _fused_ok(qkv, d, max_s) and _aligned(qkv):
        return FlashVarlenFn.apply(qkv, cu_seqlens, max_s, p_dropout, is_training, causal)
    assert not causal, "fmha_varlen: causal masking needs the fused (head_dim 64, GPU) path"
    lens = (cu_seqlens[1:] - cu_seqlens[:-1]).tolist()
    B = len(lens)
    S = max(max(lens), 1) if lens else 1
    pos = torch.arange(S, device=qkv.device).unsqueeze(0)
    valid = pos < torch.tensor(lens, device=qkv.device).unsqueeze(1)  # [B, S]
    padded = qkv.new_zeros(B, S, 3, h, d)
    padded = padded.index_put((valid.nonzero(as_tuple=True)), qkv)
    q, k, v = (padded[:, :, i].permute(0, 2, 1, 3) for i in range(3))  # [B, h, S, d]
    scores = torch.matmul(q, k.transpose(-1, -2)).mul_(d ** -0.5).reshape(B * h, S, S)
    probs = MaskSoftmaxDropoutFn.apply(scores, ~valid, MASK_PAD, h, p_dropout, is_training)
    ctx = torch.matmul(probs.view(B, h, S, S), v).permute(0, 2, 1, 3)  # [B, S, h, d]
    return ctx[valid]


class FMHAFun(torch.autograd.Function):
    """Reference-compatible entry point; autograd flows through ``fmha_varlen``."""

    @staticmethod
    def apply(qkv, cu_seqlens, p_dropout, max_s, is_training, zero_tensors=False):
        return fmha_varlen(qkv, cu_seqlens, p_dropout, max_s, is_training)


class FMHA(torch.nn.Module):
    def __init__(self, config):
        super().__init__()
        self.p_dropout = config.attention_probs_dropout_prob
        self.h = config.num_attention_heads
        self.hidden_size = config.hidden_size
        self.d = self.hidden_size // self.h
        assert self.d * self.h == self.hidden_size, "Invalid hidden size/num_heads"

    def forward(self, qkv, cu_seqlens, max_s, is_training=True, zero_tensors=False):
        ctx = FMHAFun.apply(qkv.view(-1, 3, self.h, self.d), cu_seqlens, self.p_dropout, max_s, is_training,
                            zero_tensors)
        return ctx.reshape(-1, self.hidden_size)
