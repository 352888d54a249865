"""Fused multi-head attention over variable-length packed sequences
(reference: apex/contrib/fmha/fmha.py:34-76, ``fmhalib``: sm80-only kernels for seq <= 512, head 64).

Input ``qkv`` [total_tokens, 3, heads, head_dim] with ``cu_seqlens`` [batch + 1]. Sequences are
scattered into a padded batch once. Head size 64 (the reference's only head size; its sequence
cap is 512) runs the MFMA fused attention kernels (kernels/attn.hip: whole-row kernels up to 128
tokens, flash kernels beyond; key padding mask, Philox dropout regenerated in backward) on a
[S, B*heads, 3, 64] padded layout; other head sizes use batched GEMMs (hipBLASLt) around the fused mask + softmax + dropout kernel of
``contrib.multihead_attn``. Any sequence length up to 4096 and any head size.
"""
import torch

from ..multihead_attn._core import MASK_PAD, FusedSelfAttnFn, MaskSoftmaxDropoutFn, _fused_ok


def fmha_varlen(qkv, cu_seqlens, p_dropout, max_s, is_training):
    total, three, h, d = qkv.shape
    assert three == 3
    lens = (cu_seqlens[1:] - cu_seqlens[:-1]).tolist()
    B = len(lens)
    S = max(max(lens), 1) if lens else 1
    pos = torch.arange(S, device=qkv.device).unsqueeze(0)
    valid = pos < torch.tensor(lens, device=qkv.device).unsqueeze(1)  # [B, S]
    if _fused_ok(qkv, d, S):
        # [S, B, heads, 3, d] -> q/k/v are [S, B*heads, d] views with a uniform batch*head stride
        padded = qkv.new_zeros(S, B, h, 3, d)
        tok = valid.t().nonzero(as_tuple=True)  # (t, b) of every valid token
        src = qkv[(cu_seqlens[:-1][tok[1]] + tok[0]).long()]  # [n, 3, h, d]
        padded[tok[0], tok[1]] = src.permute(0, 2, 1, 3)
        ctx = FusedSelfAttnFn.apply(padded.view(S, B * h, 3, d), h, d ** -0.5, ~valid, MASK_PAD, p_dropout,
                                    is_training)
        ctx = ctx.view(S, B, h, d).transpose(0, 1)  # [B, S, h, d]
        return ctx[valid]
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
