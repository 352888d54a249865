"""Attention building blocks shared by the self / encoder-decoder multi-head attention modules
(reference: apex/contrib/multihead_attn/*_func.py, apex/contrib/csrc/multihead_attn/*).

GEMMs (QKV projection, Q·K^T, P·V, output projection) run on hipBLASLt through differentiable
torch ops; the memory-bound middle — mask, softmax, dropout — is ONE HIP pass forward and one
backward (``fast_multihead_attn`` in kernels/mha.hip, dropout regenerated from a Philox seed so no
mask tensor is stored). On CPU the same math runs as torch ops.
"""

import torch
import torch.nn.functional as F

from ... import config
from ..._native import submodule

MASK_NONE, MASK_PAD, MASK_ADDITIVE, MASK_TIME = 0, 1, 2, 3


def _seed():
    """Philox seed for the fused dropout (CPU generator: no device sync). Tensor-parallel ranks hold
    different heads of the same layer, so their streams are decorrelated by the TP rank."""
    s = int(torch.empty((), dtype=torch.int64).random_(0, 2 ** 62).item())
    try:
        from ...transformer import parallel_state

        if parallel_state.model_parallel_is_initialized():
            s ^= (parallel_state.get_tensor_model_parallel_rank() * 0x9E3779B97F4A7C15) & (2 ** 62 - 1)
    except Exception:  # noqa: BLE001 - parallel_state unavailable / uninitialised
        pass
    return s


def _tp_rank() -> int:
    try:
        from ...transformer import parallel_state

        if parallel_state.model_parallel_is_initialized():
            return parallel_state.get_tensor_model_parallel_rank()
    except Exception:  # noqa: BLE001 - parallel_state unavailable / uninitialised
        pass
    return 0


def _seed_pair():
    """(host seed, device step seed or None): device step seeds (utils/graph_rng.py) when a captured step
    is being replayed, the host Philox seed otherwise."""
    from ...utils import graph_rng

    if graph_rng.active():
        return graph_rng.next_salt(_tp_rank()), graph_rng.step_seed()
    return _seed(), None


class MaskSoftmaxDropoutFn(torch.autograd.Function):
    """scores [B*heads, sq, sk] -> dropout(softmax(masked scores))."""

    @staticmethod
    def forward(ctx, scores, mask, mask_mode, heads, p, training):
        native = scores.is_cuda and scores.size(-1) <= submodule("fast_multihead_attn").max_sk()
        ctx.native = native
        ctx.p = p if training else 0.0
        if native:
            seed = _seed()
            sm, dropped = submodule("fast_multihead_attn").mask_softmax_dropout_forward(
                scores, mask, mask_mode, heads, p, seed, 0, training)
            ctx.seed = seed
            ctx.save_for_backward(sm)
            return dropped
        x = scores.float()
        bh, sq, sk = x.shape
        if mask_mode == MASK_TIME:
            x = x.masked_fill(mask.to(torch.bool).view(1, sq, sk), float("-inf"))
        elif mask_mode in (MASK_PAD, MASK_ADDITIVE):
            x = x.view(-1, heads, sq, sk)
            m = mask.view(-1, 1, 1, sk)
            x = x + m.float() if mask_mode == MASK_ADDITIVE else x.masked_fill(m.to(torch.bool), float("-inf"))
            x = x.view(bh, sq, sk)
        sm = torch.softmax(x, dim=-1).nan_to_num(0.0).to(scores.dtype)
        if training and p > 0:
            keep = (torch.rand_like(sm, dtype=torch.float32) >= p)
            out = sm * keep.to(sm.dtype) / (1.0 - p)
        else:
            keep = None
            out = sm
        ctx.save_for_backward(sm, keep)
        return out

    @staticmethod
    def backward(ctx, dy):
        if ctx.native:
            (sm,) = ctx.saved_tensors
            dx = submodule("fast_multihead_attn").mask_softmax_dropout_backward(dy, sm, ctx.p, ctx.seed, 0,
                                                                                  ctx.p > 0)
            return dx, None, None, None, None, None
        sm, keep = ctx.saved_tensors
        g = dy.float()
        if keep is not None:
            g = g * keep.float() / (1.0 - ctx.p)
        smf = sm.float()
        dx = smf * (g - (g * smf).sum(-1, keepdim=True))
        return dx.to(sm.dtype), None, None, None, None, None


def mask_mode_for(mask, use_time_mask, mask_additive):
    if mask is None:
        return MASK_NONE
    if use_time_mask:
        return MASK_TIME
    return MASK_ADDITIVE if mask_additive else MASK_PAD


def attention(q, k, v, heads, scale, mask, mask_mode, p, training):
    """q [sq, B*heads, hd], k/v [sk, B*heads, hd] -> context [sq, B*heads, hd]."""
    scores = torch.baddbmm(q.new_empty(q.size(1), q.size(0), k.size(0)), q.transpose(0, 1),
                           k.transpose(0, 1).transpose(1, 2), beta=0.0, alpha=scale)
    probs = MaskSoftmaxDropoutFn.apply(scores, mask, mask_mode, heads, p, training)
    return torch.bmm(probs, v.transpose(0, 1)).transpose(0, 1)


MASK_FULL, MASK_CAUSAL = 4, 5  # flash-only modes: [B, sq, sk] bool, implicit causal


def _fused_ok(x, hd, sk):
    """MFMA fused attention (kernels/attn.hip): head_dim 64, 16-bit GPU tensors; sk <= 128 runs the
    whole-row kernels, longer sequences the flash (64-key block, online softmax) kernels."""
    if not x.is_cuda or x.dtype not in (torch.float16, torch.bfloat16) or hd != 64:
        return False
    return config.get().mha_fused


def _short_ok(sk, mask_mode, fill):
    return (sk <= submodule("fused_attention").max_sk() and mask_mode <= MASK_TIME and fill == float("-inf")
            and not config.get().attn_flash_only)


class FusedSelfAttnFn(torch.autograd.Function):
    """qkv [s, B*heads, 3, 64] (the QKV projection output, viewed) -> context [s, B*heads, 64].
    Backward writes d(qkv) in the same layout, so the projection's dgrad / wgrad GEMMs consume it
    without any gather of separate dq / dk / dv tensors. ``fill`` is the value of a masked score
    (-inf: MHA semantics, a fully masked row gives zeros; -10000: Megatron semantics). ``bits``:
    the mode-4 mask packed once by ``flash_mask_bits`` (shared by every layer of a forward)."""

    @staticmethod
    def forward(ctx, qkv, heads, scale, mask, mask_mode, p, training, fill=float("-inf"), bits=None):
        seed, sd = _seed_pair()
        ctx.seed_dev = sd
        fa = submodule("fused_attention")
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        short = _short_ok(qkv.size(0), mask_mode, fill) and sd is None  # (device seeds: flash kernels only)
        if short:
            out = fa.forward(q, k, v, mask_mode, mask, heads, scale, p, training, seed)
            lse = torch.empty(0)
        else:
            out, lse = fa.flash_forward(q, k, v, mask_mode, mask, heads, scale, p, training, seed, fill, bits,
                                        seed_dev=sd)
        ctx.save_for_backward(qkv, mask if mask is not None else torch.empty(0), out if not short else torch.empty(0),
                              lse, bits if bits is not None else torch.empty(0))
        ctx.args = (heads, scale, mask_mode, p, training, seed, mask is not None, fill, short, bits is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, mask, out, lse, bits = ctx.saved_tensors
        heads, scale, mask_mode, p, training, seed, has_mask, fill, short, has_bits = ctx.args
        dqkv = torch.empty_like(qkv)
        fa = submodule("fused_attention")
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        m = mask if has_mask else None
        if short:
            fa.backward(dout.contiguous(), q, k, v, mask_mode, m, heads, scale, p, training, seed,
                        dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
        else:
            fa.flash_backward(dout.contiguous(), q, k, v, out, lse, mask_mode, m, heads, scale, p, training, seed,
                              fill, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], bits if has_bits else None,
                              seed_dev=ctx.seed_dev)
        return dqkv, None, None, None, None, None, None, None, None


class FusedEncdecAttnFn(torch.autograd.Function):
    """q [sq, B*heads, 64], kv [sk, B*heads, 2, 64] -> context [sq, B*heads, 64]."""

    @staticmethod
    def forward(ctx, q, kv, heads, scale, mask, mask_mode, p, training):
        seed, sd = _seed_pair()
        ctx.seed_dev = sd
        fa = submodule("fused_attention")
        short = _short_ok(kv.size(0), mask_mode, float("-inf")) and sd is None
        if short:
            out = fa.forward(q, kv[:, :, 0], kv[:, :, 1], mask_mode, mask, heads, scale, p, training, seed)
            lse = torch.empty(0)
        else:
            out, lse = fa.flash_forward(q, kv[:, :, 0], kv[:, :, 1], mask_mode, mask, heads, scale, p, training, seed,
                                        float("-inf"), seed_dev=sd)
        ctx.save_for_backward(q, kv, mask if mask is not None else torch.empty(0), out if not short else torch.empty(0),
                              lse)
        ctx.args = (heads, scale, mask_mode, p, training, seed, mask is not None, short)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, mask, out, lse = ctx.saved_tensors
        heads, scale, mask_mode, p, training, seed, has_mask, short = ctx.args
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        fa = submodule("fused_attention")
        m = mask if has_mask else None
        if short:
            fa.backward(dout.contiguous(), q, kv[:, :, 0], kv[:, :, 1], mask_mode, m, heads, scale, p, training, seed,
                        dq, dkv[:, :, 0], dkv[:, :, 1])
        else:
            fa.flash_backward(dout.contiguous(), q, kv[:, :, 0], kv[:, :, 1], out, lse, mask_mode, m, heads, scale, p,
                              training, seed, float("-inf"), dq, dkv[:, :, 0], dkv[:, :, 1], seed_dev=ctx.seed_dev)
        return dq, dkv, None, None, None, None, None, None


def _linear(x2d, w, b):
    return torch.addmm(b, x2d, w.t()) if b is not None else torch.mm(x2d, w.t())


def self_attention(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
                   output_biases, mask, mask_additive, dropout_prob):
    s, b, e = inputs.shape
    hd = e // heads
    qkv = _linear(inputs.reshape(s * b, e), input_weights, input_biases).view(s, b * heads, 3, hd)
    mode = mask_mode_for(mask, use_time_mask, mask_additive)
    if _fused_ok(qkv, hd, s):
        ctxt = FusedSelfAttnFn.apply(qkv, heads, scale, mask, mode, dropout_prob, is_training)
    else:
        q, k, v = qkv[:, :, 0, :], qkv[:, :, 1, :], qkv[:, :, 2, :]
        ctxt = attention(q, k, v, heads, scale, mask, mode, dropout_prob, is_training)
    out = _linear(ctxt.reshape(s * b, e), output_weights, output_biases)
    return out.view(s, b, e)


def encdec_attention(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                     input_weights_kv, output_weights, input_biases_q, input_biases_kv, output_biases, mask,
                     dropout_prob):
    sq, b, e = inputs_q.shape
    sk = inputs_kv.size(0)
    hd = e // heads
    q = _linear(inputs_q.reshape(sq * b, e), input_weights_q, input_biases_q).view(sq, b * heads, hd)
    kv = _linear(inputs_kv.reshape(sk * b, e), input_weights_kv, input_biases_kv).view(sk, b * heads, 2, hd)
    mode = mask_mode_for(mask, use_time_mask, False)
    if _fused_ok(q, hd, sk):
        ctxt = FusedEncdecAttnFn.apply(q, kv, heads, scale, mask, mode, dropout_prob, is_training)
    else:
        k, v = kv[:, :, 0, :], kv[:, :, 1, :]
        ctxt = attention(q, k, v, heads, scale, mask, mode, dropout_prob, is_training)
    return _linear(ctxt.reshape(sq * b, e), output_weights, output_biases).view(sq, b, e)


def layer_norm(x, gamma, beta):
    from ...normalization.fused_layer_norm import fused_layer_norm_affine
    return fused_layer_norm_affine(x, gamma, beta, (x.size(-1),), 1e-5)


def dropout_add(x, residual, p, training):
    return residual + F.dropout(x, p=p, training=training)
