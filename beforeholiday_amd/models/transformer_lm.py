"""Megatron-style transformer language model built from this package's TP/SP layers, fused LayerNorm,
fused scale-mask-softmax and vocab-parallel cross-entropy (reference:
apex/transformer/testing/standalone_transformer_lm.py:45-1574, standalone_gpt.py, standalone_bert.py).

Differences from the reference, MI355X-first:
* configuration is an explicit :class:`TransformerConfig` (the reference reads a global argparse
  namespace); ``transformer.testing.global_vars`` still provides the reference's ``get_args`` flow;
* bias + GELU runs as one HIP pass forward and one fused dGELU + bias-grad pass backward
  (``ops.fused_dense``), the reference's ``bias_gelu_fusion`` flag is honoured instead of ignored;
* attention scores use one batched GEMM per layer ([b*np, sq, hn] x [b*np, hn, sk]) straight into
  the fused softmax kernel (any sk up to 32768, causal or padding mask).
Layout of activations is [sequence, batch, hidden] throughout, like Megatron.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import config as _config
import torch.nn.functional as F

from ..normalization import ResidualGradLink
from ..ops import fused_dense as _fd
from ..transformer import parallel_state, tensor_parallel
from ..transformer.enums import AttnMaskType, AttnType, LayerType, ModelType
from ..transformer.functional import FusedScaleMaskSoftmax
from ..transformer.layers import FusedLayerNorm as LayerNorm
from ..transformer.utils import divide


@dataclass
class TransformerConfig:
    hidden_size: int = 1024
    num_layers: int = 24
    num_attention_heads: int = 16
    ffn_hidden_size: Optional[int] = None
    kv_channels: Optional[int] = None
    vocab_size: int = 50304
    max_position_embeddings: int = 1024
    num_tokentypes: int = 0
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    layernorm_epsilon: float = 1e-5
    init_method_std: float = 0.02
    apply_residual_connection_post_layernorm: bool = False
    apply_query_key_layer_scaling: bool = True
    attention_softmax_in_fp32: bool = False
    masked_softmax_fusion: bool = True
    bias_gelu_fusion: bool = True
    openai_gelu: bool = False
    fp32_residual_connection: bool = False
    params_dtype: torch.dtype = torch.float32
    fp16: bool = False
    bf16: bool = False
    sequence_parallel: bool = False
    use_cpu_initialization: bool = False
    gradient_accumulation_fusion: bool = False
    activations_checkpoint_method: Optional[str] = None  # None | "uniform" | "block"
    activations_checkpoint_num_layers: int = 1
    pooler: bool = False
    bert_binary_head: bool = True

    def __post_init__(self):
        if self.ffn_hidden_size is None:
            self.ffn_hidden_size = 4 * self.hidden_size
        if self.kv_channels is None:
            assert self.hidden_size % self.num_attention_heads == 0
            self.kv_channels = self.hidden_size // self.num_attention_heads


def init_method_normal(sigma):
    def init_(tensor):
        return torch.nn.init.normal_(tensor, mean=0.0, std=sigma)
    return init_


def scaled_init_method_normal(sigma, num_layers):
    std = sigma / math.sqrt(2.0 * num_layers)

    def init_(tensor):
        return torch.nn.init.normal_(tensor, mean=0.0, std=std)
    return init_


def attention_mask_func(attention_scores: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
    return attention_scores.masked_fill_(attention_mask, -10000.0)


def _flash_mask(attention_mask, b, sq):
    """The padding mask of the flash path once per forward, not once per layer: the [b, sq, sq]
    uint8 copy and its packed bits (fused_attention.flash_mask_bits) are cached on the mask tensor
    that every layer receives (invalidated by an in-place change of it)."""
    hit = getattr(attention_mask, "_bh_flash_mask", None)
    if hit is not None and hit[0] == attention_mask._version and hit[1].shape == (b, sq, sq):
        return hit[1], hit[2]
    from .._native import submodule

    mask = attention_mask.expand(b, 1, sq, sq).reshape(b, sq, sq).to(torch.uint8).contiguous()
    bits = submodule("fused_attention").flash_mask_bits(mask)
    attention_mask._bh_flash_mask = (attention_mask._version, mask, bits)
    return mask, bits


def _device(config=None):
    if (config is not None and config.use_cpu_initialization) or not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def get_linear_layer(rows, columns, init_method, params_dtype=torch.float32, device=None):
    layer = torch.nn.Linear(rows, columns, dtype=params_dtype, device=device)
    init_method(layer.weight)
    with torch.no_grad():
        layer.bias.zero_()
    return layer


def param_is_not_shared(param: torch.Tensor) -> bool:
    return not getattr(param, "shared", False)


class _BiasGeLU(torch.autograd.Function):
    """gelu(x + bias): one add + one activation pass forward; backward is ONE fused
    dGELU + bias-grad pass (kernels/dense.hip)."""

    @staticmethod
    def forward(ctx, x, bias):
        pre = x + bias
        ctx.save_for_backward(pre)
        return _fd.bias_act_forward(pre, None, _fd.ACT_GELU)

    @staticmethod
    def backward(ctx, dy):
        (pre,) = ctx.saved_tensors
        dx, db = _fd.act_backward(dy.contiguous(), pre, _fd.ACT_GELU, True)
        return dx, db


def bias_gelu_impl(x, bias):
    return _BiasGeLU.apply(x, bias)


class _FusedGeluMLP(torch.autograd.Function):
    """This rank's MLP shard  y = GELU(x W1^T + b1) W2^T  on the MFMA GEMM (kernels/gemm.hip):
    bias + GELU run in the first GEMM's epilogue (pre-activation kept as aux), and in backward the
    dGELU and the b1 gradient run in the epilogue of the W2 dgrad GEMM. The weight-gradient and
    input-gradient GEMMs are plain hipBLASLt GEMMs. TP collectives stay outside (ParallelMLP)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2):
        from .._native import submodule

        gm = submodule("gemm")
        x2d = x.reshape(-1, x.size(-1))
        inter, pre = gm.linear_act(x2d, w1, b1, _fd.ACT_GELU, True)
        y = torch.mm(inter, w2.t())
        ctx.save_for_backward(x2d, pre, inter, w1, w2)
        ctx.in_shape = x.shape
        return y.view(*x.shape[:-1], w2.size(0))

    @staticmethod
    def backward(ctx, dy):
        from .._native import submodule

        x2d, pre, inter, w1, w2 = ctx.saved_tensors
        dy2d = dy.reshape(-1, dy.size(-1)).contiguous()
        dw2 = _fd.weight_grad(dy2d, inter)
        gm = submodule("gemm")
        w2t = gm.transpose(w2) if w2.size(0) % 8 == 0 and w2.size(1) % 8 == 0 else w2.t().contiguous()
        dpre, db1 = gm.linear_dact(dy2d, w2t, pre, _fd.ACT_GELU, True)
        dw1 = _fd.weight_grad(dpre, x2d)
        dx = torch.mm(dpre, w1).view(ctx.in_shape)
        return dx, dw1, db1, dw2


def _fused_mlp_ok(x, mlp) -> bool:
    import os

    c, r = mlp.dense_h_to_4h, mlp.dense_4h_to_h
    return (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and mlp.bias_gelu_fusion
            and c.weight.dtype == x.dtype and r.weight.dtype == x.dtype and c.bias is not None
            and not c.gradient_accumulation_fusion and not r.gradient_accumulation_fusion
            and _config.get().fused_mlp)


def openai_gelu(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * x * (1.0 + 0.044715 * x * x)))


class MegatronModule(torch.nn.Module):
    """Adds tied-embedding handling across pipeline stages."""

    def __init__(self, share_word_embeddings: bool = True):
        super().__init__()
        self.share_word_embeddings = share_word_embeddings

    def state_dict_for_save_checkpoint(self, destination=None, prefix="", keep_vars=False):
        return self.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)

    def word_embeddings_weight(self):
        if self.pre_process:
            return self.language_model.embedding.word_embeddings.weight
        if not self.share_word_embeddings:
            raise Exception("word_embeddings_weight() called for last stage, but share_word_embeddings is false")
        return self.word_embeddings.weight

    def initialize_word_embeddings(self, init_method_normal_fn, config: TransformerConfig):
        """On the last stage create a copy of the word embeddings (zeroed, then overwritten by the
        first stage's values through one all-reduce over the embedding group)."""
        if not self.share_word_embeddings:
            raise Exception("initialize_word_embeddings() was called but share_word_embeddings is false")
        if parallel_state.get_pipeline_model_parallel_world_size() == 1:
            return
        if parallel_state.is_pipeline_last_stage() and not self.pre_process:
            self._word_embeddings_for_head_key = "word_embeddings_for_head"
            self.word_embeddings = tensor_parallel.VocabParallelEmbedding(
                config.vocab_size, config.hidden_size, init_method=init_method_normal_fn(config.init_method_std),
                params_dtype=config.params_dtype, use_cpu_initialization=config.use_cpu_initialization)
            with torch.no_grad():
                self.word_embeddings.weight.zero_()
            self.word_embeddings.weight.shared = True
        if torch.distributed.is_initialized() and parallel_state.is_rank_in_embedding_group():
            torch.distributed.all_reduce(self.word_embeddings_weight().data,
                                         group=parallel_state.get_embedding_group())


class ParallelMLP(MegatronModule):
    """h -> 4h (column parallel) -> GELU -> h (row parallel)."""

    def __init__(self, config: TransformerConfig, init_method, output_layer_init_method):
        super().__init__()
        self.dense_h_to_4h = tensor_parallel.ColumnParallelLinear(
            config.hidden_size, config.ffn_hidden_size, gather_output=False, init_method=init_method,
            skip_bias_add=True, params_dtype=config.params_dtype, use_cpu_initialization=config.use_cpu_initialization,
            sequence_parallel_enabled=config.sequence_parallel,
            no_async_tensor_model_parallel_allreduce=config.sequence_parallel,
            gradient_accumulation_fusion=config.gradient_accumulation_fusion)
        self.bias_gelu_fusion = config.bias_gelu_fusion and not config.openai_gelu
        self.activation_func = openai_gelu if config.openai_gelu else F.gelu
        self.dense_4h_to_h = tensor_parallel.RowParallelLinear(
            config.ffn_hidden_size, config.hidden_size, input_is_parallel=True, init_method=output_layer_init_method,
            skip_bias_add=True, params_dtype=config.params_dtype, use_cpu_initialization=config.use_cpu_initialization,
            sequence_parallel_enabled=config.sequence_parallel,
            gradient_accumulation_fusion=config.gradient_accumulation_fusion)

    def forward(self, hidden_states):
        if _fused_mlp_ok(hidden_states, self):
            # same collectives as ColumnParallelLinear -> RowParallelLinear, one fused compute core
            c, r = self.dense_h_to_4h, self.dense_4h_to_h
            if c.sequence_parallel_enabled:
                x = tensor_parallel.mappings.gather_from_sequence_parallel_region(hidden_states)
            else:
                x = tensor_parallel.mappings.copy_to_tensor_model_parallel_region(hidden_states)
            y = _FusedGeluMLP.apply(x, c.weight, c.bias, r.weight)
            if r.sequence_parallel_enabled:
                y = tensor_parallel.mappings.reduce_scatter_to_sequence_parallel_region(y)
            else:
                y = tensor_parallel.mappings.reduce_from_tensor_model_parallel_region(y)
            return y, r.bias
        inter, bias = self.dense_h_to_4h(hidden_states)
        if self.bias_gelu_fusion:
            inter = bias_gelu_impl(inter, bias)
        else:
            inter = self.activation_func(inter + bias)
        return self.dense_4h_to_h(inter)


class CoreAttention(MegatronModule):
    """softmax(Q K^T / sqrt(d) [masked]) V for [sq, b, np, hn] inputs of this TP rank's heads."""

    def __init__(self, config: TransformerConfig, layer_number: int, attn_mask_type=AttnMaskType.padding):
        super().__init__()
        self.fp16, self.bf16 = config.fp16, config.bf16
        self.apply_query_key_layer_scaling = config.apply_query_key_layer_scaling
        self.attention_softmax_in_fp32 = config.attention_softmax_in_fp32 or self.apply_query_key_layer_scaling
        self.layer_number = max(1, layer_number)
        self.attn_mask_type = attn_mask_type
        self.sequence_parallel = config.sequence_parallel
        projection_size = config.kv_channels * config.num_attention_heads
        world = parallel_state.get_tensor_model_parallel_world_size()
        self.hidden_size_per_partition = divide(projection_size, world)
        self.hidden_size_per_attention_head = divide(projection_size, config.num_attention_heads)
        self.num_attention_heads_per_partition = divide(config.num_attention_heads, world)
        coeff = self.layer_number if self.apply_query_key_layer_scaling else None
        self.norm_factor = math.sqrt(self.hidden_size_per_attention_head)
        if coeff:
            self.norm_factor *= coeff
        self.scale_mask_softmax = FusedScaleMaskSoftmax(self.fp16, self.bf16, attn_mask_type,
                                                        config.masked_softmax_fusion, attention_mask_func,
                                                        self.attention_softmax_in_fp32, coeff)
        self.attention_dropout = torch.nn.Dropout(config.attention_dropout)

    def flash_ok(self, x, hn) -> bool:
        """MFMA flash attention (kernels/attn.hip) for head size 64 on fp16 / bf16 GPU tensors."""
        import os

        return (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and hn == 64
                and _config.get().flash_attn)

    def flash(self, qkv, attention_mask):
        """qkv [sq, b*np, 3, 64] (the fused QKV projection output, viewed) -> context [sq, b, np*64].
        Same math as forward(): scale 1/sqrt(hn) (the query-key layer-scaling coefficient cancels),
        padding masks fill -10000 like attention_mask_func, causal masks are implicit, attention
        dropout is Philox-regenerated in backward; d(qkv) comes back in the projection layout."""
        from ..contrib.multihead_attn._core import MASK_CAUSAL, MASK_FULL, MASK_NONE, FusedSelfAttnFn

        sq, bnp = qkv.shape[0], qkv.shape[1]
        b = bnp // self.num_attention_heads_per_partition
        if self.attn_mask_type == AttnMaskType.causal:
            mode, mask, fill = MASK_CAUSAL, None, float("-inf")
        elif attention_mask is not None:
            mode, fill = MASK_FULL, -10000.0
            mask, bits = _flash_mask(attention_mask, b, sq)
        else:
            mode, mask, fill = MASK_NONE, None, float("-inf")
        p = self.attention_dropout.p if self.training else 0.0
        ctx = FusedSelfAttnFn.apply(qkv, self.num_attention_heads_per_partition,
                                    1.0 / math.sqrt(self.hidden_size_per_attention_head), mask, mode, p,
                                    self.training, fill, bits if mode == MASK_FULL else None)
        return ctx.view(sq, b, self.hidden_size_per_partition)

    def forward(self, query, key, value, attention_mask):
        sq, b, np_, hn = query.shape
        sk = key.size(0)
        q = query.reshape(sq, b * np_, hn).transpose(0, 1)  # [b*np, sq, hn]
        k = key.reshape(sk, b * np_, hn).permute(1, 2, 0)  # [b*np, hn, sk]
        scores = torch.bmm(q, k).mul_(1.0 / self.norm_factor).view(b, np_, sq, sk)
        probs = self.scale_mask_softmax(scores, attention_mask)
        if self.sequence_parallel or parallel_state.get_tensor_model_parallel_world_size() > 1:
            with tensor_parallel.get_cuda_rng_tracker().fork():
                probs = self.attention_dropout(probs)
        else:
            probs = self.attention_dropout(probs)
        v = value.reshape(sk, b * np_, hn).transpose(0, 1)  # [b*np, sk, hn]
        ctx = torch.bmm(probs.view(b * np_, sq, sk), v)  # [b*np, sq, hn]
        ctx = ctx.view(b, np_, sq, hn).permute(2, 0, 1, 3).contiguous()
        return ctx.view(sq, b, self.hidden_size_per_partition)


class ParallelAttention(MegatronModule):
    """Self-attention (fused QKV projection) or cross-attention; output projection row parallel."""

    def __init__(self, config: TransformerConfig, init_method, output_layer_init_method, layer_number,
                 attention_type=AttnType.self_attn, attn_mask_type=AttnMaskType.padding):
        super().__init__()
        self.attention_type = attention_type
        projection_size = config.kv_channels * config.num_attention_heads
        world = parallel_state.get_tensor_model_parallel_world_size()
        self.hidden_size_per_attention_head = divide(projection_size, config.num_attention_heads)
        self.num_attention_heads_per_partition = divide(config.num_attention_heads, world)
        common = dict(gather_output=False, init_method=init_method, params_dtype=config.params_dtype,
                      use_cpu_initialization=config.use_cpu_initialization,
                      sequence_parallel_enabled=config.sequence_parallel,
                      no_async_tensor_model_parallel_allreduce=config.sequence_parallel,
                      gradient_accumulation_fusion=config.gradient_accumulation_fusion)
        if attention_type == AttnType.self_attn:
            self.query_key_value = tensor_parallel.ColumnParallelLinear(config.hidden_size, 3 * projection_size,
                                                                        **common)
        else:
            self.query = tensor_parallel.ColumnParallelLinear(config.hidden_size, projection_size, **common)
            self.key_value = tensor_parallel.ColumnParallelLinear(config.hidden_size, 2 * projection_size, **common)
        self.core_attention = CoreAttention(config, layer_number, attn_mask_type)
        self.dense = tensor_parallel.RowParallelLinear(
            projection_size, config.hidden_size, input_is_parallel=True, init_method=output_layer_init_method,
            skip_bias_add=True, params_dtype=config.params_dtype, use_cpu_initialization=config.use_cpu_initialization,
            sequence_parallel_enabled=config.sequence_parallel,
            gradient_accumulation_fusion=config.gradient_accumulation_fusion)

    def forward(self, hidden_states, attention_mask, encoder_output=None):
        np_, hn = self.num_attention_heads_per_partition, self.hidden_size_per_attention_head
        if self.attention_type == AttnType.self_attn:
            mixed, _ = self.query_key_value(hidden_states)
            if self.core_attention.flash_ok(mixed, hn):
                qkv = mixed.view(mixed.shape[0], mixed.shape[1] * np_, 3, hn)
                return self.dense(self.core_attention.flash(qkv, attention_mask))
            mixed = mixed.view(*mixed.shape[:-1], np_, 3 * hn)
            q, k, v = tensor_parallel.split_tensor_along_last_dim(mixed, 3)
        else:
            kv, _ = self.key_value(encoder_output)
            kv = kv.view(*kv.shape[:-1], np_, 2 * hn)
            k, v = tensor_parallel.split_tensor_along_last_dim(kv, 2)
            q, _ = self.query(hidden_states)
            q = q.view(*q.shape[:-1], np_, hn)
        ctx = self.core_attention(q, k, v, attention_mask)
        return self.dense(ctx)


def bias_dropout_add(x, bias, residual, prob: float, training: bool, model_parallel: bool = False, resid_link=None):
    """residual + dropout(x + bias): one fused HIP pass on GPU (ops/fused_dense.py), PyTorch on CPU."""
    return _fd.bias_dropout_add(x, bias, residual, prob, training, model_parallel, resid_link)


class ParallelTransformerLayer(MegatronModule):
    """LN -> attention -> bias-dropout-add -> LN -> MLP -> bias-dropout-add (pre-LN)."""

    def __init__(self, config: TransformerConfig, init_method, output_layer_init_method, layer_number,
                 layer_type=LayerType.encoder, self_attn_mask_type=AttnMaskType.padding):
        super().__init__()
        self.layer_number = layer_number
        self.layer_type = layer_type
        self.apply_residual_connection_post_layernorm = config.apply_residual_connection_post_layernorm
        self.fp32_residual_connection = config.fp32_residual_connection
        self.hidden_dropout = config.hidden_dropout
        self.sequence_parallel = config.sequence_parallel
        ln = dict(eps=config.layernorm_epsilon, sequence_parallel_enabled=config.sequence_parallel)
        self.input_layernorm = LayerNorm(config.hidden_size, **ln)
        self.self_attention = ParallelAttention(config, init_method, output_layer_init_method, layer_number,
                                                AttnType.self_attn, self_attn_mask_type)
        self.post_attention_layernorm = LayerNorm(config.hidden_size, **ln)
        if layer_type == LayerType.decoder:
            self.inter_attention = ParallelAttention(config, init_method, output_layer_init_method, layer_number,
                                                     AttnType.cross_attn)
            self.post_inter_attention_layernorm = LayerNorm(config.hidden_size, **ln)
        self.mlp = ParallelMLP(config, init_method, output_layer_init_method)

    def _bda(self, out, bias, residual, link=None):
        # sequence parallel: each TP rank holds a different sequence shard -> its own dropout mask
        # (Megatron forks the model-parallel RNG here); otherwise the replicas must agree
        return bias_dropout_add(out, bias, residual, self.hidden_dropout, self.training, self.sequence_parallel,
                                link)

    def _link(self, x):
        """Pre-LN: x feeds both the LayerNorm and the residual add, so its two gradients are summed by
        the LayerNorm backward kernel (normalization.ResidualGradLink; Config.ln_residual_grad)."""
        if (self.apply_residual_connection_post_layernorm or not _config.get().ln_residual_grad or not x.is_cuda
                or not x.requires_grad or not torch.is_grad_enabled()):
            return None
        return ResidualGradLink()

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None):
        link = self._link(hidden_states)
        ln_out = self.input_layernorm(hidden_states, resid_link=link)
        attn_out, attn_bias = self.self_attention(ln_out, attention_mask)
        residual = ln_out if self.apply_residual_connection_post_layernorm else hidden_states
        ln_in = self._bda(attn_out, attn_bias, residual, link)
        link = self._link(ln_in) if self.layer_type != LayerType.decoder else None
        ln_out = self.post_attention_layernorm(ln_in, resid_link=link)
        if self.layer_type == LayerType.decoder:
            attn_out, attn_bias = self.inter_attention(ln_out, enc_dec_attn_mask, encoder_output=encoder_output)
            residual = ln_out if self.apply_residual_connection_post_layernorm else ln_in
            ln_in = self._bda(attn_out, attn_bias, residual)
            ln_out = self.post_inter_attention_layernorm(ln_in)
        mlp_out, mlp_bias = self.mlp(ln_out)
        residual = ln_out if self.apply_residual_connection_post_layernorm else ln_in
        return self._bda(mlp_out, mlp_bias, residual, link)


def get_num_layers(config: TransformerConfig, is_encoder_and_decoder_model: bool = False) -> int:
    pp = parallel_state.get_pipeline_model_parallel_world_size()
    if pp > 1:
        assert config.num_layers % pp == 0, "num_layers must be divisible by pipeline_model_parallel_size"
        return config.num_layers // pp
    return config.num_layers


class ParallelTransformer(MegatronModule):
    """This stage's slice of the layer stack (+ final LN on the last stage)."""

    def __init__(self, config: TransformerConfig, init_method, output_layer_init_method,
                 layer_type=LayerType.encoder, self_attn_mask_type=AttnMaskType.padding, post_layer_norm=True,
                 pre_process=True, post_process=True):
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.post_layer_norm = post_layer_norm
        self.input_tensor = None
        self.sequence_parallel = config.sequence_parallel
        self.checkpoint_method = config.activations_checkpoint_method
        self.checkpoint_num_layers = config.activations_checkpoint_num_layers
        self.num_layers = get_num_layers(config)
        vpp = parallel_state.get_virtual_pipeline_model_parallel_world_size()
        if vpp is not None:
            assert config.num_layers % vpp == 0
            self.num_layers = self.num_layers // vpp
            offset = (parallel_state.get_virtual_pipeline_model_parallel_rank() * (config.num_layers // vpp) +
                      parallel_state.get_pipeline_model_parallel_rank() * self.num_layers)
        else:
            offset = parallel_state.get_pipeline_model_parallel_rank() * self.num_layers
        self.layers = torch.nn.ModuleList([
            ParallelTransformerLayer(config, init_method, output_layer_init_method, i + 1 + offset, layer_type,
                                     self_attn_mask_type) for i in range(self.num_layers)])
        if post_process and post_layer_norm:
            self.final_layernorm = LayerNorm(config.hidden_size, eps=config.layernorm_epsilon,
                                             sequence_parallel_enabled=config.sequence_parallel)

    def set_input_tensor(self, input_tensor):
        self.input_tensor = input_tensor

    def _checkpointed_forward(self, hidden_states, attention_mask, encoder_output, enc_dec_attn_mask):
        def custom(start, end):
            def fwd(x, mask, enc, encmask):
                for layer in self.layers[start:end]:
                    x = layer(x, mask, enc, encmask)
                return x
            return fwd
        n = self.checkpoint_num_layers
        if self.checkpoint_method == "uniform":
            for l in range(0, self.num_layers, n):
                hidden_states = tensor_parallel.checkpoint(custom(l, l + n), False, hidden_states, attention_mask,
                                                           encoder_output, enc_dec_attn_mask)
        else:  # block: checkpoint the first n layers only
            for l in range(self.num_layers):
                if l < n:
                    hidden_states = tensor_parallel.checkpoint(custom(l, l + 1), False, hidden_states,
                                                               attention_mask, encoder_output, enc_dec_attn_mask)
                else:
                    hidden_states = custom(l, l + 1)(hidden_states, attention_mask, encoder_output,
                                                     enc_dec_attn_mask)
        return hidden_states

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None):
        if not self.pre_process:
            hidden_states = self.input_tensor
        if self.checkpoint_method is not None and self.training:
            hidden_states = self._checkpointed_forward(hidden_states, attention_mask, encoder_output,
                                                       enc_dec_attn_mask)
        else:
            for layer in self.layers:
                hidden_states = layer(hidden_states, attention_mask, encoder_output, enc_dec_attn_mask)
        if self.post_process and self.post_layer_norm:
            hidden_states = self.final_layernorm(hidden_states)
        return hidden_states


class Embedding(MegatronModule):
    """word (vocab parallel) + position (+ tokentype) embeddings, dropout; [b, s] -> [s, b, h]."""

    def __init__(self, config: TransformerConfig, init_method, num_tokentypes=0):
        super().__init__()
        self.hidden_size = config.hidden_size
        self.init_method = init_method
        self.num_tokentypes = num_tokentypes
        self.sequence_parallel = config.sequence_parallel
        self.fp32_residual_connection = config.fp32_residual_connection
        self.word_embeddings = tensor_parallel.VocabParallelEmbedding(
            config.vocab_size, config.hidden_size, init_method=init_method, params_dtype=config.params_dtype,
            use_cpu_initialization=config.use_cpu_initialization)
        dev = None if config.use_cpu_initialization or not torch.cuda.is_available() else torch.cuda.current_device()
        self.position_embeddings = torch.nn.Embedding(config.max_position_embeddings, config.hidden_size,
                                                      dtype=config.params_dtype, device=dev)
        init_method(self.position_embeddings.weight)
        if num_tokentypes > 0:
            self.tokentype_embeddings = torch.nn.Embedding(num_tokentypes, config.hidden_size,
                                                           dtype=config.params_dtype, device=dev)
            init_method(self.tokentype_embeddings.weight)
        else:
            self.tokentype_embeddings = None
        self.embedding_dropout = torch.nn.Dropout(config.hidden_dropout)

    def forward(self, input_ids, position_ids, tokentype_ids=None):
        emb = self.word_embeddings(input_ids) + _fd.embedding(position_ids, self.position_embeddings.weight)
        if tokentype_ids is not None:
            assert self.tokentype_embeddings is not None
            emb = emb + _fd.embedding(tokentype_ids, self.tokentype_embeddings.weight)
        emb = emb.transpose(0, 1).contiguous()
        if self.fp32_residual_connection:
            emb = emb.float()
        if self.sequence_parallel:
            emb = tensor_parallel.scatter_to_sequence_parallel_region(emb)
            with tensor_parallel.get_cuda_rng_tracker().fork():
                return self.embedding_dropout(emb)
        return self.embedding_dropout(emb)


class Pooler(MegatronModule):
    def __init__(self, hidden_size, init_method, sequence_parallel=False, params_dtype=torch.float32, device=None):
        super().__init__()
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method, params_dtype, device)
        self.sequence_parallel = sequence_parallel

    def forward(self, hidden_states, sequence_index=0):
        if self.sequence_parallel:
            hidden_states = tensor_parallel.gather_from_sequence_parallel_region(hidden_states,
                                                                                 to_model_parallel=False)
        return torch.tanh(self.dense(hidden_states[sequence_index, :, :]))


class TransformerLanguageModel(MegatronModule):
    def __init__(self, config: TransformerConfig, init_method, output_layer_init_method, encoder_attn_mask_type,
                 num_tokentypes=0, add_pooler=False, pre_process=True, post_process=True):
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.add_pooler = add_pooler
        if pre_process:
            self.embedding = Embedding(config, init_method, num_tokentypes)
        self.encoder = ParallelTransformer(config, init_method, output_layer_init_method,
                                           self_attn_mask_type=encoder_attn_mask_type, pre_process=pre_process,
                                           post_process=post_process)
        if post_process and add_pooler:
            self.pooler = Pooler(config.hidden_size, init_method, config.sequence_parallel, config.params_dtype,
                                 _device(config))

    def set_input_tensor(self, input_tensor):
        if not isinstance(input_tensor, list):
            input_tensor = [input_tensor]
        self.encoder.set_input_tensor(input_tensor[0])

    def forward(self, enc_input_ids, enc_position_ids, enc_attn_mask, tokentype_ids=None, pooling_sequence_index=0):
        enc_in = self.embedding(enc_input_ids, enc_position_ids, tokentype_ids) if self.pre_process else None
        out = self.encoder(enc_in, enc_attn_mask)
        if self.post_process and self.add_pooler:
            return out, self.pooler(out, pooling_sequence_index)
        return out


def get_language_model(config, num_tokentypes, add_pooler, encoder_attn_mask_type, init_method=None,
                       scaled_init_method=None, pre_process=True, post_process=True):
    init_method = init_method or init_method_normal(config.init_method_std)
    scaled_init_method = scaled_init_method or scaled_init_method_normal(config.init_method_std, config.num_layers)
    lm = TransformerLanguageModel(config, init_method, scaled_init_method, encoder_attn_mask_type, num_tokentypes,
                                  add_pooler, pre_process, post_process)
    return lm, "language_model"


def parallel_lm_logits(input_, word_embeddings_weight, parallel_output, bias=None, sequence_parallel=False):
    """[s, b, h] x [V/tp, h]^T -> vocab-parallel logits (gathered if not ``parallel_output``)."""
    if sequence_parallel:
        input_parallel = tensor_parallel.gather_from_sequence_parallel_region(input_, to_model_parallel=True)
    else:
        input_parallel = tensor_parallel.copy_to_tensor_model_parallel_region(input_)
    logits = F.linear(input_parallel, word_embeddings_weight, bias)
    if parallel_output:
        return logits
    return tensor_parallel.gather_from_tensor_model_parallel_region(logits)


def post_language_model_processing(lm_output, labels, logit_weights, parallel_output, fp16_lm_cross_entropy,
                                   sequence_parallel=False):
    output = parallel_lm_logits(lm_output, logit_weights, parallel_output, sequence_parallel=sequence_parallel)
    if labels is None:
        return output.transpose(0, 1).contiguous()  # [b, s, V/tp]
    labels = labels.transpose(0, 1).contiguous()  # [s, b]
    if fp16_lm_cross_entropy:
        assert output.dtype == torch.half
        loss = tensor_parallel.vocab_parallel_cross_entropy(output, labels)
    elif output.is_cuda:
        # fp32 math inside the kernels and an fp32 loss, without materialising fp32 logits
        loss = tensor_parallel.vocab_parallel_cross_entropy(output, labels, loss_dtype=torch.float32)
    else:
        loss = tensor_parallel.vocab_parallel_cross_entropy(output.float(), labels)
    return loss.transpose(0, 1).contiguous()  # [b, s]


class GPTModel(MegatronModule):
    """Causal LM: forward(input_ids [b,s], position_ids [b,s], attention_mask, labels=None) ->
    per-token loss [b, s] (labels given) or vocab-parallel logits."""

    def __init__(self, config: TransformerConfig, num_tokentypes=0, parallel_output=True, pre_process=True,
                 post_process=True, fp16_lm_cross_entropy=False):
        super().__init__(share_word_embeddings=True)
        self.config = config
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        self.fp16_lm_cross_entropy = fp16_lm_cross_entropy
        self.language_model, self._language_model_key = get_language_model(
            config, num_tokentypes, False, AttnMaskType.causal, pre_process=pre_process, post_process=post_process)
        self.initialize_word_embeddings(init_method_normal, config)

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, input_ids, position_ids, attention_mask, labels=None, tokentype_ids=None):
        lm_output = self.language_model(input_ids, position_ids, attention_mask, tokentype_ids=tokentype_ids)
        if self.post_process:
            return post_language_model_processing(lm_output, labels, self.word_embeddings_weight(),
                                                  self.parallel_output, self.fp16_lm_cross_entropy,
                                                  self.config.sequence_parallel)
        return lm_output


def bert_extended_attention_mask(attention_mask):
    """[b, s] padding mask (1 = keep) -> [b, 1, s, s] boolean mask (True = masked)."""
    m_b1s = attention_mask.unsqueeze(1)
    m_bs1 = attention_mask.unsqueeze(2)
    return (m_b1s * m_bs1).unsqueeze(1) < 0.5


def bert_position_ids(token_ids):
    s = token_ids.size(1)
    return torch.arange(s, dtype=torch.long, device=token_ids.device).unsqueeze(0).expand_as(token_ids)


class BertLMHead(MegatronModule):
    """dense -> GELU -> LayerNorm -> tied vocab-parallel projection (+ bias)."""

    def __init__(self, mpu_vocab_size, hidden_size, init_method, layernorm_epsilon, parallel_output,
                 sequence_parallel=False, params_dtype=torch.float32, device=None):
        super().__init__()
        self.bias = torch.nn.Parameter(torch.zeros(mpu_vocab_size, dtype=params_dtype, device=device))
        tensor_parallel.set_tensor_model_parallel_attributes(self.bias, True, 0, 1)
        self.parallel_output = parallel_output
        self.sequence_parallel = sequence_parallel
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method, params_dtype, device)
        self.layernorm = LayerNorm(hidden_size, eps=layernorm_epsilon).to(device)

    def forward(self, hidden_states, word_embeddings_weight):
        h = self.layernorm(F.gelu(self.dense(hidden_states)))
        return parallel_lm_logits(h, word_embeddings_weight, self.parallel_output, bias=self.bias,
                                  sequence_parallel=self.sequence_parallel)


class BertModel(MegatronModule):
    """Masked LM (+ optional next-sentence binary head)."""

    def __init__(self, config: TransformerConfig, num_tokentypes=2, add_binary_head=True, parallel_output=True,
                 pre_process=True, post_process=True, fp16_lm_cross_entropy=False):
        super().__init__(share_word_embeddings=True)
        self.config = config
        self.add_binary_head = add_binary_head
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        self.fp16_lm_cross_entropy = fp16_lm_cross_entropy
        init_method = init_method_normal(config.init_method_std)
        self.language_model, self._language_model_key = get_language_model(
            config, num_tokentypes, add_binary_head, AttnMaskType.padding, pre_process=pre_process,
            post_process=post_process)
        self.initialize_word_embeddings(init_method_normal, config)
        if post_process:
            self.lm_head = BertLMHead(self.word_embeddings_weight().size(0), config.hidden_size, init_method,
                                      config.layernorm_epsilon, parallel_output, config.sequence_parallel,
                                      config.params_dtype, _device(config))
            self.binary_head = (get_linear_layer(config.hidden_size, 2, init_method, config.params_dtype,
                                                 _device(config)) if add_binary_head else None)

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, bert_model_input, attention_mask, tokentype_ids=None, lm_labels=None):
        ext_mask = bert_extended_attention_mask(attention_mask)
        position_ids = bert_position_ids(bert_model_input) if self.pre_process else None
        lm_output = self.language_model(bert_model_input, position_ids, ext_mask, tokentype_ids=tokentype_ids)
        if not self.post_process:
            return lm_output
        if self.add_binary_head:
            lm_output, pooled = lm_output
        else:
            pooled = None
        lm_logits = self.lm_head(lm_output, self.word_embeddings_weight())
        binary_logits = self.binary_head(pooled) if self.binary_head is not None and pooled is not None else None
        if lm_labels is None:
            return lm_logits.transpose(0, 1).contiguous(), binary_logits
        labels = lm_labels.transpose(0, 1).contiguous()
        if self.fp16_lm_cross_entropy:
            loss = tensor_parallel.vocab_parallel_cross_entropy(lm_logits, labels)
        elif lm_logits.is_cuda:  # fp32 math in the kernels, fp32 loss, no fp32 copy of the logits
            loss = tensor_parallel.vocab_parallel_cross_entropy(lm_logits, labels, loss_dtype=torch.float32)
        else:
            loss = tensor_parallel.vocab_parallel_cross_entropy(lm_logits.float(), labels)
        loss = loss.transpose(0, 1).contiguous()
        return loss, binary_logits


def module_size(m: torch.nn.Module, only_trainable: bool = False):
    params = [p for p in m.parameters() if p.requires_grad or not only_trainable]
    return sum(p.numel() for p in {id(p): p for p in params}.values())


def finalize_model_grads(model_chunks) -> None:
    """Cross-rank gradient fix-ups a Megatron training step needs after backward:
    * parameters tagged ``sequence_parallel_enabled`` (LayerNorms, row-parallel biases under SP) hold
      partial grads per sequence shard -> one flat all-reduce over the TP group;
    * the word embedding is tied between the first and last pipeline stage -> all-reduce its grad
      over the embedding group."""
    from ..transformer.layers import allreduce_sequence_parallel_grads
    chunks = model_chunks if isinstance(model_chunks, (list, tuple)) else [model_chunks]
    for m in chunks:
        allreduce_sequence_parallel_grads(m)
    if parallel_state.get_pipeline_model_parallel_world_size() > 1 and parallel_state.is_rank_in_embedding_group(
            ignore_virtual=True):
        if parallel_state.is_pipeline_first_stage(ignore_virtual=True):
            m = chunks[0]
        elif parallel_state.is_pipeline_last_stage(ignore_virtual=True):
            m = chunks[-1]
        else:
            return
        m = getattr(m, "module", m)
        if getattr(m, "share_word_embeddings", False):
            w = m.word_embeddings_weight()
            g = w.main_grad if hasattr(w, "main_grad") else w.grad
            if g is not None:
                torch.distributed.all_reduce(g, group=parallel_state.get_embedding_group())
