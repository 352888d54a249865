"""Encoder-decoder multi-head attention module
(reference: apex/contrib/multihead_attn/encdec_multihead_attn.py:19-190)."""
import math

import torch
from torch import nn
from torch.nn import Parameter

from ...normalization.fused_layer_norm import FusedLayerNorm
from . import _core
from .functions import encdec_attn_func, fast_encdec_attn_func, fast_encdec_attn_norm_add_func


class EncdecMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False, impl="fast"):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.bias = bias
        self.include_norm_add = include_norm_add
        self.impl = impl
        self.scaling = self.head_dim ** -0.5
        if impl not in ("fast", "default"):
            raise AssertionError(f"Unsupported impl: {impl} !")
        if impl == "fast" and bias:
            raise AssertionError("Fast impl does not support bias")
        self.in_proj_weight_q = Parameter(torch.empty(embed_dim, embed_dim))
        self.in_proj_weight_kv = Parameter(torch.empty(2 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            self.in_proj_bias_q = Parameter(torch.empty(embed_dim))
            self.in_proj_bias_kv = Parameter(torch.empty(2 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            self.in_proj_bias_q = self.in_proj_bias_kv = self.out_proj_bias = None
        if include_norm_add:
            if impl == "fast":
                self.lyr_nrm_gamma_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm_beta_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm = None
            else:
                self.lyr_nrm_gamma_weights = self.lyr_nrm_beta_weights = None
                self.lyr_nrm = FusedLayerNorm(embed_dim)
        self.reset_parameters()
        if include_norm_add:
            self.attn_func = fast_encdec_attn_norm_add_func if impl == "fast" else encdec_attn_func
        else:
            self.attn_func = fast_encdec_attn_func if impl == "fast" else encdec_attn_func

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight_q)
        # [2h, h] initialised like an [h, h] matrix: gain sqrt(1.5)
        nn.init.xavier_uniform_(self.in_proj_weight_kv, gain=math.sqrt(1.5))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            nn.init.constant_(self.in_proj_bias_q, 0.0)
            nn.init.constant_(self.in_proj_bias_kv, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)
        if self.include_norm_add:
            if self.impl == "fast":
                nn.init.ones_(self.lyr_nrm_gamma_weights)
                nn.init.zeros_(self.lyr_nrm_beta_weights)
            else:
                self.lyr_nrm.reset_parameters()

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None, is_training=True):
        if key_padding_mask is not None:
            assert attn_mask is None, "ERROR attn_mask and key_padding_mask should not be both defined!"
            mask = key_padding_mask
        else:
            mask = attn_mask
        use_time = attn_mask is not None
        if self.include_norm_add:
            if self.impl == "fast":
                out = self.attn_func(use_time, is_training, self.num_heads, query, key, self.lyr_nrm_gamma_weights,
                                     self.lyr_nrm_beta_weights, self.in_proj_weight_q, self.in_proj_weight_kv,
                                     self.out_proj_weight, mask, self.dropout)
            else:
                ln = self.lyr_nrm(query)
                out = self.attn_func(use_time, is_training, self.num_heads, self.scaling, ln, key,
                                     self.in_proj_weight_q, self.in_proj_weight_kv, self.out_proj_weight,
                                     self.in_proj_bias_q, self.in_proj_bias_kv, self.out_proj_bias, mask, self.dropout)
                out = _core.dropout_add(out, query, self.dropout, is_training)
        elif self.impl == "fast":
            out = self.attn_func(use_time, is_training, self.num_heads, query, key, self.in_proj_weight_q,
                                 self.in_proj_weight_kv, self.out_proj_weight, mask, self.dropout)
        else:
            out = self.attn_func(use_time, is_training, self.num_heads, self.scaling, query, key,
                                 self.in_proj_weight_q, self.in_proj_weight_kv, self.out_proj_weight,
                                 self.in_proj_bias_q, self.in_proj_bias_kv, self.out_proj_bias, mask, self.dropout)
        return out, None
