"""Self multi-head attention module (reference: apex/contrib/multihead_attn/self_multihead_attn.py:19-270).
Inputs are [time, batch, channel]; ``impl`` 'fast' (fused mask-softmax-dropout kernel, scale
head_dim^-0.5 inside) or 'default' (same kernels, explicit scaling); ``include_norm_add`` adds
pre-LayerNorm and a dropout-residual."""
import math

import torch
from torch import nn
from torch.nn import Parameter

from ...normalization.fused_layer_norm import FusedLayerNorm
from . import _core
from .functions import fast_self_attn_func, fast_self_attn_norm_add_func, self_attn_func


class SelfMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False, impl="fast",
                 separate_qkv_params=False, mask_additive=False):
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
        self.separate_qkv_params = separate_qkv_params
        self.mask_additive = mask_additive
        if mask_additive:
            assert not include_norm_add, "additive mask not supported with layer norm"
            assert impl == "default" or (impl == "fast" and bias), \
                "additive mask not supported for fast mode without bias"
        if impl not in ("fast", "default"):
            raise AssertionError(f"Unsupported impl: {impl} !")
        if separate_qkv_params:
            self.q_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.k_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.v_weight = Parameter(torch.empty(embed_dim, embed_dim))
        else:
            self.in_proj_weight = Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            if separate_qkv_params:
                self.q_bias = Parameter(torch.empty(embed_dim))
                self.k_bias = Parameter(torch.empty(embed_dim))
                self.v_bias = Parameter(torch.empty(embed_dim))
            else:
                self.in_proj_bias = Parameter(torch.empty(3 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            if separate_qkv_params:
                self.q_bias = self.k_bias = self.v_bias = None
            else:
                self.in_proj_bias = None
            self.out_proj_bias = None
        if include_norm_add:
            if impl == "fast":
                self.lyr_nrm_gamma_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm_beta_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm = None
            else:
                self.lyr_nrm_gamma_weights = None
                self.lyr_nrm_beta_weights = None
                self.lyr_nrm = FusedLayerNorm(embed_dim)
        self.reset_parameters()
        if include_norm_add:
            self.attn_func = fast_self_attn_norm_add_func if impl == "fast" else self_attn_func
        else:
            self.attn_func = fast_self_attn_func if impl == "fast" else self_attn_func

    def reset_parameters(self):
        if self.separate_qkv_params:
            nn.init.xavier_uniform_(self.q_weight)
            nn.init.xavier_uniform_(self.k_weight)
            nn.init.xavier_uniform_(self.v_weight)
        else:
            # [3h, h] initialised like an [h, h] matrix: gain sqrt(2)
            nn.init.xavier_uniform_(self.in_proj_weight, gain=math.sqrt(2))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            if self.separate_qkv_params:
                nn.init.constant_(self.q_bias, 0.0)
                nn.init.constant_(self.k_bias, 0.0)
                nn.init.constant_(self.v_bias, 0.0)
            else:
                nn.init.constant_(self.in_proj_bias, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)
        if self.include_norm_add:
            if self.impl == "fast":
                nn.init.ones_(self.lyr_nrm_gamma_weights)
                nn.init.zeros_(self.lyr_nrm_beta_weights)
            else:
                self.lyr_nrm.reset_parameters()

    def _input_weights(self):
        if not self.separate_qkv_params:
            return self.in_proj_weight, self.in_proj_bias
        h, d, e = self.num_heads, self.head_dim, self.embed_dim
        w = torch.cat([self.q_weight.view(h, 1, d, e), self.k_weight.view(h, 1, d, e),
                       self.v_weight.view(h, 1, d, e)], dim=1).reshape(3 * e, e)
        b = None
        if self.bias:
            b = torch.cat([self.q_bias.view(h, 1, d), self.k_bias.view(h, 1, d), self.v_bias.view(h, 1, d)],
                          dim=1).reshape(3 * e)
        return w, b

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None, is_training=True):
        """query [T, B, C]; key_padding_mask [B, S] (1 = pad) or attn_mask [T, S] (1 = masked)."""
        w, b = self._input_weights()
        if key_padding_mask is not None:
            assert attn_mask is None, "ERROR attn_mask and key_padding_mask should not be both defined!"
            mask = key_padding_mask
        elif attn_mask is not None:
            assert not self.mask_additive, "additive mask not supported for time mask"
            mask = attn_mask
        else:
            mask = None
        use_time = attn_mask is not None
        if self.include_norm_add:
            if self.impl == "fast":
                out = self.attn_func(use_time, is_training, self.num_heads, query, self.lyr_nrm_gamma_weights,
                                     self.lyr_nrm_beta_weights, w, self.out_proj_weight, mask, self.dropout)
            else:
                ln = self.lyr_nrm(query)
                out = self.attn_func(use_time, is_training, self.num_heads, self.scaling, ln, w, self.out_proj_weight,
                                     b, self.out_proj_bias, mask, self.mask_additive, self.dropout)
                out = _core.dropout_add(out, query, self.dropout, is_training)
        elif self.impl == "fast":
            out = self.attn_func(use_time, is_training, self.num_heads, query, w, self.out_proj_weight, b,
                                 self.out_proj_bias, mask, self.mask_additive, self.dropout)
        else:
            out = self.attn_func(use_time, is_training, self.num_heads, self.scaling, query, w, self.out_proj_weight,
                                 b, self.out_proj_bias, mask, self.mask_additive, self.dropout)
        return out, None
