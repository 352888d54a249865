from .encdec_multihead_attn import EncdecMultiheadAttn
from .functions import (encdec_attn_func, fast_encdec_attn_func, fast_encdec_attn_norm_add_func,
                        fast_mask_softmax_dropout_func, fast_self_attn_func, fast_self_attn_norm_add_func,
                        self_attn_func)
from .self_multihead_attn import SelfMultiheadAttn

__all__ = ["SelfMultiheadAttn", "EncdecMultiheadAttn", "fast_mask_softmax_dropout_func", "self_attn_func",
           "fast_self_attn_func", "fast_self_attn_norm_add_func", "encdec_attn_func", "fast_encdec_attn_func",
           "fast_encdec_attn_norm_add_func"]
