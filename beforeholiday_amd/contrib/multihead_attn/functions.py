"""Function-level entry points with the reference's names and argument orders
(reference: apex/contrib/multihead_attn/{self,encdec}_multihead_attn_func.py,
fast_{self,encdec}_multihead_attn{,_norm_add}_func.py, mask_softmax_dropout_func.py)."""
from . import _core


def self_attn_func(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
                   output_biases, mask, is_additive_mask, dropout_prob):
    """'default' implementation."""
    return _core.self_attention(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights,
                                input_biases, output_biases, mask, is_additive_mask, dropout_prob)


def fast_self_attn_func(use_time_mask, is_training, heads, inputs, input_weights, output_weights, input_biases,
                        output_biases, pad_mask, mask_additive, dropout_prob):
    hd = inputs.size(2) // heads
    return _core.self_attention(use_time_mask, is_training, heads, hd ** -0.5, inputs, input_weights,
                                output_weights, input_biases, output_biases, pad_mask, mask_additive, dropout_prob)


def fast_self_attn_norm_add_func(use_time_mask, is_training, heads, inputs, lyr_nrm_gamma_weights,
                                 lyr_nrm_beta_weights, input_weights, output_weights, pad_mask, dropout_prob):
    """inputs + dropout(attention(LayerNorm(inputs)))."""
    hd = inputs.size(2) // heads
    ln = _core.layer_norm(inputs, lyr_nrm_gamma_weights, lyr_nrm_beta_weights)
    out = _core.self_attention(use_time_mask, is_training, heads, hd ** -0.5, ln, input_weights, output_weights,
                               None, None, pad_mask, False, dropout_prob)
    return _core.dropout_add(out, inputs, dropout_prob, is_training)


def encdec_attn_func(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q, input_weights_kv,
                     output_weights, input_biases_q, input_biases_kv, output_biases, mask, dropout_prob):
    return _core.encdec_attention(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                                  input_weights_kv, output_weights, input_biases_q, input_biases_kv, output_biases,
                                  mask, dropout_prob)


def fast_encdec_attn_func(use_time_mask, is_training, heads, inputs_q, inputs_kv, input_weights_q, input_weights_kv,
                          output_weights, pad_mask, dropout_prob):
    hd = inputs_q.size(2) // heads
    return _core.encdec_attention(use_time_mask, is_training, heads, hd ** -0.5, inputs_q, inputs_kv,
                                  input_weights_q, input_weights_kv, output_weights, None, None, None, pad_mask,
                                  dropout_prob)


def fast_encdec_attn_norm_add_func(use_time_mask, is_training, heads, inputs_q, inputs_kv, lyr_nrm_gamma_weights,
                                   lyr_nrm_beta_weights, input_weights_q, input_weights_kv, output_weights, pad_mask,
                                   dropout_prob):
    hd = inputs_q.size(2) // heads
    ln = _core.layer_norm(inputs_q, lyr_nrm_gamma_weights, lyr_nrm_beta_weights)
    out = _core.encdec_attention(use_time_mask, is_training, heads, hd ** -0.5, ln, inputs_kv, input_weights_q,
                                 input_weights_kv, output_weights, None, None, None, pad_mask, dropout_prob)
    return _core.dropout_add(out, inputs_q, dropout_prob, is_training)


def fast_mask_softmax_dropout_func(is_training, heads, inputs, pad_mask, mask_additive, dropout_prob):
    """inputs [B*heads, sq, sk] (already scaled) -> dropout(softmax(mask(inputs)))."""
    mode = _core.mask_mode_for(pad_mask, False, mask_additive)
    return _core.MaskSoftmaxDropoutFn.apply(inputs, pad_mask, mode, heads, dropout_prob, is_training)
