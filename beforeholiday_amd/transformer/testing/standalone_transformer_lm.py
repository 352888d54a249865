"""Standalone Megatron transformer LM (reference: apex/transformer/testing/standalone_transformer_lm.py).
The implementation lives in :mod:`beforeholiday_amd.models.transformer_lm`."""
from ...models.transformer_lm import *  # noqa: F401,F403
from ...models.transformer_lm import (BertLMHead, CoreAttention, Embedding, MegatronModule, ParallelAttention,  # noqa
                                      ParallelMLP, ParallelTransformer, ParallelTransformerLayer, Pooler,
                                      TransformerLanguageModel, bias_dropout_add, get_language_model,
                                      get_linear_layer, init_method_normal, module_size, parallel_lm_logits,
                                      post_language_model_processing, scaled_init_method_normal)
