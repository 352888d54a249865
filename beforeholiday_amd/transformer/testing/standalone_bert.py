"""BERT provider for pipeline tests (reference: apex/transformer/testing/standalone_bert.py:20-255)."""
from ...models.transformer_lm import BertLMHead, BertModel, bert_extended_attention_mask, bert_position_ids
from .arguments import to_config
from .global_vars import get_args


def bert_model_provider(pre_process=True, post_process=True, cpu_offload=False) -> BertModel:
    args = get_args()
    cfg = to_config(args)
    return BertModel(cfg, num_tokentypes=2, add_binary_head=cfg.bert_binary_head, parallel_output=True,
                     pre_process=pre_process, post_process=post_process)


__all__ = ["BertModel", "BertLMHead", "bert_model_provider", "bert_extended_attention_mask", "bert_position_ids"]
