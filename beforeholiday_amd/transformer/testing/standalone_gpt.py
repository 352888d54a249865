"""GPT provider for pipeline tests (reference: apex/transformer/testing/standalone_gpt.py:33-111)."""
from ...models.transformer_lm import GPTModel
from .arguments import to_config
from .global_vars import get_args


def gpt_model_provider(pre_process: bool = True, post_process: bool = True, cpu_offload: bool = False) -> GPTModel:
    args = get_args()
    return GPTModel(to_config(args), num_tokentypes=0, parallel_output=True, pre_process=pre_process,
                    post_process=post_process, fp16_lm_cross_entropy=args.fp16_lm_cross_entropy)


__all__ = ["GPTModel", "gpt_model_provider"]
