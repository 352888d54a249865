"""Reference workloads built from this library's layers: ResNet-50 (the headline benchmark) and the
Megatron-style GPT / BERT transformer language models (TP / SP / PP capable)."""
from .resnet import Bottleneck, ResNet, resnet18_like, resnet50, resnet50_fused
from .transformer_lm import (BertModel, GPTModel, TransformerConfig, TransformerLanguageModel, finalize_model_grads)

__all__ = ["ResNet", "Bottleneck", "resnet50", "resnet18_like", "resnet50_fused", "GPTModel", "BertModel",
           "TransformerConfig", "TransformerLanguageModel", "finalize_model_grads"]
