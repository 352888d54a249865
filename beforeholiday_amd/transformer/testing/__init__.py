"""Test harness for model-parallel code: toy models, step functions, distributed test bases, standalone
GPT/BERT (reference: apex/transformer/testing)."""
