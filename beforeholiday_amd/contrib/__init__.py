"""Contrib modules (reference: apex/contrib): xentropy, focal_loss, index_mul_2d, transducer,
multihead_attn, optimizers (ZeRO DistributedFusedAdam/LAMB), clip_grad, groupbn, peer_memory,
sparsity (ASP), bottleneck, conv_bias_relu, layer_norm, fmha."""
