"""Megatron-style command-line arguments for the standalone models
(reference: apex/transformer/testing/arguments.py:23-971 — network size, regularisation, training,
initialisation, learning rate, mixed precision, distributed, data groups; the subset the models and
schedules here consume, plus ``to_config`` producing a :class:`TransformerConfig`)."""
import argparse
import os

import torch


def _add_network_size_args(p):
    g = p.add_argument_group("network size")
    g.add_argument("--num-layers", type=int, default=None)
    g.add_argument("--hidden-size", type=int, default=None)
    g.add_argument("--ffn-hidden-size", type=int, default=None)
    g.add_argument("--num-attention-heads", type=int, default=None)
    g.add_argument("--kv-channels", type=int, default=None)
    g.add_argument("--max-position-embeddings", type=int, default=None)
    g.add_argument("--padded-vocab-size", type=int, default=None)
    g.add_argument("--make-vocab-size-divisible-by", type=int, default=128)
    g.add_argument("--layernorm-epsilon", type=float, default=1e-5)
    g.add_argument("--apply-residual-connection-post-layernorm", action="store_true")
    g.add_argument("--openai-gelu", action="store_true")
    g.add_argument("--onnx-safe", type=bool, default=None)
    g.add_argument("--bert-no-binary-head", action="store_false", dest="bert_binary_head")
    g.add_argument("--num-experts", type=int, default=None)


def _add_regularization_args(p):
    g = p.add_argument_group("regularization")
    g.add_argument("--attention-dropout", type=float, default=0.1)
    g.add_argument("--hidden-dropout", type=float, default=0.1)
    g.add_argument("--weight-decay", type=float, default=0.01)
    g.add_argument("--clip-grad", type=float, default=1.0)
    g.add_argument("--adam-beta1", type=float, default=0.9)
    g.add_argument("--adam-beta2", type=float, default=0.999)
    g.add_argument("--adam-eps", type=float, default=1e-08)
    g.add_argument("--sgd-momentum", type=float, default=0.9)


def _add_training_args(p):
    g = p.add_argument_group("training")
    g.add_argument("--micro-batch-size", type=int, default=None)
    g.add_argument("--global-batch-size", type=int, default=None)
    g.add_argument("--rampup-batch-size", nargs="*", default=None)
    g.add_argument("--checkpoint-activations", action="store_true")
    g.add_argument("--activations-checkpoint-method", type=str, default=None, choices=["uniform", "block"])
    g.add_argument("--activations-checkpoint-num-layers", type=int, default=1)
    g.add_argument("--train-iters", type=int, default=None)
    g.add_argument("--log-interval", type=int, default=100)
    g.add_argument("--no-masked-softmax-fusion", action="store_false", dest="masked_softmax_fusion")
    g.add_argument("--no-bias-gelu-fusion", action="store_false", dest="bias_gelu_fusion")
    g.add_argument("--no-bias-dropout-fusion", action="store_false", dest="bias_dropout_fusion")
    g.add_argument("--optimizer", type=str, default="adam", choices=["adam", "sgd", "lamb"])
    g.add_argument("--cpu-offload", action="store_true")


def _add_initialization_args(p):
    g = p.add_argument_group("initialization")
    g.add_argument("--seed", type=int, default=1234)
    g.add_argument("--init-method-std", type=float, default=0.02)
    g.add_argument("--init-method-xavier-uniform", action="store_true")


def _add_learning_rate_args(p):
    g = p.add_argument_group("learning rate")
    g.add_argument("--lr", type=float, default=None)
    g.add_argument("--lr-decay-style", type=str, default="linear", choices=["constant", "linear", "cosine"])
    g.add_argument("--lr-warmup-fraction", type=float, default=None)
    g.add_argument("--min-lr", type=float, default=0.0)


def _add_mixed_precision_args(p):
    g = p.add_argument_group("mixed precision")
    g.add_argument("--fp16", action="store_true")
    g.add_argument("--bf16", action="store_true")
    g.add_argument("--loss-scale", type=float, default=None)
    g.add_argument("--initial-loss-scale", type=float, default=2 ** 32)
    g.add_argument("--min-loss-scale", type=float, default=1.0)
    g.add_argument("--loss-scale-window", type=float, default=1000)
    g.add_argument("--hysteresis", type=int, default=2)
    g.add_argument("--fp32-residual-connection", action="store_true")
    g.add_argument("--no-query-key-layer-scaling", action="store_false", dest="apply_query_key_layer_scaling")
    g.add_argument("--attention-softmax-in-fp32", action="store_true")
    g.add_argument("--accumulate-allreduce-grads-in-fp32", action="store_true")
    g.add_argument("--fp16-lm-cross-entropy", action="store_true")


def _add_distributed_args(p):
    g = p.add_argument_group("distributed")
    g.add_argument("--tensor-model-parallel-size", type=int, default=1)
    g.add_argument("--pipeline-model-parallel-size", type=int, default=1)
    g.add_argument("--pipeline-model-parallel-split-rank", type=int, default=None)
    g.add_argument("--num-layers-per-virtual-pipeline-stage", type=int, default=None)
    g.add_argument("--distributed-backend", default="nccl", choices=["nccl", "gloo", "ucc"])
    g.add_argument("--DDP-impl", default="local", choices=["local", "torch"])
    g.add_argument("--use-contiguous-buffers-in-local-ddp", action="store_true")
    g.add_argument("--local_rank", type=int, default=None)
    g.add_argument("--lazy-mpu-init", type=bool, default=None)
    g.add_argument("--use-cpu-initialization", action="store_true", default=None)
    g.add_argument("--sequence-parallel", action="store_true")
    g.add_argument("--gradient-accumulation-fusion", action="store_true")


def _add_data_args(p):
    g = p.add_argument_group("data")
    g.add_argument("--seq-length", type=int, default=None)
    g.add_argument("--encoder-seq-length", type=int, default=None)
    g.add_argument("--decoder-seq-length", type=int, default=None)
    g.add_argument("--vocab-size", type=int, default=None)
    g.add_argument("--data-path", nargs="*", default=None)
    g.add_argument("--num-workers", type=int, default=2)


def parse_args(extra_args_provider=None, defaults={}, override_args={}, ignore_unknown_args=False, argv=None):
    """``argv`` defaults to no command-line arguments (library use); pass ``sys.argv[1:]`` for scripts."""
    p = argparse.ArgumentParser(description="beforeholiday_amd transformer arguments", allow_abbrev=False)
    for add in (_add_network_size_args, _add_regularization_args, _add_training_args, _add_initialization_args,
                _add_learning_rate_args, _add_mixed_precision_args, _add_distributed_args, _add_data_args):
        add(p)
    if extra_args_provider is not None:
        p = extra_args_provider(p)
    argv = [] if argv is None else argv
    args = p.parse_known_args(argv)[0] if ignore_unknown_args else p.parse_args(argv)
    for k, v in defaults.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    for k, v in override_args.items():
        setattr(args, k, v)
    args.rank = int(os.getenv("RANK", "0"))
    args.world_size = int(os.getenv("WORLD_SIZE", "1"))
    if torch.distributed.is_initialized():
        args.rank = torch.distributed.get_rank()
        args.world_size = torch.distributed.get_world_size()
    mp = args.tensor_model_parallel_size * args.pipeline_model_parallel_size
    args.data_parallel_size = max(1, args.world_size // mp)
    if args.ffn_hidden_size is None and args.hidden_size is not None:
        args.ffn_hidden_size = 4 * args.hidden_size
    if args.kv_channels is None and args.hidden_size is not None and args.num_attention_heads:
        args.kv_channels = args.hidden_size // args.num_attention_heads
    if args.seq_length is not None and args.encoder_seq_length is None:
        args.encoder_seq_length = args.seq_length
    if args.checkpoint_activations and args.activations_checkpoint_method is None:
        args.activations_checkpoint_method = "uniform"
    if args.padded_vocab_size is None and args.vocab_size is not None:
        mult = args.make_vocab_size_divisible_by * args.tensor_model_parallel_size
        args.padded_vocab_size = ((args.vocab_size + mult - 1) // mult) * mult
    args.params_dtype = torch.half if args.fp16 else (torch.bfloat16 if args.bf16 else torch.float)
    args.virtual_pipeline_model_parallel_size = None
    if args.num_layers_per_virtual_pipeline_stage is not None and args.num_layers:
        args.virtual_pipeline_model_parallel_size = (args.num_layers // args.pipeline_model_parallel_size //
                                                     args.num_layers_per_virtual_pipeline_stage)
    return args


def to_config(args):
    """TransformerConfig from a parsed argument namespace."""
    from ...models.transformer_lm import TransformerConfig
    return TransformerConfig(
        hidden_size=args.hidden_size, num_layers=args.num_layers, num_attention_heads=args.num_attention_heads,
        ffn_hidden_size=args.ffn_hidden_size, kv_channels=args.kv_channels,
        vocab_size=args.padded_vocab_size or args.vocab_size or 50304,
        max_position_embeddings=args.max_position_embeddings or args.seq_length or 1024,
        hidden_dropout=args.hidden_dropout, attention_dropout=args.attention_dropout,
        layernorm_epsilon=args.layernorm_epsilon, init_method_std=args.init_method_std,
        apply_residual_connection_post_layernorm=args.apply_residual_connection_post_layernorm,
        apply_query_key_layer_scaling=args.apply_query_key_layer_scaling,
        attention_softmax_in_fp32=args.attention_softmax_in_fp32, masked_softmax_fusion=args.masked_softmax_fusion,
        bias_gelu_fusion=args.bias_gelu_fusion, openai_gelu=args.openai_gelu,
        fp32_residual_connection=args.fp32_residual_connection, params_dtype=args.params_dtype, fp16=args.fp16,
        bf16=args.bf16, sequence_parallel=args.sequence_parallel,
        use_cpu_initialization=bool(args.use_cpu_initialization),
        gradient_accumulation_fusion=args.gradient_accumulation_fusion,
        activations_checkpoint_method=args.activations_checkpoint_method,
        activations_checkpoint_num_layers=args.activations_checkpoint_num_layers,
        bert_binary_head=args.bert_binary_head)
