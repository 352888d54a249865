"""Megatron-style command-line arguments for the standalone models and the pipeline / tensor-parallel
test harness (reference: apex/transformer/testing/arguments.py:23-971).

Every flag of the reference's 15 groups (inference, network size, logging, regularization, training,
initialization, learning rate, checkpointing, mixed precision, distributed, validation, data and
dataloader, autoresume, biencoder, vision) with the same name, type, default and choices lives in one
table, ``_SPEC``; the parser is built from it, so a flag is one line. ``parse_args`` then applies the
reference's derivations and consistency checks (parallel sizes, deprecated flags, recompute
granularity, batch sizes, iteration- vs sample-based schedules, dtype rules, sequence parallelism).

Deviations, all for library use: ``argv`` defaults to no command-line arguments (pass
``sys.argv[1:]`` from a script), ``override_args`` are applied after parsing, a missing
``max_position_embeddings`` / ``micro_batch_size`` is derived (from ``seq_length`` / left unset)
instead of failing, the argument dump is printed only with ``BH_ARGS_VERBOSE=1``, and three flags
this package adds live in the last group (``--vocab-size``, ``--padded-vocab-size``,
``--activations-checkpoint-method/--num-layers`` for :class:`TransformerConfig`).
"""
import argparse
import os

import torch

# (group title, [(flags, add_argument keywords)]) -- reference flag set, in reference order
_SPEC = [
    ('inference', [
        (('--inference-batch-times-seqlen-threshold',), dict(type=int, default=512)),
    ]),
    ('network size', [
        (('--num-layers',), dict(type=int, default=None)),
        (('--hidden-size',), dict(type=int, default=None)),
        (('--ffn-hidden-size',), dict(type=int, default=None)),
        (('--num-attention-heads',), dict(type=int, default=None)),
        (('--kv-channels',), dict(type=int, default=None)),
        (('--max-position-embeddings',), dict(type=int, default=None)),
        (('--make-vocab-size-divisible-by',), dict(type=int, default=128)),
        (('--layernorm-epsilon',), dict(type=float, default=1e-05)),
        (('--apply-residual-connection-post-layernorm',), dict(action='store_true')),
        (('--openai-gelu',), dict(action='store_true')),
        (('--onnx-safe',), dict(type=bool, required=False)),
        (('--bert-no-binary-head',), dict(action='store_false', dest='bert_binary_head')),
        (('--num-experts',), dict(type=int, default=None)),
    ]),
    ('logging', [
        (('--log-params-norm',), dict(action='store_true')),
        (('--log-num-zeros-in-grad',), dict(action='store_true')),
        (('--tensorboard-log-interval',), dict(type=int, default=1)),
        (('--tensorboard-queue-size',), dict(type=int, default=1000)),
        (('--log-timers-to-tensorboard',), dict(action='store_true')),
        (('--log-batch-size-to-tensorboard',), dict(action='store_true')),
        (('--no-log-learnig-rate-to-tensorboard',), dict(action='store_false', dest='log_learning_rate_to_tensorboard')),
        (('--no-log-loss-scale-to-tensorboard',), dict(action='store_false', dest='log_loss_scale_to_tensorboard')),
        (('--log-validation-ppl-to-tensorboard',), dict(action='store_true')),
        (('--log-memory-to-tensorboard',), dict(action='store_true')),
        (('--log-world-size-to-tensorboard',), dict(action='store_true')),
    ]),
    ('regularization', [
        (('--attention-dropout',), dict(type=float, default=0.1)),
        (('--hidden-dropout',), dict(type=float, default=0.1)),
        (('--weight-decay',), dict(type=float, default=0.01)),
        (('--start-weight-decay',), dict(type=float)),
        (('--end-weight-decay',), dict(type=float)),
        (('--weight-decay-incr-style',), dict(type=str, default='constant', choices=['constant', 'linear', 'cosine'])),
        (('--clip-grad',), dict(type=float, default=1.0)),
        (('--adam-beta1',), dict(type=float, default=0.9)),
        (('--adam-beta2',), dict(type=float, default=0.999)),
        (('--adam-eps',), dict(type=float, default=1e-08)),
        (('--sgd-momentum',), dict(type=float, default=0.9)),
    ]),
    ('training', [
        (('--micro-batch-size',), dict(type=int, default=None)),
        (('--batch-size',), dict(type=int, default=None)),
        (('--global-batch-size',), dict(type=int, default=None)),
        (('--rampup-batch-size',), dict(nargs='*', default=None)),
        (('--recompute-activations',), dict(action='store_true')),
        (('--recompute-granularity',), dict(type=str, default=None, choices=['full', 'selective'])),
        (('--distribute-saved-activations',), dict(action='store_true')),
        (('--recompute-method',), dict(type=str, default=None, choices=['uniform', 'block'])),
        (('--recompute-num-layers',), dict(type=int, default=1)),
        (('--checkpoint-activations',), dict(action='store_true')),
        (('--train-iters',), dict(type=int, default=None)),
        (('--train-samples',), dict(type=int, default=None)),
        (('--log-interval',), dict(type=int, default=100)),
        (('--exit-interval',), dict(type=int, default=None)),
        (('--exit-duration-in-mins',), dict(type=int, default=None)),
        (('--tensorboard-dir',), dict(type=str, default=None)),
        (('--no-masked-softmax-fusion',), dict(action='store_false', dest='masked_softmax_fusion')),
        (('--no-bias-gelu-fusion',), dict(action='store_false', dest='bias_gelu_fusion')),
        (('--no-bias-dropout-fusion',), dict(action='store_false', dest='bias_dropout_fusion')),
        (('--optimizer',), dict(type=str, default='adam', choices=['adam', 'sgd', 'lamb'])),
        (('--dataloader-type',), dict(type=str, default=None, choices=['single', 'cyclic'])),
        (('--no-async-tensor-model-parallel-allreduce',), dict(action='store_true', dest='async_tensor_model_parallel_allreduce')),
        (('--no-persist-layer-norm',), dict(action='store_true')),
        (('--sequence-parallel',), dict(action='store_true')),
        (('--no-gradient-accumulation-fusion',), dict(action='store_false', dest='gradient_accumulation_fusion')),
    ]),
    ('initialization', [
        (('--seed',), dict(type=int, default=1234)),
        (('--init-method-std',), dict(type=float, default=0.02)),
        (('--init-method-xavier-uniform',), dict(action='store_true')),
    ]),
    ('learning rate', [
        (('--lr',), dict(type=float, default=None)),
        (('--lr-decay-style',), dict(type=str, default='linear', choices=['constant', 'linear', 'cosine'])),
        (('--lr-decay-iters',), dict(type=int, default=None)),
        (('--lr-decay-samples',), dict(type=int, default=None)),
        (('--lr-warmup-fraction',), dict(type=float, default=None)),
        (('--lr-warmup-iters',), dict(type=int, default=0)),
        (('--lr-warmup-samples',), dict(type=int, default=0)),
        (('--warmup',), dict(type=int, default=None)),
        (('--min-lr',), dict(type=float, default=0.0)),
        (('--override-lr-scheduler',), dict(action='store_true')),
        (('--use-checkpoint-lr-scheduler',), dict(action='store_true')),
    ]),
    ('checkpointing', [
        (('--save',), dict(type=str, default=None)),
        (('--save-interval',), dict(type=int, default=None)),
        (('--no-save-optim',), dict(action='store_true', default=None)),
        (('--no-save-rng',), dict(action='store_true', default=None)),
        (('--load',), dict(type=str, default=None)),
        (('--no-load-optim',), dict(action='store_true', default=None)),
        (('--no-load-rng',), dict(action='store_true', default=None)),
        (('--finetune',), dict(action='store_true')),
    ]),
    ('mixed precision', [
        (('--fp16',), dict(action='store_true')),
        (('--bf16',), dict(action='store_true')),
        (('--loss-scale',), dict(type=float, default=None)),
        (('--initial-loss-scale',), dict(type=float, default=2 ** 32)),
        (('--min-loss-scale',), dict(type=float, default=1.0)),
        (('--loss-scale-window',), dict(type=float, default=1000)),
        (('--hysteresis',), dict(type=int, default=2)),
        (('--fp32-residual-connection',), dict(action='store_true')),
        (('--no-query-key-layer-scaling',), dict(action='store_false', dest='apply_query_key_layer_scaling')),
        (('--attention-softmax-in-fp32',), dict(action='store_true')),
        (('--accumulate-allreduce-grads-in-fp32',), dict(action='store_true')),
        (('--fp16-lm-cross-entropy',), dict(action='store_true')),
    ]),
    ('distributed', [
        (('--tensor-model-parallel-size',), dict(type=int, default=1)),
        (('--pipeline-model-parallel-size',), dict(type=int, default=1)),
        (('--pipeline-model-parallel-split-rank',), dict(type=int, default=None)),
        (('--model-parallel-size',), dict(type=int, default=None)),
        (('--num-layers-per-virtual-pipeline-stage',), dict(type=int, default=None)),
        (('--distributed-backend',), dict(default='nccl', choices=['nccl', 'gloo'])),
        (('--DDP-impl',), dict(default='local', choices=['local', 'torch'])),
        (('--no-contiguous-buffers-in-local-ddp',), dict(action='store_false', dest='use_contiguous_buffers_in_local_ddp')),
        (('--no-scatter-gather-tensors-in-pipeline',), dict(action='store_false', dest='scatter_gather_tensors_in_pipeline')),
        (('--local_rank',), dict(type=int, default=None)),
        (('--lazy-mpu-init',), dict(type=bool, required=False)),
        (('--use-cpu-initialization',), dict(action='store_true', default=None)),
        (('--empty-unused-memory-level',), dict(default=0, type=int, choices=[0, 1, 2])),
        (('--standalone-embedding-stage',), dict(action='store_true', default=False)),
    ]),
    ('validation', [
        (('--eval-iters',), dict(type=int, default=100)),
        (('--eval-interval',), dict(type=int, default=1000)),
    ]),
    ('data and dataloader', [
        (('--data-path',), dict(nargs='*', default=None)),
        (('--split',), dict(type=str, default='969, 30, 1')),
        (('--vocab-file',), dict(type=str, default=None)),
        (('--merge-file',), dict(type=str, default=None)),
        (('--vocab-extra-ids',), dict(type=int, default=0)),
        (('--seq-length',), dict(type=int, default=None)),
        (('--encoder-seq-length',), dict(type=int, default=None)),
        (('--decoder-seq-length',), dict(type=int, default=None)),
        (('--retriever-seq-length',), dict(type=int, default=256)),
        (('--sample-rate',), dict(type=float, default=1.0)),
        (('--mask-prob',), dict(type=float, default=0.15)),
        (('--short-seq-prob',), dict(type=float, default=0.1)),
        (('--mmap-warmup',), dict(action='store_true')),
        (('--num-workers',), dict(type=int, default=2)),
        (('--tokenizer-type',), dict(type=str, default=None, choices=['BertWordPieceLowerCase', 'BertWordPieceCase', 'GPT2BPETokenizer'])),
        (('--data-impl',), dict(type=str, default='infer', choices=['lazy', 'cached', 'mmap', 'infer'])),
        (('--reset-position-ids',), dict(action='store_true')),
        (('--reset-attention-mask',), dict(action='store_true')),
        (('--eod-mask-loss',), dict(action='store_true')),
    ]),
    ('autoresume', [
        (('--adlr-autoresume',), dict(action='store_true')),
        (('--adlr-autoresume-interval',), dict(type=int, default=1000)),
    ]),
    ('biencoder', [
        (('--ict-head-size',), dict(type=int, default=None)),
        (('--biencoder-projection-dim',), dict(type=int, default=0)),
        (('--biencoder-shared-query-context-model',), dict(action='store_true')),
        (('--ict-load',), dict(type=str, default=None)),
        (('--bert-load',), dict(type=str, default=None)),
        (('--titles-data-path',), dict(type=str, default=None)),
        (('--query-in-block-prob',), dict(type=float, default=0.1)),
        (('--use-one-sent-docs',), dict(action='store_true')),
        (('--evidence-data-path',), dict(type=str, default=None)),
        (('--retriever-report-topk-accuracies',), dict(nargs='+', type=int, default=[])),
        (('--retriever-score-scaling',), dict(action='store_true')),
        (('--block-data-path',), dict(type=str, default=None)),
        (('--embedding-path',), dict(type=str, default=None)),
        (('--indexer-batch-size',), dict(type=int, default=128)),
        (('--indexer-log-interval',), dict(type=int, default=1000)),
    ]),
    ('vision', [
        (('--num-classes',), dict(type=int, default=1000)),
        (('--img-h',), dict(type=int, default=224)),
        (('--img-w',), dict(type=int, default=224)),
        (('--num-channels',), dict(type=int, default=3)),
        (('--patch-dim',), dict(type=int, default=16)),
        (('--classes-fraction',), dict(type=float, default=1.0)),
        (('--data-per-class-fraction',), dict(type=float, default=1.0)),
        (('--no-data-sharding',), dict(action='store_false', dest='data_sharding')),
        (('--head-lr-mult',), dict(type=float, default=1.0)),
        (('--vision-pretraining',), dict(action='store_true')),
        (('--vision-pretraining-type',), dict(type=str, default='classify', choices=['classify', 'inpaint', 'dino'])),
        (('--vision-backbone-type',), dict(type=str, default='vit', choices=['vit', 'mit', 'swin'])),
        (('--swin-backbone-type',), dict(type=str, default='tiny', choices=['tiny', 'base', 'h3'])),
        (('--mask-type',), dict(type=str, default='random', choices=['random', 'row'])),
        (('--mask-factor',), dict(type=float, default=1.0)),
        (('--iter-per-epoch',), dict(type=int, default=1250)),
        (('--dino-local-img-size',), dict(type=int, default=96)),
        (('--dino-local-crops-number',), dict(type=int, default=10)),
        (('--dino-head-hidden-size',), dict(type=int, default=2048)),
        (('--dino-bottleneck-size',), dict(type=int, default=256)),
        (('--dino-freeze-last-layer',), dict(type=float, default=1)),
        (('--dino-norm-last-layer',), dict(action='store_true')),
        (('--dino-warmup-teacher-temp',), dict(type=float, default=0.04)),
        (('--dino-teacher-temp',), dict(type=float, default=0.07)),
        (('--dino-warmup-teacher-temp-epochs',), dict(type=int, default=30)),
    ]),
    ('beforeholiday extensions', [
        (('--vocab-size',), dict(type=int, default=None)),
        (('--padded-vocab-size',), dict(type=int, default=None)),
        (('--activations-checkpoint-method',), dict(type=str, default=None, choices=['uniform', 'block'])),
        (('--activations-checkpoint-num-layers',), dict(type=int, default=1)),
    ]),
]


def build_parser():
    p = argparse.ArgumentParser(description="beforeholiday_amd transformer arguments", allow_abbrev=False)
    for title, args in _SPEC:
        g = p.add_argument_group(title=title)
        for flags, kw in args:
            g.add_argument(*flags, **kw)
    p.add_argument("--cpu-offload", action="store_true", default=False)
    return p


def _fail(cond, msg):
    if not cond:
        raise AssertionError(msg)


def _say(args, msg):
    if args.rank == 0 and os.environ.get("BH_ARGS_VERBOSE") == "1":
        print(msg, flush=True)


def _parallel_sizes(args):
    args.tensor_model_parallel_size = min(args.tensor_model_parallel_size, args.world_size)
    _fail(args.world_size % args.tensor_model_parallel_size == 0,
          f"world size ({args.world_size}) is not divisible by tensor model parallel size "
          f"({args.tensor_model_parallel_size})")
    args.pipeline_model_parallel_size = min(args.pipeline_model_parallel_size,
                                            args.world_size // args.tensor_model_parallel_size)
    args.transformer_pipeline_model_parallel_size = (args.pipeline_model_parallel_size -
                                                     (1 if args.standalone_embedding_stage else 0))
    mp = args.pipeline_model_parallel_size * args.tensor_model_parallel_size
    _fail(args.world_size % mp == 0, f"world size ({args.world_size}) is not divisible by tensor ({args.tensor_model_parallel_size}) x pipeline ({args.pipeline_model_parallel_size}) parallel size")
    args.data_parallel_size = args.world_size // mp
    if args.pipeline_model_parallel_size > 1 and args.pipeline_model_parallel_split_rank is not None:
        _fail(args.pipeline_model_parallel_split_rank < args.pipeline_model_parallel_size,
              "pipeline split rank must be smaller than the pipeline model parallel size")


def _deprecated(args):
    for old, new in (("batch_size", "--micro-batch-size"), ("warmup", "--lr-warmup-fraction"),
                     ("model_parallel_size", "--tensor-model-parallel-size")):
        _fail(getattr(args, old) is None, f"--{old.replace('_', '-')} is no longer valid, use {new} instead")
        delattr(args, old)
    if args.checkpoint_activations:  # old flag -> full / uniform recompute
        args.recompute_granularity, args.recompute_method = "full", "uniform"
    del args.checkpoint_activations
    if args.recompute_activations:
        args.recompute_granularity = "selective"
    del args.recompute_activations


def _schedules(args):
    args.consumed_train_samples = 0
    args.consumed_valid_samples = 0
    if args.train_iters:
        _fail(args.train_samples is None, "expected iteration-based training")
        _fail(args.lr_decay_samples is None, "expected iteration-based learning rate decay")
        _fail(args.lr_warmup_samples == 0, "expected iteration-based learning rate warmup")
        _fail(args.rampup_batch_size is None, "expected no batch-size rampup for iteration-based training")
        if args.lr_warmup_fraction is not None:
            _fail(args.lr_warmup_iters == 0, "give only one of --lr-warmup-fraction and --lr-warmup-iters")
    if args.train_samples:
        _fail(args.train_iters is None, "expected sample-based training")
        _fail(args.lr_decay_iters is None, "expected sample-based learning rate decay")
        _fail(args.lr_warmup_iters == 0, "expected sample-based learning rate warmup")
        if args.lr_warmup_fraction is not None:
            _fail(args.lr_warmup_samples == 0, "give only one of --lr-warmup-fraction and --lr-warmup-samples")


def _precision(args):
    _fail(not (args.fp16 and args.bf16), "--fp16 and --bf16 are exclusive")
    args.params_dtype = torch.half if args.fp16 else (torch.bfloat16 if args.bf16 else torch.float)
    if args.bf16 and not args.accumulate_allreduce_grads_in_fp32:
        args.accumulate_allreduce_grads_in_fp32 = True  # bf16 gradients accumulate and reduce in fp32
        _say(args, "accumulate and all-reduce gradients in fp32 for bfloat16 parameters")
    if args.accumulate_allreduce_grads_in_fp32:
        _fail(args.DDP_impl == "local", "fp32 gradient accumulation needs --DDP-impl local")
        _fail(args.use_contiguous_buffers_in_local_ddp, "fp32 gradient accumulation needs contiguous DDP buffers")
    elif args.gradient_accumulation_fusion:
        args.gradient_accumulation_fusion = False  # only defined for fp32 main-grad accumulation
        _say(args, "gradient accumulation fusion needs fp32 gradient accumulation: disabled")
    if args.DDP_impl == "torch":
        args.use_contiguous_buffers_in_local_ddp = False
    if args.fp16_lm_cross_entropy:
        _fail(args.fp16, "fp16 lm cross entropy needs --fp16")
    if args.fp32_residual_connection:
        _fail(args.fp16 or args.bf16, "fp32 residual connections need --fp16 or --bf16")


def _model_shape(args):
    if args.max_position_embeddings is None:  # library use: size the table to the sequence
        args.max_position_embeddings = args.seq_length or args.encoder_seq_length
    for name in ("num_layers", "hidden_size", "num_attention_heads", "max_position_embeddings"):
        _fail(getattr(args, name) is not None, f"{name} argument is None")
    if args.ffn_hidden_size is None:
        args.ffn_hidden_size = 4 * args.hidden_size
    if args.kv_channels is None:
        _fail(args.hidden_size % args.num_attention_heads == 0, "hidden size not divisible by attention heads")
        args.kv_channels = args.hidden_size // args.num_attention_heads
    if args.seq_length is not None:
        _fail(args.encoder_seq_length is None, "give --seq-length or --encoder-seq-length, not both")
        args.encoder_seq_length = args.seq_length
    else:
        args.seq_length = args.encoder_seq_length
    for name in ("seq_length", "decoder_seq_length"):
        v = getattr(args, name)
        if v is not None:
            _fail(args.max_position_embeddings >= v, f"{name} exceeds max_position_embeddings")
    if args.padded_vocab_size is None and args.vocab_size is not None:
        mult = args.make_vocab_size_divisible_by * args.tensor_model_parallel_size
        args.padded_vocab_size = -(-args.vocab_size // mult) * mult


def _recompute(args):
    if args.distribute_saved_activations:
        _fail(args.tensor_model_parallel_size > 1, "distributed saved activations need tensor parallelism")
        _fail(args.recompute_granularity == "full", "distributed saved activations need full recompute")
        _fail(args.recompute_method is not None, "distributed saved activations need a recompute method")
    if args.recompute_granularity == "selective":
        _fail(args.recompute_method is None, "selective recompute takes no recompute method")
    if args.activations_checkpoint_method is None and args.recompute_granularity == "full":
        args.activations_checkpoint_method = args.recompute_method
        args.activations_checkpoint_num_layers = args.recompute_num_layers


def parse_args(extra_args_provider=None, defaults={}, override_args={}, ignore_unknown_args=False, argv=None):
    """Parse ``argv`` (default: none), apply ``defaults`` to unset arguments and ``override_args``
    unconditionally, then derive and check as the reference does."""
    p = build_parser()
    if extra_args_provider is not None:
        p = extra_args_provider(p)
    argv = [] if argv is None else list(argv)
    args = p.parse_known_args(argv)[0] if ignore_unknown_args else p.parse_args(argv)

    args.rank = int(os.getenv("RANK", "0"))
    args.world_size = int(os.getenv("WORLD_SIZE", "1"))
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        args.rank = torch.distributed.get_rank()
        args.world_size = torch.distributed.get_world_size()
    for k, v in defaults.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
        else:
            _say(args, f"WARNING: argument {k}={getattr(args, k)} overrides the default {v}")
    for k, v in override_args.items():
        setattr(args, k, v)

    _parallel_sizes(args)
    _deprecated(args)
    if args.micro_batch_size is not None:
        _fail(args.micro_batch_size > 0, "micro batch size must be positive")
        if args.global_batch_size is None:
            args.global_batch_size = args.micro_batch_size * args.data_parallel_size
        _fail(args.global_batch_size > 0, "global batch size must be positive")
    if args.num_layers_per_virtual_pipeline_stage is not None:
        _fail(args.pipeline_model_parallel_size > 2, "the interleaved schedule needs pipeline parallel size > 2")
        _fail(args.num_layers % args.num_layers_per_virtual_pipeline_stage == 0,
              "layers not divisible by layers per virtual pipeline stage")
        args.virtual_pipeline_model_parallel_size = (args.num_layers // args.pipeline_model_parallel_size //
                                                     args.num_layers_per_virtual_pipeline_stage)
    else:
        args.virtual_pipeline_model_parallel_size = None
    _precision(args)
    if args.dataloader_type is None:
        args.dataloader_type = "single"
    _schedules(args)
    _model_shape(args)
    if args.lr is not None:
        _fail(args.min_lr <= args.lr, "min lr above lr")
    if args.save is not None:
        _fail(args.save_interval is not None, "--save needs --save-interval")
    if args.weight_decay_incr_style == "constant":
        _fail(args.start_weight_decay is None and args.end_weight_decay is None,
              "constant weight decay takes no start / end values")
        args.start_weight_decay = args.end_weight_decay = args.weight_decay
    else:
        _fail(args.start_weight_decay is not None and args.end_weight_decay is not None,
              "an incremented weight decay needs start and end values")
    _recompute(args)
    if args.sequence_parallel:
        args.async_tensor_model_parallel_allreduce = False
    if args.rank == 0 and os.environ.get("BH_ARGS_VERBOSE") == "1":
        print("-------- arguments --------")
        for k in sorted(vars(args)):
            print(f"  {k} {'.' * max(1, 48 - len(k))} {getattr(args, k)}")
        print("---------------------------", flush=True)
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
