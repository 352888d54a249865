"""Megatron argument parity (reference: apex/transformer/testing/arguments.py): every reference flag
parses with its default, and parse_args applies the reference's derivations and checks."""
import ast
import warnings

import pytest

from beforeholiday_amd.transformer.testing.arguments import build_parser, parse_args

REF = "/root/reference/apex/transformer/testing/arguments.py"
BASE = ["--num-layers", "2", "--hidden-size", "16", "--num-attention-heads", "4", "--seq-length", "8",
        "--max-position-embeddings", "8", "--micro-batch-size", "2"]


def _reference_flags():
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            tree = ast.parse(open(REF).read())
    except OSError:
        pytest.skip("reference tree not present")
    flags = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "add_argument":
            flags.update(ast.literal_eval(a) for a in node.args)
    return flags


def test_every_reference_flag_is_accepted():
    ours = {s for a in build_parser()._actions for s in a.option_strings}
    missing = _reference_flags() - ours
    assert not missing, sorted(missing)


def test_defaults_and_derivations():
    a = parse_args(argv=BASE)
    assert a.ffn_hidden_size == 64 and a.kv_channels == 4 and a.encoder_seq_length == 8
    assert a.global_batch_size == 2 and a.data_parallel_size == 1 and a.dataloader_type == "single"
    assert a.initial_loss_scale == 2 ** 32 and a.use_contiguous_buffers_in_local_ddp
    assert a.start_weight_decay == a.end_weight_decay == a.weight_decay
    assert a.virtual_pipeline_model_parallel_size is None and a.consumed_train_samples == 0
    assert not hasattr(a, "batch_size") and not hasattr(a, "checkpoint_activations")


def test_deprecated_and_recompute_flags():
    with pytest.raises(AssertionError, match="micro-batch-size"):
        parse_args(argv=BASE + ["--batch-size", "4"])
    a = parse_args(argv=BASE + ["--checkpoint-activations"])
    assert a.recompute_granularity == "full" and a.recompute_method == "uniform"
    assert a.activations_checkpoint_method == "uniform"
    assert parse_args(argv=BASE + ["--recompute-activations"]).recompute_granularity == "selective"
    with pytest.raises(AssertionError):
        parse_args(argv=BASE + ["--recompute-activations", "--recompute-method", "block"])


def test_precision_rules():
    a = parse_args(argv=BASE + ["--bf16"])
    assert a.accumulate_allreduce_grads_in_fp32 and a.gradient_accumulation_fusion
    a = parse_args(argv=BASE + ["--fp16"])
    assert not a.gradient_accumulation_fusion  # needs fp32 accumulation
    with pytest.raises(AssertionError):
        parse_args(argv=BASE + ["--fp16", "--bf16"])
    with pytest.raises(AssertionError):
        parse_args(argv=BASE + ["--fp32-residual-connection"])
    assert not parse_args(argv=BASE + ["--sequence-parallel"]).async_tensor_model_parallel_allreduce


def test_schedule_checks():
    with pytest.raises(AssertionError, match="iteration-based"):
        parse_args(argv=BASE + ["--train-iters", "10", "--train-samples", "100"])
    with pytest.raises(AssertionError):
        parse_args(argv=BASE + ["--train-iters", "10", "--lr-warmup-fraction", "0.1", "--lr-warmup-iters", "5"])
    with pytest.raises(AssertionError):
        parse_args(argv=BASE + ["--weight-decay-incr-style", "linear"])
    a = parse_args(argv=BASE + ["--weight-decay-incr-style", "linear", "--start-weight-decay", "0.0",
                                "--end-weight-decay", "0.1"])
    assert a.end_weight_decay == 0.1


def test_defaults_dict_fills_only_unset():
    a = parse_args(argv=["--hidden-size", "32"], defaults=dict(num_layers=2, hidden_size=16, num_attention_heads=4,
                                                               seq_length=8, micro_batch_size=1))
    assert a.hidden_size == 32 and a.num_layers == 2 and a.max_position_embeddings == 8
