"""Standalone GPT / BERT: tensor-parallel (tp=2, +SP) and pipeline-parallel (pp=2) runs reproduce the
single-rank model exactly (fp64, dropout off, CPU ranks over gloo)."""
import pytest
import torch

from beforeholiday_amd import config

from tests._dist import run_distributed


def _seed():
    from beforeholiday_amd.transformer import tensor_parallel
    tensor_parallel.model_parallel_cuda_manual_seed(123)


def _cfg(**kw):
    from beforeholiday_amd.models import TransformerConfig
    base = dict(hidden_size=16, num_layers=2, num_attention_heads=4, vocab_size=64, max_position_embeddings=16,
                hidden_dropout=0.0, attention_dropout=0.0, params_dtype=torch.float64, use_cpu_initialization=True,
                masked_softmax_fusion=False)
    base.update(kw)
    return TransformerConfig(**base)


def _gpt_loss_and_grads(cfg, tokens, labels, seed=7):
    from beforeholiday_amd.models import GPTModel, finalize_model_grads
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    torch.manual_seed(seed)
    model = GPTModel(cfg)
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)
    loss = model(tokens, pos, mask, labels=labels)
    loss.mean().backward()
    finalize_model_grads(model)
    return model, loss.detach()


def _gpt_tp(rank, world, sequence_parallel):
    from beforeholiday_amd.transformer import parallel_state as ps
    torch.manual_seed(0)
    tokens = torch.randint(0, 64, (2, 8))
    labels = torch.randint(0, 64, (2, 8))
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    ref_model, ref_loss = _gpt_loss_and_grads(_cfg(), tokens, labels)
    ref_emb_grad = ref_model.language_model.embedding.word_embeddings.weight.grad
    ps.destroy_model_parallel()
    ps.initialize_model_parallel(world, 1, default_backend="gloo")
    _seed()
    model, loss = _gpt_loss_and_grads(_cfg(sequence_parallel=sequence_parallel), tokens, labels)
    torch.testing.assert_close(loss, ref_loss)
    emb_grad = model.language_model.embedding.word_embeddings.weight.grad
    torch.testing.assert_close(emb_grad, ref_emb_grad.chunk(world, 0)[rank])
    # LayerNorm grads (replicated params) agree with the single-rank model
    ln = model.language_model.encoder.final_layernorm.weight.grad
    torch.testing.assert_close(ln, ref_model.language_model.encoder.final_layernorm.weight.grad)
    qkv = model.language_model.encoder.layers[0].self_attention.query_key_value.weight.grad
    assert qkv.shape[0] == 3 * 16 // world
    ps.destroy_model_parallel()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("sequence_parallel", [False, True])
def test_gpt_tensor_parallel_matches_single_rank(sequence_parallel, world):
    """TP = 2 and TP = 4 (BASELINE configs[4]'s degree: one head and a quarter of the vocabulary per
    rank), with and without sequence parallelism."""
    run_distributed(_gpt_tp, world, sequence_parallel)


def _gpt_pp(rank, world):
    from beforeholiday_amd.models import GPTModel
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer.pipeline_parallel import build_model, get_forward_backward_func
    from beforeholiday_amd.transformer.pipeline_parallel import utils as pu
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    torch.manual_seed(0)
    mbs, nm, seq = 2, 4, 8
    tokens = torch.randint(0, 64, (mbs * nm, seq))
    labels = torch.randint(0, 64, (mbs * nm, seq))
    # single-rank reference over the same microbatches
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    cfg = _cfg()
    torch.manual_seed(7)
    ref = GPTModel(cfg)
    ref_losses = []
    for k in range(nm):
        t, l = tokens[k * mbs:(k + 1) * mbs], labels[k * mbs:(k + 1) * mbs]
        mask, _, pos = get_ltor_masks_and_position_ids(t, -1, False, False, False)
        loss = ref(t, pos, mask, labels=l).mean()
        (loss / nm).backward()
        ref_losses.append(loss.detach())
    ps.destroy_model_parallel()
    # pp=2: stage 0 holds embedding + layer 0, stage 1 holds layer 1 + final LN + tied head.
    ps.initialize_model_parallel(1, 2, default_backend="gloo")
    _seed()
    pu._reconfigure_microbatch_calculator(rank, None, mbs * nm, mbs, 1)
    torch.manual_seed(7)
    ref_state = ref.state_dict()

    def provider(pre_process, post_process):
        return GPTModel(_cfg(num_layers=2), pre_process=pre_process, post_process=post_process)

    model = build_model(provider, False)
    m = model[0]
    # load the single-rank weights into this stage (layer index offset by the stage)
    own = m.state_dict()
    stage = ps.get_pipeline_model_parallel_rank()
    for k in own:
        src = k
        if ".layers." in k:
            pre, rest = k.split(".layers.", 1)
            idx, tail = rest.split(".", 1)
            src = f"{pre}.layers.{int(idx) + stage}.{tail}"
        if k == "word_embeddings.weight":
            src = "language_model.embedding.word_embeddings.weight"
        own[k] = ref_state[src]
    m.load_state_dict(own)

    def step(batch, model):
        t, l = batch
        mask, _, pos = get_ltor_masks_and_position_ids(t, -1, False, False, False)
        out = model(t, pos, mask, labels=l)

        def loss_func(x):
            loss = x.mean()
            return loss, {"loss": loss.detach()}
        return out, loss_func

    fwd_bwd = get_forward_backward_func(None, 2)
    losses = fwd_bwd(step, [tokens, labels], m, forward_only=False, tensor_shape=(seq, mbs, 16),
                     dtype=torch.float64)
    from beforeholiday_amd.models import finalize_model_grads
    finalize_model_grads(m)
    if stage == 1:
        for got, want in zip(losses, ref_losses):
            torch.testing.assert_close(got["loss"], want)
        g = m.word_embeddings.weight.grad
    else:
        g = m.language_model.embedding.word_embeddings.weight.grad
    torch.testing.assert_close(g, ref.language_model.embedding.word_embeddings.weight.grad)
    pu.destroy_microbatch_calculator()
    ps.destroy_model_parallel()


def test_gpt_pipeline_parallel_matches_single_rank():
    if torch.cuda.is_available():
        pytest.skip("CPU (gloo) rehearsal: build_model places stages on the GPU when one is visible")
    run_distributed(_gpt_pp, 2)


def test_bert_forward_backward_cpu():
    import torch.distributed as dist
    from tests._dist import run_distributed as _rd  # noqa: F401
    run_distributed(_bert, 1)


def _bert(rank, world):
    from beforeholiday_amd.models import BertModel
    from beforeholiday_amd.transformer import parallel_state as ps
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    torch.manual_seed(1)
    model = BertModel(_cfg(), num_tokentypes=2)
    tokens = torch.randint(0, 64, (2, 8))
    att = torch.ones(2, 8, dtype=torch.long)
    att[1, 6:] = 0
    types = torch.zeros(2, 8, dtype=torch.long)
    labels = torch.randint(0, 64, (2, 8))
    loss, binary = model(tokens, att, tokentype_ids=types, lm_labels=labels)
    assert loss.shape == (2, 8) and binary.shape == (2, 2)
    (loss.mean() + binary.sum()).backward()
    assert model.language_model.embedding.word_embeddings.weight.grad is not None
    logits, _ = model(tokens, att, tokentype_ids=types)
    assert logits.shape == (2, 8, 64)
    ps.destroy_model_parallel()


def test_global_args_providers():
    from beforeholiday_amd.transformer.testing import global_vars
    from beforeholiday_amd.transformer.testing.arguments import to_config
    args = global_vars.set_global_variables(args_defaults=dict(num_layers=2, hidden_size=16, num_attention_heads=4,
                                                               seq_length=8, vocab_size=60, micro_batch_size=2,
                                                               global_batch_size=4))
    cfg = to_config(args)
    assert cfg.vocab_size == 128 and cfg.ffn_hidden_size == 64 and cfg.kv_channels == 4
    assert global_vars.get_num_microbatches() == 2
    global_vars.destroy_global_vars()


def _gpt_gpu_vs_cpu(rank, world):
    from beforeholiday_amd.models import GPTModel
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    cfg = _cfg(params_dtype=torch.float32, masked_softmax_fusion=True, hidden_size=64, num_attention_heads=4,
               vocab_size=128, max_position_embeddings=32)
    torch.manual_seed(7)
    cpu = GPTModel(cfg)
    torch.manual_seed(7)
    gpu = GPTModel(cfg).cuda()
    gpu.load_state_dict(cpu.state_dict())
    tokens = torch.randint(0, 128, (2, 32))
    labels = torch.randint(0, 128, (2, 32))
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)
    lc = cpu(tokens, pos, mask, labels=labels)
    lc.mean().backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg = gpu(tokens.cuda(), pos.cuda(), mask.cuda(), labels=labels.cuda())
    lg.mean().backward()
    torch.testing.assert_close(lg.float().cpu(), lc, rtol=3e-2, atol=3e-2)
    gw = gpu.language_model.encoder.layers[0].mlp.dense_h_to_4h.weight.grad.float().cpu()
    cw = cpu.language_model.encoder.layers[0].mlp.dense_h_to_4h.weight.grad
    assert torch.nn.functional.cosine_similarity(gw.flatten(), cw.flatten(), dim=0) > 0.99
    ps.destroy_model_parallel()


@pytest.mark.gpu
def test_gpt_gpu_fused_kernels_match_cpu():
    run_distributed(_gpt_gpu_vs_cpu, 1)


def _gpt_fused_mlp(rank, world):
    import os
    from beforeholiday_amd.models import GPTModel
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    cfg = _cfg(params_dtype=torch.bfloat16, masked_softmax_fusion=True, hidden_size=256, num_attention_heads=4,
               vocab_size=512, max_position_embeddings=64)
    torch.manual_seed(7)
    model = GPTModel(cfg).cuda()
    tokens = torch.randint(0, 512, (4, 64)).cuda()
    labels = torch.randint(0, 512, (4, 64)).cuda()
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)
    res = {}
    for fused in ("1", "0"):
        config.set(fused_mlp=fused == "1")
        model.zero_grad(set_to_none=True)
        loss = model(tokens, pos, mask, labels=labels)
        loss.float().mean().backward()
        mlp = model.language_model.encoder.layers[0].mlp
        res[fused] = (loss.detach().float(), mlp.dense_h_to_4h.weight.grad.float(), mlp.dense_h_to_4h.bias.grad.float(),
                      mlp.dense_4h_to_h.weight.grad.float(), model.language_model.embedding.word_embeddings.weight.grad.float())
    for a, b in zip(res["1"], res["0"]):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)
    ps.destroy_model_parallel()


@pytest.mark.gpu
def test_gpt_fused_mfma_mlp_matches_unfused():
    """ParallelMLP on the MFMA GEMM (bias+GELU epilogue, dGELU+bias-grad epilogue) == the unfused path."""
    run_distributed(_gpt_fused_mlp, 1)


def _flash_vs_unfused(rank, world, kind):
    import os
    from beforeholiday_amd.models import BertModel, GPTModel
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    cfg = _cfg(params_dtype=torch.bfloat16, masked_softmax_fusion=True, hidden_size=256, num_attention_heads=4,
               vocab_size=512, max_position_embeddings=256)
    torch.manual_seed(3)
    S = 200
    tokens = torch.randint(0, 512, (2, S)).cuda()
    labels = torch.randint(0, 512, (2, S)).cuda()
    if kind == "gpt":
        model = GPTModel(cfg).cuda()
        mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)
        run = lambda: model(tokens, pos, mask, labels=labels).float().mean()  # noqa: E731
    else:
        model = BertModel(cfg, num_tokentypes=2).cuda()
        att = torch.ones(2, S, dtype=torch.long, device="cuda")
        att[1, 150:] = 0  # padded tail: padding-mask path with the -10000 fill
        types = torch.zeros(2, S, dtype=torch.long, device="cuda")

        def run():
            loss, binary = model(tokens, att, tokentype_ids=types, lm_labels=labels)
            return loss.float().mean() + binary.float().sum() * 0.01
    res = {}
    for flash in ("1", "0"):
        config.set(flash_attn=flash == "1")
        model.zero_grad(set_to_none=True)
        loss = run()
        loss.backward()
        layer = model.language_model.encoder.layers[1]
        res[flash] = (loss.detach(), layer.self_attention.query_key_value.weight.grad.float(),
                      layer.self_attention.dense.weight.grad.float(),
                      model.language_model.embedding.word_embeddings.weight.grad.float())
    for a, b in zip(res["1"], res["0"]):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)
    ps.destroy_model_parallel()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gpt", "bert"])
def test_flash_attention_matches_unfused_megatron_path(kind):
    """CoreAttention on the MFMA flash kernels (causal for GPT, -10000 padding fill for BERT) == the
    bmm + fused-softmax + bmm path."""
    run_distributed(_flash_vs_unfused, 1, kind)


@pytest.mark.gpu
def test_vocab_ce_16bit_logits_fp32_loss_matches_fp32_logits():
    """bf16 logits + loss_dtype=fp32 (no fp32 logits copy) == the .float() path: same loss, same grad."""
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer import tensor_parallel as tp

    ps.set_tensor_model_parallel_rank(0)
    ps.set_tensor_model_parallel_world_size(1)
    try:
        torch.manual_seed(0)
        logits = (torch.randn(64, 4, 50304, device="cuda") * 3).to(torch.bfloat16)
        labels = torch.randint(0, 50304, (64, 4), device="cuda")
        a = logits.clone().requires_grad_(True)
        b = logits.clone().requires_grad_(True)
        la = tp.vocab_parallel_cross_entropy(a, labels, loss_dtype=torch.float32)
        lb = tp.vocab_parallel_cross_entropy(b.float(), labels)
        assert la.dtype == torch.float32
        torch.testing.assert_close(la, lb, atol=1e-5, rtol=1e-5)
        g = torch.randn_like(la)
        la.backward(g)
        lb.backward(g)
        assert a.grad.dtype == torch.bfloat16
        torch.testing.assert_close(a.grad.float(), b.grad.float(), atol=1e-2, rtol=1e-2)
    finally:
        ps.set_tensor_model_parallel_rank(None)
        ps.set_tensor_model_parallel_world_size(None)


def _ln_resid(rank, world):
    from beforeholiday_amd.models import GPTModel
    from beforeholiday_amd.transformer import parallel_state as ps
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    ps.initialize_model_parallel(1, 1, default_backend="gloo")
    _seed()
    cfg = _cfg(params_dtype=torch.bfloat16, masked_softmax_fusion=True, hidden_size=256, num_attention_heads=4,
               vocab_size=512, max_position_embeddings=64, hidden_dropout=0.1)
    torch.manual_seed(11)
    model = GPTModel(cfg).cuda()
    tokens = torch.randint(0, 512, (4, 64)).cuda()
    labels = torch.randint(0, 512, (4, 64)).cuda()
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, -1, False, False, False)
    res = {}
    for fused in (True, False):
        config.set(ln_residual_grad=fused)
        _seed()  # the same dropout masks in both runs
        model.zero_grad(set_to_none=True)
        loss = model(tokens, pos, mask, labels=labels).float().mean()
        loss.backward()
        enc = model.language_model.encoder
        res[fused] = [loss.detach()] + [p.grad.float().clone() for p in (
            enc.layers[0].input_layernorm.weight, enc.layers[0].self_attention.query_key_value.weight,
            enc.layers[1].post_attention_layernorm.bias, model.language_model.embedding.word_embeddings.weight)]
    # the fused path adds the residual gradient in fp32 and rounds once (the separate add rounds twice)
    for a, b in zip(res[True], res[False]):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2)
    ps.destroy_model_parallel()


@pytest.mark.gpu
def test_layernorm_residual_grad_link_matches_unfused():
    """Pre-LN blocks: the residual add parks its input gradient in a ResidualGradLink and the LayerNorm
    dx kernel adds it (no separate autograd add): same gradients as the unfused graph."""
    run_distributed(_ln_resid, 1)
