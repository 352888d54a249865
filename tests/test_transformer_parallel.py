"""Tensor / sequence / pipeline parallelism on CPU ranks (gloo), checked against single-process math.

Mirrors the reference's tests/L0/run_transformer suite (parallel_state, mappings, layers,
cross_entropy, data, random, pipeline schedules, microbatches, batch samplers, grad scaler).
"""
import pytest
import torch
import torch.nn.functional as F

from tests._dist import run_distributed


def _init(tp, pp, vpp=None):
    from beforeholiday_amd.transformer import parallel_state
    parallel_state.destroy_model_parallel()
    parallel_state.initialize_model_parallel(tp, pp, vpp, default_backend="gloo", p2p_backend="gloo")
    return parallel_state


# ----------------------------------------------------------------------------------------------
def _topology(rank, world):
    ps = _init(2, 2)
    assert ps.model_parallel_is_initialized()
    assert ps.get_tensor_model_parallel_world_size() == 2
    assert ps.get_pipeline_model_parallel_world_size() == 2
    assert ps.get_data_parallel_world_size() == world // 4
    # TP groups are consecutive ranks, PP groups strided by world/pp
    assert ps.get_tensor_model_parallel_rank() == rank % 2
    assert ps.get_tensor_model_parallel_src_rank() == rank - rank % 2
    assert ps.get_pipeline_model_parallel_rank() == rank // 2
    assert ps.get_pipeline_model_parallel_first_rank() == rank % 2
    assert ps.get_pipeline_model_parallel_last_rank() == rank % 2 + 2
    assert ps.get_pipeline_model_parallel_next_rank() == (rank + 2) % 4
    assert ps.get_pipeline_model_parallel_prev_rank() == (rank - 2) % 4
    assert ps.is_pipeline_first_stage() == (rank < 2)
    assert ps.is_pipeline_last_stage() == (rank >= 2)
    assert ps.is_rank_in_embedding_group()
    assert ps.is_rank_in_position_embedding_group() == (rank < 2)
    assert ps.get_rank_info() == (rank % 2, rank // 2, 0)
    # virtual pipeline
    ps.destroy_model_parallel()
    ps.initialize_model_parallel(1, 4, 2, default_backend="gloo")
    assert ps.get_virtual_pipeline_model_parallel_world_size() == 2
    ps.set_virtual_pipeline_model_parallel_rank(1)
    assert not ps.is_pipeline_first_stage()
    assert ps.is_pipeline_first_stage(ignore_virtual=True) == (rank == 0)
    assert ps.is_pipeline_last_stage() == (rank == 3)
    ps.destroy_model_parallel()
    assert not ps.model_parallel_is_initialized()
    # split rank (encoder/decoder)
    ps.initialize_model_parallel(1, 4, None, 2, default_backend="gloo")
    assert ps.get_pipeline_model_parallel_split_rank() == 2
    assert ps.is_pipeline_stage_before_split() == (rank < 2)
    assert ps.is_pipeline_stage_after_split() == (rank >= 2)
    assert ps.is_pipeline_stage_at_split() == (rank == 1)
    assert ps.is_rank_in_embedding_group(ignore_virtual=True) == (rank in (0, 2, 3))
    ps.destroy_model_parallel()


def test_parallel_state_topology():
    run_distributed(_topology, 4)


def _indivisible(rank, world):
    from beforeholiday_amd.transformer import parallel_state as ps
    with pytest.raises(RuntimeError):
        ps.initialize_model_parallel(3, 1, default_backend="gloo")


def test_initialize_rejects_indivisible():
    run_distributed(_indivisible, 4)


# ----------------------------------------------------------------------------------------------
def _mappings(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    torch.manual_seed(0)
    full = torch.randn(8, 3, 4 * world, dtype=torch.float64)
    mine = full.chunk(world, dim=-1)[rank].clone().requires_grad_()
    g = tp.gather_from_tensor_model_parallel_region(mine)
    torch.testing.assert_close(g, full)
    g.backward(torch.ones_like(g) * (rank + 1))
    torch.testing.assert_close(mine.grad, torch.full_like(mine, rank + 1.0))
    s = tp.scatter_to_tensor_model_parallel_region(full.clone().requires_grad_())
    torch.testing.assert_close(s, full.chunk(world, -1)[rank])
    x = torch.full((4, 2), float(rank + 1), dtype=torch.float64, requires_grad=True)
    r = tp.reduce_from_tensor_model_parallel_region(x * 1.0)
    torch.testing.assert_close(r, torch.full((4, 2), float(sum(range(1, world + 1))), dtype=torch.float64))
    c = tp.copy_to_tensor_model_parallel_region(x)
    c.backward(torch.ones_like(c))
    torch.testing.assert_close(x.grad, torch.full_like(x, float(world)))
    # sequence parallel: first-dim scatter/gather/reduce-scatter
    seq = full.clone()
    part = tp.scatter_to_sequence_parallel_region(seq)
    torch.testing.assert_close(part, full.chunk(world, 0)[rank])
    part = part.clone().requires_grad_()
    gathered = tp.gather_from_sequence_parallel_region(part)
    torch.testing.assert_close(gathered, full)
    gathered.backward(torch.ones_like(gathered))
    torch.testing.assert_close(part.grad, torch.full_like(part, float(world)))  # reduce-scatter of ones
    y = (full * (rank + 1)).requires_grad_()
    rs = tp.reduce_scatter_to_sequence_parallel_region(y)
    torch.testing.assert_close(rs, full.chunk(world, 0)[rank] * sum(range(1, world + 1)))
    ps.destroy_model_parallel()


def test_tp_mappings():
    run_distributed(_mappings, 2)


# ----------------------------------------------------------------------------------------------
def _layers(rank, world, sequence_parallel):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    torch.manual_seed(1234)
    s, b, h, o = 4, 2, 8, 12
    col = tp.ColumnParallelLinear(h, o, gather_output=not sequence_parallel, keep_master_weight_for_test=True,
                                  use_cpu_initialization=True, params_dtype=torch.float64,
                                  sequence_parallel_enabled=sequence_parallel,
                                  no_async_tensor_model_parallel_allreduce=sequence_parallel)
    row = tp.RowParallelLinear(o, h, input_is_parallel=True, keep_master_weight_for_test=True,
                               use_cpu_initialization=True, params_dtype=torch.float64,
                               sequence_parallel_enabled=sequence_parallel)
    with torch.no_grad():
        col.bias.copy_(torch.arange(o // world, dtype=torch.float64) + rank * (o // world))
        row.bias.fill_(0.5)
    torch.manual_seed(99)
    x = torch.randn(s, b, h, dtype=torch.float64)
    # reference: full weights
    W1 = col.master_weight.clone().requires_grad_()
    b1 = torch.arange(o, dtype=torch.float64).requires_grad_()
    W2 = row.master_weight.clone().requires_grad_()
    b2 = torch.full((h,), 0.5, dtype=torch.float64, requires_grad=True)
    xr = x.clone().requires_grad_()
    ref = F.linear(torch.relu(F.linear(xr, W1, b1)), W2, b2)
    ref.sum().backward()
    xin = x.chunk(world, 0)[rank].clone() if sequence_parallel else x.clone()
    xin.requires_grad_()
    hcol, _ = col(xin)
    if not sequence_parallel:  # gathered output: feed the row layer this rank's shard
        hcol = hcol.chunk(world, -1)[rank]
    out, _ = row(torch.relu(hcol))
    expect = ref.detach().chunk(world, 0)[rank] if sequence_parallel else ref.detach()
    torch.testing.assert_close(out, expect)
    out.sum().backward()
    shard = o // world
    torch.testing.assert_close(col.weight.grad, W1.grad[rank * shard:(rank + 1) * shard])
    torch.testing.assert_close(col.bias.grad, b1.grad[rank * shard:(rank + 1) * shard])
    torch.testing.assert_close(row.weight.grad, W2.grad[:, rank * shard:(rank + 1) * shard])
    if sequence_parallel:
        torch.testing.assert_close(xin.grad, xr.grad.chunk(world, 0)[rank])
        # row bias grad is partial per sequence shard under SP
        assert getattr(row.bias, "sequence_parallel_enabled", False)
    else:
        torch.testing.assert_close(xin.grad, xr.grad)
        torch.testing.assert_close(row.bias.grad, b2.grad)
    ps.destroy_model_parallel()


@pytest.mark.parametrize("sequence_parallel", [False, True])
def test_column_row_parallel_linear(sequence_parallel):
    run_distributed(_layers, 2, sequence_parallel)


def _grad_accum_fusion(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    layer = tp.ColumnParallelLinear(6, 8, gather_output=False, use_cpu_initialization=True,
                                    gradient_accumulation_fusion=True)
    layer.weight.main_grad = torch.zeros_like(layer.weight, dtype=torch.float32)
    x = torch.randn(3, 2, 6)
    for _ in range(2):
        y, _ = layer(x)
        y.sum().backward()
    expect = 2 * torch.ones(3 * 2, 8 // world).t() @ x.reshape(-1, 6)
    torch.testing.assert_close(layer.weight.main_grad, expect, rtol=1e-5, atol=1e-5)
    assert layer.weight.grad is None
    ps.destroy_model_parallel()


def test_gradient_accumulation_fusion_cpu():
    run_distributed(_grad_accum_fusion, 2)


def _embedding_and_xent(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    torch.manual_seed(5)
    V, H = 16, 6
    emb = tp.VocabParallelEmbedding(V, H, use_cpu_initialization=True, params_dtype=torch.float64)
    master = torch.empty(V, H, dtype=torch.float)
    torch.manual_seed(5)
    torch.nn.init.xavier_normal_(master)
    master = master.double()
    torch.testing.assert_close(emb.weight.detach(), master.chunk(world, 0)[rank])
    tok = torch.randint(0, V, (5, 3))
    out = emb(tok)
    torch.testing.assert_close(out, F.embedding(tok, master))
    out.sum().backward()
    ref_w = master.clone().requires_grad_()
    F.embedding(tok, ref_w).sum().backward()
    torch.testing.assert_close(emb.weight.grad, ref_w.grad.chunk(world, 0)[rank])
    # vocab-parallel cross entropy
    logits = torch.randn(4, 3, V, dtype=torch.float64)
    target = torch.randint(0, V, (4, 3))
    mine = logits.chunk(world, -1)[rank].clone().requires_grad_()
    loss = tp.vocab_parallel_cross_entropy(mine, target)
    ref_l = logits.clone().requires_grad_()
    ref = F.cross_entropy(ref_l.view(-1, V), target.view(-1), reduction="none").view(4, 3)
    torch.testing.assert_close(loss, ref)
    w = torch.rand(4, 3, dtype=torch.float64)
    (loss * w).sum().backward()
    (ref * w).sum().backward()
    torch.testing.assert_close(mine.grad, ref_l.grad.chunk(world, -1)[rank])
    ps.destroy_model_parallel()


def test_vocab_parallel_embedding_and_cross_entropy():
    run_distributed(_embedding_and_xent, 2)


def _broadcast(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    data = {"text": torch.arange(12).view(3, 4) + 100, "types": torch.arange(6).view(2, 3)}
    if rank != 0:
        data = {k: torch.zeros_like(v) for k, v in data.items()}
    out = tp.broadcast_data(["text", "types"], data, torch.int64)
    torch.testing.assert_close(out["text"], torch.arange(12).view(3, 4) + 100)
    torch.testing.assert_close(out["types"], torch.arange(6).view(2, 3))
    ps.destroy_model_parallel()


def test_broadcast_data():
    run_distributed(_broadcast, 2)


def _rng_and_checkpoint(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer import tensor_parallel as tp
    tp.model_parallel_cuda_manual_seed(123)
    tracker = tp.get_cuda_rng_tracker()
    with tracker.fork():
        a = torch.rand(4)
    with tracker.fork():
        b = torch.rand(4)
    assert not torch.equal(a, b)
    dflt = torch.rand(4)
    gathered = [torch.empty(4) for _ in range(world)]
    torch.distributed.all_gather(gathered, a)
    assert not torch.equal(gathered[0], gathered[1])  # TP stream differs per rank
    torch.distributed.all_gather(gathered, dflt)
    assert torch.equal(gathered[0], gathered[1])  # default stream same per rank
    # checkpoint with dropout: recompute must replay the same mask
    x = torch.randn(6, 5, requires_grad=True)
    lin = torch.nn.Linear(5, 5)

    def f(inp):
        with tracker.fork():
            return F.dropout(lin(inp), p=0.5, training=True)

    tp.model_parallel_cuda_manual_seed(7)
    y = tp.checkpoint(f, False, x)
    y.sum().backward()
    gx = x.grad.clone()
    x.grad = None
    lin.zero_grad()
    tp.model_parallel_cuda_manual_seed(7)
    y2 = f(x)
    y2.sum().backward()
    torch.testing.assert_close(y, y2)
    torch.testing.assert_close(x.grad, gx)
    ps.destroy_model_parallel()


def test_rng_tracker_and_checkpoint():
    run_distributed(_rng_and_checkpoint, 2)


# ----------------------------------------------------------------------------------------------
# pipeline schedules vs. sequential single-process math
# ----------------------------------------------------------------------------------------------
def _pipeline(rank, world, pp, vpp, num_micro, forward_only):
    ps = _init(1, pp, vpp)
    from beforeholiday_amd.transformer.pipeline_parallel import build_model, get_forward_backward_func
    from beforeholiday_amd.transformer.pipeline_parallel import utils as pu
    from beforeholiday_amd.transformer.testing import commons

    hidden, mbs = 4, 2
    pu._reconfigure_microbatch_calculator(rank, None, mbs * num_micro, mbs, 1)
    chunks = vpp or 1
    n_layers = pp * chunks
    torch.manual_seed(0)
    weights = [torch.randn(hidden, hidden, dtype=torch.float64) * 0.3 for _ in range(n_layers)]
    biases = [torch.randn(hidden, dtype=torch.float64) * 0.1 for _ in range(n_layers)]
    batch = [torch.randn(mbs * num_micro, 1, hidden, dtype=torch.float64)]

    model = build_model(commons.model_provider_func, False, vpp, hidden_size=hidden)
    for c, m in enumerate(model):
        layer = c * pp + ps.get_pipeline_model_parallel_rank()  # chunk c of rank r holds layer c*pp + r
        m.double()
        with torch.no_grad():
            m.layer.layer.weight.copy_(weights[layer])
            m.layer.layer.bias.copy_(biases[layer])
    fwd_bwd = get_forward_backward_func(vpp, pp)
    losses = fwd_bwd(commons.fwd_step_func, batch, model if vpp else model[0], forward_only=forward_only,
                     tensor_shape=(mbs, 1, hidden), dtype=torch.float64)
    # reference: whole network in one process
    W = [w.clone().requires_grad_() for w in weights]
    B = [b.clone().requires_grad_() for b in biases]
    ref_losses = []
    for k in range(num_micro):
        y = batch[0][k * mbs:(k + 1) * mbs]
        for i in range(n_layers):
            y = F.linear(y, W[i], B[i])
        loss = y.sum()
        ref_losses.append(loss.detach())
        if not forward_only:
            (loss / num_micro).backward()
    if ps.is_pipeline_last_stage(ignore_virtual=True):
        assert len(losses) == num_micro
        for l, r in zip(losses, ref_losses):
            torch.testing.assert_close(l["avg"].view(()), r)
    else:
        assert losses == []
    if not forward_only:
        for c, m in enumerate(model):
            layer = c * pp + ps.get_pipeline_model_parallel_rank()
            torch.testing.assert_close(m.layer.layer.weight.grad, W[layer].grad)
            torch.testing.assert_close(m.layer.layer.bias.grad, B[layer].grad)
    pu.destroy_microbatch_calculator()
    ps.destroy_model_parallel()


@pytest.mark.parametrize("forward_only", [False, True])
def test_no_pipelining(forward_only):
    run_distributed(_pipeline, 1, 1, None, 4, forward_only)


@pytest.mark.parametrize("forward_only", [False, True])
def test_1f1b_pipelining(forward_only):
    run_distributed(_pipeline, 4, 4, None, 8, forward_only)


def test_1f1b_fewer_microbatches_than_stages():
    run_distributed(_pipeline, 4, 4, None, 2, False)


@pytest.mark.parametrize("num_micro", [4, 8])
def test_interleaved_pipelining(num_micro):
    run_distributed(_pipeline, 4, 4, 2, num_micro, False)


def _tp_pp_mlp(rank, world, sequence_parallel):
    """tp=2 x pp=2 toy parallel MLP through the 1F1B schedule (SP optional) — runs and agrees across TP."""
    ps = _init(2, 2)
    from beforeholiday_amd.transformer.pipeline_parallel import build_model, get_forward_backward_func
    from beforeholiday_amd.transformer.pipeline_parallel import utils as pu
    from beforeholiday_amd.transformer.testing import commons
    hidden, mbs, seq, nm = 8, 2, 4, 4
    pu._reconfigure_microbatch_calculator(rank, None, mbs * nm, mbs, 1)
    commons.set_random_seed(11)
    model = build_model(commons.mlp_provider_func, False, None, hidden_size=hidden,
                        sequence_parallel_enabled=sequence_parallel, use_cpu_initialization=True)
    torch.manual_seed(3)
    batch = [torch.randn(mbs * nm, seq, hidden)]
    fwd_bwd = get_forward_backward_func(None, 2)
    losses = fwd_bwd(commons.ToyParallelMLPFwdBwdStepFunc(sequence_parallel), batch, model[0], forward_only=False,
                     tensor_shape=(seq, mbs, hidden), dtype=torch.float32,
                     sequence_parallel_enabled=sequence_parallel)
    if ps.is_pipeline_last_stage():
        assert len(losses) == nm
        vals = torch.stack([l["avg"].view(()) for l in losses])
        assert torch.isfinite(vals).all()
        other = [torch.empty_like(vals) for _ in range(2)]
        torch.distributed.all_gather(other, vals, group=ps.get_tensor_model_parallel_group())
        if not sequence_parallel:
            torch.testing.assert_close(other[0], other[1])
    for p in model[0].parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()
    pu.destroy_microbatch_calculator()
    ps.destroy_model_parallel()


@pytest.mark.parametrize("sequence_parallel", [False, True])
def test_tp_pp_toy_mlp(sequence_parallel):
    run_distributed(_tp_pp_mlp, 4, sequence_parallel)


# ----------------------------------------------------------------------------------------------
def _grad_scaler(rank, world):
    ps = _init(world, 1)
    from beforeholiday_amd.transformer.amp import GradScaler
    p = torch.nn.Parameter(torch.ones(3))
    opt = torch.optim.SGD([p], lr=1.0)
    scaler = GradScaler(init_scale=4.0, device="cpu")
    loss = (p * (float("inf") if rank == 1 else 1.0)).sum()
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    # rank 1 overflowed -> every rank skipped and backed off
    torch.testing.assert_close(p.detach(), torch.ones(3))
    assert scaler.get_scale() == 2.0
    opt.zero_grad()
    scaler.scale(p.sum()).backward()
    scaler.step(opt)
    scaler.update()
    torch.testing.assert_close(p.detach(), torch.zeros(3))
    ps.destroy_model_parallel()


def test_mp_grad_scaler():
    run_distributed(_grad_scaler, 2)


# ----------------------------------------------------------------------------------------------
def test_microbatch_calculators():
    from beforeholiday_amd.transformer.microbatches import (ConstantNumMicroBatches, RampupBatchsizeNumMicroBatches,
                                                            build_num_microbatches_calculator)
    c = build_num_microbatches_calculator(0, None, 64, 4, 2)
    assert isinstance(c, ConstantNumMicroBatches) and c.get() == 8 and c.get_current_global_batch_size() == 64
    with pytest.raises(AssertionError):
        ConstantNumMicroBatches(30, 4, 2)
    r = build_num_microbatches_calculator(0, [16, 16, 64], 64, 4, 2)
    assert isinstance(r, RampupBatchsizeNumMicroBatches)
    assert r.get_current_global_batch_size() == 16 and r.get() == 2
    r.update(22, True)
    assert r.get_current_global_batch_size() == 32 and r.get() == 4
    r.update(1000, True)
    assert r.get_current_global_batch_size() == 64 and r.get() == 8


def test_batch_samplers():
    from beforeholiday_amd.transformer._data import MegatronPretrainingRandomSampler, MegatronPretrainingSampler
    seen = []
    for r in range(2):
        s = MegatronPretrainingSampler(20, 0, 4, r, 2)
        batches = list(s)
        assert all(len(b) == 4 for b in batches) and len(batches) == 2
        seen += [i for b in batches for i in b]
    assert sorted(seen) == list(range(16))
    seen = []
    for r in range(2):
        s = MegatronPretrainingRandomSampler(20, 0, 4, r, 2)
        batches = list(s)
        assert len(batches) == 2
        seen += [i for b in batches for i in b]
    assert sorted(seen) == list(range(16))
    # resume mid-epoch reproduces the tail of the permutation
    full = list(MegatronPretrainingRandomSampler(20, 0, 4, 0, 2))
    resumed = list(MegatronPretrainingRandomSampler(20, 8, 4, 0, 2))
    assert resumed == full[1:]


def test_ltor_masks():
    from beforeholiday_amd.transformer.pipeline_parallel.utils import get_ltor_masks_and_position_ids
    data = torch.tensor([[5, 1, 0, 7, 8], [1, 2, 3, 4, 0]])
    mask, loss_mask, pos = get_ltor_masks_and_position_ids(data, 0, True, True, True)
    assert mask.shape == (2, 1, 5, 5) and mask.dtype == torch.bool
    assert pos[0].tolist() == [0, 1, 2, 0, 1]
    assert loss_mask[0].tolist() == [1, 1, 0, 1, 1]
    assert mask[0, 0, 3, 1].item() and not mask[0, 0, 3, 3].item()


def _bda_masks(rank, world):
    """Bias-dropout-add masks across TP ranks: identical without sequence parallelism (replicas hold
    the same activations), different with it (each rank holds its own sequence shard). Covers both the
    fused kernel's host seed streams and the PyTorch fallback (forked model-parallel RNG)."""
    from beforeholiday_amd.models.transformer_lm import bias_dropout_add
    from beforeholiday_amd.transformer import tensor_parallel
    from beforeholiday_amd.transformer.tensor_parallel.random import dropout_seed

    _init(world, 1)
    torch.manual_seed(100 + rank)  # per-rank base seeds (as bench scripts do) must not matter
    tensor_parallel.model_parallel_cuda_manual_seed(1234)
    seeds = {mp: torch.tensor([dropout_seed(mp) for _ in range(4)]) for mp in (False, True)}
    x = torch.ones(64, 2, 32)
    masks = {mp: (bias_dropout_add(x, None, torch.zeros_like(x), 0.5, True, mp) != 0).float() for mp in (False, True)}
    for mp in (False, True):
        for t in (seeds[mp], masks[mp]):
            g = [torch.empty_like(t) for _ in range(world)]
            torch.distributed.all_gather(g, t)
            same = torch.equal(g[0], g[1])
            assert same == (not mp), (mp, t.dtype)


def test_bias_dropout_add_masks_across_tp_ranks():
    run_distributed(_bda_masks, 2)
