"""Replayable dropout seeds (utils/graph_rng.py): a per-call salt fixed by the call's position in the step
plus a device step seed the kernels read (kernels/attn.hip eff_seed, kernels/dense.hip bias-dropout-add).
Checks the host bookkeeping on the CPU, and on the GPU that (a) a device-seeded kernel computes exactly what
the host-seeded kernel computes with the combined seed, (b) a captured step replays to the eager step's bits
from the same step seed and draws new masks on the next replay."""
import pytest
import torch

G = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def test_salts_repeat_per_step_and_differ_per_call():
    from beforeholiday_amd.utils import graph_rng

    graph_rng._step_seed, graph_rng._calls = torch.zeros(1, dtype=torch.int64), 0  # CPU stand-in
    try:
        graph_rng.new_step()
        a = [graph_rng.next_salt(), graph_rng.next_salt(), graph_rng.next_salt(1)]
        graph_rng.new_step()
        b = [graph_rng.next_salt(), graph_rng.next_salt(), graph_rng.next_salt(1)]
        assert a == b and len(set(a)) == 3
        assert int(graph_rng.step_seed()) == 2
        assert graph_rng.state_tensors() == [graph_rng.step_seed()]
    finally:
        graph_rng.disable()
    assert not graph_rng.active() and graph_rng.state_tensors() == []


def _signed(v):
    return v - (1 << 64) if v >= 1 << 63 else v


@pytest.mark.gpu
def test_device_seed_equals_combined_host_seed(monkeypatch):
    """Flash attention (forward and the regenerated mask in backward) and bias-dropout-add under a device
    step seed S and salt s equal the host-seeded kernels with seed s ^ (S * golden)."""
    from beforeholiday_amd.contrib.multihead_attn import _core
    from beforeholiday_amd.ops.fused_dense import bias_dropout_add
    from beforeholiday_amd.utils import graph_rng

    torch.manual_seed(0)
    s, heads, b = 384, 4, 2
    qkv = torch.randn(s, b * heads, 3, 64, device="cuda", dtype=torch.float16, requires_grad=True)
    dout = torch.randn(s, b * heads, 64, device="cuda", dtype=torch.float16)
    x = torch.randn(512, 1024, device="cuda", dtype=torch.float16)
    r = torch.randn_like(x)
    salt = 123457
    monkeypatch.setattr(graph_rng, "next_salt", lambda stream=0: salt)
    graph_rng.enable(seed=7)
    try:
        graph_rng.new_step()  # step seed 8
        o_dev = _core.FusedSelfAttnFn.apply(qkv, heads, 0.125, None, _core.MASK_NONE, 0.3, True)
        (g_dev,) = torch.autograd.grad(o_dev, qkv, dout)
        y_dev = bias_dropout_add(x, None, r, 0.4, True)
    finally:
        graph_rng.disable()
    eff = salt ^ ((8 * G) & M64)
    monkeypatch.setattr(_core, "_seed", lambda: _signed(eff))
    o_host = _core.FusedSelfAttnFn.apply(qkv, heads, 0.125, None, _core.MASK_NONE, 0.3, True)
    (g_host,) = torch.autograd.grad(o_host, qkv, dout)
    assert torch.equal(o_dev, o_host) and torch.equal(g_dev, g_host)
    import beforeholiday_amd.transformer.tensor_parallel.random as rnd

    eff32 = (salt & 0xFFFFFFFF) ^ ((((8 * G) & M64) >> 32) & 0xFFFFFFFF)
    monkeypatch.setattr(rnd, "dropout_seed", lambda model_parallel=False: eff32)
    y_host = bias_dropout_add(x, None, r, 0.4, True)
    assert torch.equal(y_dev, y_host)
    assert not torch.equal(y_dev, r)  # dropout did something


@pytest.mark.gpu
def test_captured_step_replays_eager_bits_and_advances():
    from beforeholiday_amd.contrib.multihead_attn import _core
    from beforeholiday_amd.ops.fused_dense import bias_dropout_add
    from beforeholiday_amd.utils import GraphedStep, graph_rng

    torch.manual_seed(1)
    s, heads, b = 256, 4, 2
    qkv = torch.randn(s, b * heads, 3, 64, device="cuda", dtype=torch.float16)
    x = torch.randn(256, 512, device="cuda", dtype=torch.float16)
    graph_rng.enable(seed=3)
    try:
        def fn():
            graph_rng.new_step()
            o = _core.FusedSelfAttnFn.apply(qkv, heads, 0.125, None, _core.MASK_NONE, 0.2, True)
            y = bias_dropout_add(x, None, torch.zeros_like(x), 0.5, True)
            return o.float().sum() + y.float().sum()

        e1, e2 = fn().item(), fn().item()
        assert e1 != e2  # a new step seed draws new masks
        g = GraphedStep(fn, warmup=1)
        g.capture()
        seed = graph_rng.step_seed()
        s0 = seed.clone()
        rep = g().clone()
        seed.copy_(s0)
        eag = fn().clone()
        assert torch.equal(rep, eag)
        rep2 = g().clone()
        assert not torch.equal(rep2, rep)
        assert int(seed) == int(s0) + 2
    finally:
        graph_rng.disable()


def test_checkpoint_recompute_reuses_salts():
    """An activation-checkpoint recompute (tensor_parallel.random.CheckpointFunction) replays the per-step
    call counter, so the recomputed dropout calls get the forward's salts (same masks)."""
    from beforeholiday_amd.transformer.tensor_parallel.random import checkpoint
    from beforeholiday_amd.utils import graph_rng

    seen = []

    def f(x):
        seen.append(graph_rng.next_salt())
        return x * 2

    graph_rng._step_seed, graph_rng._calls = torch.zeros(1, dtype=torch.int64), 0  # CPU stand-in
    try:
        x = torch.randn(4, requires_grad=True)
        y = checkpoint(f, False, x)
        after = graph_rng._calls
        y.sum().backward()
        assert len(seen) == 2 and seen[0] == seen[1]
        assert graph_rng._calls == after  # the backward's own counter is restored after the recompute
        assert torch.equal(x.grad, torch.full((4,), 2.0))
    finally:
        graph_rng.disable()
