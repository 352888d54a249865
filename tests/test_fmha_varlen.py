"""Packed variable-length FMHA on the flash kernels (contrib/fmha/fmha.py ``FlashVarlenFn``;
reference: apex/contrib/fmha/fmha.py:34-76 with ``cu_seqlens`` taken by fmhalib fwd / bwd,
apex/contrib/csrc/fmha/fmha_api.cpp:358-360).

Checked against per-sequence fp32 attention (forward and d(qkv)): long and short sequences in one
batch (several 64-key blocks, partial tiles, a one-token and an empty sequence), a max_s larger than
every length, causal masking, dropout determinism, and a forward + backward captured in a HIP graph
and replayed on new data (no host read of the lengths anywhere)."""
import types

import pytest
import torch


def _ref(qkv, lens, h, d, causal=False):
    q3 = qkv.float().view(-1, 3, h, d)
    outs, s0 = [], 0
    for n in lens:
        q, k, v = (q3[s0:s0 + n, j].transpose(0, 1) for j in range(3))  # [h, n, d]
        s = q @ k.transpose(-1, -2) / d ** 0.5
        if causal:
            s = s.masked_fill(torch.ones(n, n, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
        outs.append((torch.softmax(s, -1) @ v).transpose(0, 1).reshape(n, h * d))
        s0 += n
    return torch.cat(outs)


def _cu(lens):
    return torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")


def _fmha(h, d, p=0.0):
    from beforeholiday_amd.contrib.fmha import FMHA

    return FMHA(types.SimpleNamespace(attention_probs_dropout_prob=p, num_attention_heads=h, hidden_size=h * d))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
def test_varlen_matches_per_sequence_fp32(dtype, causal):
    from beforeholiday_amd.contrib.fmha.fmha import fmha_varlen

    torch.manual_seed(0)
    h, d = 4, 64
    lens = [300, 1, 0, 129, 64, 517]
    max_s = 600
    qkv = torch.randn(sum(lens), 3 * h * d, device="cuda", dtype=dtype, requires_grad=True)
    cu = _cu(lens)
    out = fmha_varlen(qkv.view(-1, 3, h, d), cu, 0.0, max_s, True, causal=causal).reshape(-1, h * d)
    qf = qkv.detach().float().requires_grad_(True)
    ref = _ref(qf, lens, h, d, causal)
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)
    g = torch.randn_like(out)
    g1 = torch.autograd.grad(out, qkv, g)[0]
    g2 = torch.autograd.grad(ref, qf, g.float())[0]
    torch.testing.assert_close(g1.float(), g2, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_varlen_module_and_dropout():
    """The reference module API; dropout is regenerated from the seed (same seed -> same output),
    p is ignored outside training, and the gradients are finite."""
    from beforeholiday_amd.contrib.multihead_attn import _core

    torch.manual_seed(1)
    h, d = 2, 64
    lens = [200, 77]
    qkv = torch.randn(sum(lens), 3 * h * d, device="cuda", dtype=torch.float16, requires_grad=True)
    cu = _cu(lens)
    m = _fmha(h, d, p=0.2)
    ref = _ref(qkv.detach(), lens, h, d)
    torch.testing.assert_close(m(qkv, cu, 256, is_training=False).float(), ref, rtol=2e-2, atol=2e-2)
    seed = _core._seed
    try:
        _core._seed = lambda: 1234
        import beforeholiday_amd.contrib.fmha.fmha as fm

        fm._seed = _core._seed
        a = m(qkv, cu, 256, is_training=True)
        b = m(qkv, cu, 256, is_training=True)
    finally:
        _core._seed = seed
        fm._seed = seed
    assert torch.equal(a, b)
    assert not torch.allclose(a.float(), ref, atol=1e-2)  # something was dropped
    (gq,) = torch.autograd.grad(a.float().sum(), qkv)
    assert torch.isfinite(gq).all()


@pytest.mark.gpu
def test_varlen_graph_capture():
    """Forward + backward captured once, replayed on new contents of the same buffers: the lengths
    live in a device tensor, so a replay with different lengths (same max_s) is honoured."""
    from beforeholiday_amd.contrib.fmha.fmha import fmha_varlen

    torch.manual_seed(2)
    h, d, total, max_s = 2, 64, 384, 256
    qkv = torch.randn(total, 3, h, d, device="cuda", dtype=torch.float16, requires_grad=True)
    cu = _cu([256, 128])
    g = torch.randn(total, h, d, device="cuda", dtype=torch.float16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up (allocator, plans) off the capture
        for _ in range(2):
            qkv.grad = None
            fmha_varlen(qkv, cu, 0.0, max_s, True).backward(g)
    torch.cuda.current_stream().wait_stream(s)
    qkv.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fmha_varlen(qkv, cu, 0.0, max_s, True)
        out.backward(g)
    for lens in ([128, 256], [256, 128], [192, 192]):
        with torch.no_grad():
            qkv.copy_(torch.randn_like(qkv))
        cu.copy_(_cu(lens))
        graph.replay()
        torch.cuda.synchronize()
        qf = qkv.detach().float().reshape(total, -1).requires_grad_(True)
        ref = _ref(qf, lens, h, d)
        torch.testing.assert_close(out.float().reshape(total, -1), ref, rtol=2e-2, atol=2e-2)
        gref = torch.autograd.grad(ref, qf, g.float().reshape(total, -1))[0]
        torch.testing.assert_close(qkv.grad.float().reshape(total, -1), gref, rtol=2e-2, atol=2e-2)
