"""RNN-T loss / joint vs an autograd reference (reference tests: apex/contrib/test/transducer/)."""
import pytest
import torch

from tests.conftest import devices


def _autograd_loss(x, label, f_len, y_len, blank):
    """-log P(y|x) per sequence with the alpha recursion in differentiable torch ops."""
    logp = torch.log_softmax(x.double(), -1)
    losses = []
    for b in range(x.size(0)):
        T, U = int(f_len[b]), int(y_len[b])
        alpha = [[None] * (U + 1) for _ in range(T)]
        for t in range(T):
            for u in range(U + 1):
                if t == 0 and u == 0:
                    alpha[t][u] = logp.new_zeros(())
                    continue
                terms = []
                if t > 0:
                    terms.append(alpha[t - 1][u] + logp[b, t - 1, u, blank])
                if u > 0:
                    terms.append(alpha[t][u - 1] + logp[b, t, u - 1, label[b, u - 1]])
                alpha[t][u] = torch.logsumexp(torch.stack(terms), 0)
        losses.append(-(alpha[T - 1][U] + logp[b, T - 1, U, blank]))
    return torch.stack(losses)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_transducer_loss(device, fuse, dtype):
    if device == "cpu" and dtype != torch.float32:
        pytest.skip("fp32 on CPU")
    from beforeholiday_amd.contrib.transducer import TransducerLoss
    torch.manual_seed(0)
    B, T, U, V, blank = 3, 6, 4, 9, 0
    f_len = torch.tensor([6, 4, 5], dtype=torch.int32)
    y_len = torch.tensor([4, 2, 3], dtype=torch.int32)
    label = torch.randint(1, V, (B, U))
    x = torch.randn(B, T, U + 1, V)
    xa = x.detach().clone().to(device, dtype).requires_grad_()
    loss = TransducerLoss(fuse_softmax_backward=fuse)(xa, label.to(device), f_len.to(device), y_len.to(device), blank)
    xr = x.detach().double().requires_grad_()
    ref = _autograd_loss(xr, label, f_len, y_len, blank)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(loss.double().cpu(), ref.detach(), rtol=tol, atol=tol)
    w = torch.rand(B, dtype=torch.float64)
    (loss.double().cpu() * w).sum().backward()
    (ref * w).sum().backward()
    g = xa.grad.double().cpu()
    for b in range(B):  # only the valid lattice region carries gradient
        torch.testing.assert_close(g[b, :f_len[b], :y_len[b] + 1], xr.grad[b, :f_len[b], :y_len[b] + 1],
                                   rtol=tol, atol=tol)
        assert g[b, f_len[b]:].abs().sum() == 0


@pytest.mark.parametrize("device", devices())
def test_transducer_loss_packed(device):
    from beforeholiday_amd.contrib.transducer import TransducerLoss
    torch.manual_seed(1)
    B, T, U, V, blank = 2, 5, 3, 7, 0
    f_len = torch.tensor([5, 3])
    y_len = torch.tensor([3, 1])
    label = torch.randint(1, V, (B, U))
    x = torch.randn(B, T, U + 1, V)
    padded = TransducerLoss()(x.to(device), label.to(device), f_len.to(device), y_len.to(device), blank)
    rows = [x[b, :f_len[b], :y_len[b] + 1].reshape(-1, V) for b in range(B)]
    xp = torch.cat(rows).to(device).requires_grad_()
    bo = torch.cumsum(f_len * (y_len + 1), 0).to(device)
    packed = TransducerLoss(packed_input=True)(xp, label.to(device), f_len.to(device), y_len.to(device), blank,
                                               batch_offset=bo, max_f_len=T)
    torch.testing.assert_close(packed, padded, rtol=1e-5, atol=1e-5)
    packed.sum().backward()
    assert torch.isfinite(xp.grad).all()


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("pack", [False, True])
@pytest.mark.parametrize("relu", [False, True])
def test_transducer_joint(device, pack, relu):
    from beforeholiday_amd.contrib.transducer import TransducerJoint
    torch.manual_seed(2)
    B, T, U, H = 2, 5, 4, 8
    f = torch.randn(B, T, H, device=device, requires_grad=True)
    g = torch.randn(B, U, H, device=device, requires_grad=True)
    f_len = torch.tensor([5, 3], device=device)
    g_len = torch.tensor([4, 2], device=device)
    bo = torch.cumsum(f_len * g_len, 0)
    j = TransducerJoint(pack_output=pack, relu=relu)
    h = j(f, g, f_len, g_len, batch_offset=bo, packed_batch=int(bo[-1]))
    fr, gr = f.detach().clone().requires_grad_(), g.detach().clone().requires_grad_()
    hr = fr.unsqueeze(2) + gr.unsqueeze(1)
    if relu:
        hr = torch.relu(hr)
    rows = [hr[b, :f_len[b], :g_len[b]].reshape(-1, H) for b in range(B)]
    if pack:
        ref = torch.cat(rows)
        torch.testing.assert_close(h, ref)
    else:
        for b in range(B):
            torch.testing.assert_close(h[b, :f_len[b], :g_len[b]], hr[b, :f_len[b], :g_len[b]])
        ref = torch.cat(rows)
    gh = torch.randn_like(ref)
    ref.backward(gh)
    if pack:
        h.backward(gh)
    else:
        full = torch.zeros_like(h)
        off = 0
        for b in range(B):
            n = int(f_len[b] * g_len[b])
            full[b, :f_len[b], :g_len[b]] = gh[off:off + n].view(int(f_len[b]), int(g_len[b]), H)
            off += n
        h.backward(full)
    torch.testing.assert_close(f.grad, fr.grad)
    torch.testing.assert_close(g.grad, gr.grad)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("pack", [False, True])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_transducer_joint_dropout_with_probe(device, pack, relu, dtype):
    """Fused ReLU + dropout: the probed mask drives an fp32 reference for the output and both input
    gradients (the HIP backward regenerates the dropout bits from the counter hash)."""
    from beforeholiday_amd.contrib.transducer import TransducerJoint
    torch.manual_seed(3)
    B, T, U, H, p = 3, 7, 9, 64, 0.3
    f = torch.randn(B, T, H, device=device).to(dtype).requires_grad_()
    g = torch.randn(B, U, H, device=device).to(dtype).requires_grad_()
    f_len = torch.tensor([7, 4, 1], device=device)
    g_len = torch.tensor([9, 5, 2], device=device)
    bo = torch.cumsum(f_len * g_len, 0)
    j = TransducerJoint(pack_output=pack, relu=relu, dropout=True, dropout_prob=p, probe_mask=True)
    j.train()
    h = j(f, g, f_len, g_len, batch_offset=bo, packed_batch=int(bo[-1]))
    mask = j.mask_probe[-1].float()
    assert mask.shape == h.shape
    hr = f.detach().float().unsqueeze(2) + g.detach().float().unsqueeze(1)
    rows = [hr[b, :f_len[b], :g_len[b]].reshape(-1, H) for b in range(B)]
    ref_in = torch.cat(rows)
    if pack:
        m_valid = mask
    else:
        m_valid = torch.cat([mask[b, :f_len[b], :g_len[b]].reshape(-1, H) for b in range(B)])
    if relu:
        assert bool(((ref_in <= 0) & (m_valid > 0)).sum() <= 2)  # relu'd elements are masked (bf16 ties aside)
    keep_frac = m_valid.mean().item()
    want = (1 - p) * (0.5 if relu else 1.0)
    assert abs(keep_frac - want) < 0.05, keep_frac
    ref_out = ref_in * m_valid / (1 - p)
    got = h if pack else torch.cat([h[b, :f_len[b], :g_len[b]].reshape(-1, H) for b in range(B)])
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(got.float(), ref_out, rtol=tol, atol=tol)
    gh = torch.randn_like(ref_out)
    if pack:
        h.backward(gh.to(dtype))
    else:
        full = torch.zeros(h.shape, dtype=dtype, device=device)
        off = 0
        for b in range(B):
            n = int(f_len[b] * g_len[b])
            full[b, :f_len[b], :g_len[b]] = gh[off:off + n].view(int(f_len[b]), int(g_len[b]), H).to(dtype)
            off += n
        h.backward(full)
    gm = gh.to(dtype).float() * m_valid / (1 - p)
    df = torch.zeros(B, T, H, device=device)
    dg = torch.zeros(B, U, H, device=device)
    off = 0
    for b in range(B):
        fl, gl = int(f_len[b]), int(g_len[b])
        blk = gm[off:off + fl * gl].view(fl, gl, H)
        df[b, :fl] = blk.sum(1)
        dg[b, :gl] = blk.sum(0)
        off += fl * gl
    torch.testing.assert_close(f.grad.float(), df, rtol=tol, atol=tol * 4)
    torch.testing.assert_close(g.grad.float(), dg, rtol=tol, atol=tol * 4)
