"""apex.RNN equivalents vs torch.nn.LSTM / GRU / RNN with copied weights."""
import pytest
import torch

from tests.conftest import devices


def _copy(cell, ref_layer_params):
    w_ih, w_hh, b_ih, b_hh = ref_layer_params
    with torch.no_grad():
        cell.w_ih.copy_(w_ih)
        cell.w_hh.copy_(w_hh)
        cell.b_ih.copy_(b_ih)
        cell.b_hh.copy_(b_hh)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("kind", ["LSTM", "GRU", "Tanh", "ReLU"])
def test_rnn_matches_torch(device, kind):
    from beforeholiday_amd import RNN
    torch.manual_seed(0)
    T, B, I, H, L = 7, 3, 10, 16, 2
    ours = getattr(RNN, kind)(I, H, L).to(device)
    if kind in ("LSTM", "GRU"):
        ref = getattr(torch.nn, kind)(I, H, L).to(device)
    else:
        ref = torch.nn.RNN(I, H, L, nonlinearity=kind.lower()).to(device)
    for l in range(L):
        _copy(ours.rnns[l], [getattr(ref, f"{n}_l{l}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")])
    x = torch.randn(T, B, I, device=device, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    out, hid = ours(x)
    out_r, hid_r = ref(xr)
    torch.testing.assert_close(out, out_r, rtol=1e-4, atol=1e-5)
    h_r = hid_r[0] if kind == "LSTM" else hid_r
    torch.testing.assert_close(hid[0], h_r, rtol=1e-4, atol=1e-5)
    out.sum().backward()
    out_r.sum().backward()
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("device", devices())
def test_bidirectional_and_mlstm(device):
    from beforeholiday_amd import RNN
    torch.manual_seed(1)
    T, B, I, H = 5, 2, 6, 8
    bi = RNN.LSTM(I, H, 2, bidirectional=True).to(device)
    out, hid = bi(torch.randn(T, B, I, device=device))
    assert out.shape == (T, B, 2 * H) and hid[0].shape == (2, B, 2 * H)
    m = RNN.mLSTM(I, H, 1, output_size=5).to(device)
    out, hid = m(torch.randn(T, B, I, device=device))
    assert out.shape == (T, B, 5)
    out.sum().backward()
    assert m.rnns[0].w_mih.grad is not None
