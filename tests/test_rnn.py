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


# ---------------------------------------------------------------------------------------------
# amp O1 / O4 casting of torch.nn recurrent layers (reference: tests/L0/run_amp/test_rnn.py:11-121)
# ---------------------------------------------------------------------------------------------
def _amp_cases():
    return [pytest.param("cpu", torch.bfloat16),
            pytest.param("cuda", torch.float16, marks=pytest.mark.gpu),
            pytest.param("cuda", torch.bfloat16, marks=pytest.mark.gpu)]


@pytest.fixture
def amp_handle(request):
    from beforeholiday_amd import amp
    handles = []

    def make(dtype):
        h = amp.init(enabled=True, patch_type=dtype)
        handles.append(h)
        return h

    yield make
    for h in handles:
        h._deactivate()
    amp.deactivate()


@pytest.mark.parametrize("device,dtype", _amp_cases())
@pytest.mark.parametrize("kind", ["RNNCell", "GRUCell", "LSTMCell"])
def test_amp_rnn_cells_run_low_precision(amp_handle, device, dtype, kind):
    amp_handle(dtype)
    torch.manual_seed(0)
    b, h, t = 4, 16, 3
    cell = getattr(torch.nn, kind)(h, h).to(device)
    for in_dt in (torch.float32, dtype):
        xs = [torch.randn(b, h, device=device, dtype=in_dt, requires_grad=True) for _ in range(t)]
        hid = torch.zeros(b, h, device=device, dtype=in_dt)
        hid = (hid, hid.clone()) if kind == "LSTMCell" else hid
        outs = []
        for x in xs:
            hid = cell(x, hid)
            outs.append(hid[0] if kind == "LSTMCell" else hid)
        assert all(o.dtype == dtype for o in outs)
        outs[-1].float().sum().backward()
        for x in xs:
            assert x.grad.dtype == x.dtype
        assert all(p.grad.dtype == torch.float32 for p in cell.parameters())


@pytest.mark.parametrize("device,dtype", _amp_cases())
@pytest.mark.parametrize("kind", ["RNN", "GRU", "LSTM"])
@pytest.mark.parametrize("layers,bidir", [(1, False), (2, False), (2, True)])
def test_amp_rnns_run_low_precision(amp_handle, device, dtype, kind, layers, bidir):
    amp_handle(dtype)
    torch.manual_seed(0)
    t, b, h = 5, 3, 16
    kw = dict(nonlinearity="relu") if kind == "RNN" else {}
    rnn = getattr(torch.nn, kind)(input_size=h, hidden_size=h, num_layers=layers, bidirectional=bidir, **kw).to(device)
    ref = getattr(torch.nn, kind)(input_size=h, hidden_size=h, num_layers=layers, bidirectional=bidir, **kw).to(device)
    ref.load_state_dict(rnn.state_dict())
    for in_dt in (torch.float32, dtype):
        x = torch.randn(t, b, h, device=device, dtype=in_dt, requires_grad=True)
        hid = torch.zeros(layers * (2 if bidir else 1), b, h, device=device, dtype=in_dt)
        hid = (hid, hid.clone()) if kind == "LSTM" else hid
        out, _ = rnn(x, hid)
        assert out.dtype == dtype
        out[-1].float().sum().backward()
        assert x.grad.dtype == x.dtype
        assert all(p.grad is not None and p.grad.dtype == torch.float32 for p in rnn.parameters())
    # numerics: the low-precision run tracks an fp32 run of the same weights (casts off)
    from beforeholiday_amd import amp
    xr = torch.randn(t, b, h, device=device)
    with amp.disable_casts():
        want, _ = ref(xr)
    got, _ = rnn(xr)
    torch.testing.assert_close(got.float(), want, rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("device,dtype", _amp_cases())
def test_amp_lstm_packed_sequence(amp_handle, device, dtype):
    amp_handle(dtype)
    torch.manual_seed(1)
    h, b = 8, 3
    lens = [5, 3, 2]
    rnn = torch.nn.LSTM(h, h, num_layers=2, bidirectional=True).to(device)
    x = torch.randn(max(lens), b, h, device=device, requires_grad=True)
    packed = torch.nn.utils.rnn.pack_padded_sequence(x, lens)
    out, (hn, cn) = rnn(packed)
    assert out.data.dtype == dtype and hn.dtype == dtype
    padded, _ = torch.nn.utils.rnn.pad_packed_sequence(out)
    padded.float().sum().backward()
    assert x.grad.dtype == torch.float32
    assert all(p.grad.dtype == torch.float32 for p in rnn.parameters())


def test_amp_rnn_patch_is_removed_on_deactivate():
    from beforeholiday_amd import amp
    import torch.nn.modules.rnn as rnn_mod

    orig = rnn_mod._VF
    h = amp.init(enabled=True, patch_type=torch.bfloat16)
    assert rnn_mod._VF is not orig
    h._deactivate()
    amp.deactivate()
    assert rnn_mod._VF is orig
    out, _ = torch.nn.LSTM(4, 4)(torch.randn(2, 1, 4))
    assert out.dtype == torch.float32
