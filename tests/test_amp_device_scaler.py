"""Device-resident dynamic loss scaling (BH_AMP_DEVICE_SCALER=1, amp/scaler.py ``enable_device_mode``):
no host sync per step, the overflow flag is the fused optimizer's noop flag.

Checked on the GPU against the host scaler (the reference's behaviour, apex/amp/scaler.py:197-226):
matching parameter trajectories and identical loss scales while no step overflows (including a scale
growth after ``scale_window`` clean steps), and on an injected overflow: parameters unchanged by
the skipped step and the scale halved."""
import pytest
import torch

from beforeholiday_amd import config
import torch.nn.functional as F


def _run(device_mode, steps, inf_at=None, monkeypatch=None, window=3, init_scale=256.0, micro=1, state=None):
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp._amp_state import _amp_state
    from beforeholiday_amd.optimizers import FusedLAMB

    config.set(amp_device_scaler=device_mode)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.BatchNorm1d(64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 8)).cuda()
    opt = FusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01)
    model, opt = amp.initialize(model, opt, opt_level="O2", keep_batchnorm_fp32=True, verbosity=0,
                                loss_scale="dynamic")
    _amp_state.loss_scalers[0]._scale_seq_len = window
    _amp_state.loss_scalers[0]._loss_scale = init_scale  # before the first scale_loss (device mode copies it)
    x = torch.randn(16, 32, device="cuda", dtype=torch.half)
    y = torch.randint(0, 8, (16,), device="cuda")
    scales, snaps = [], []
    for i in range(steps):
        for m in range(micro):  # gradient accumulation: one scale_loss per micro-batch
            loss = F.cross_entropy(model(x[m::micro]).float(), y[m::micro])
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
                if inf_at == i and m == 0:
                    next(model.parameters()).grad.view(-1)[0] = float("inf")
        if state is not None and i == 1:
            state.append(amp.state_dict())
        opt.step()
        opt.zero_grad()
        scales.append(_amp_state.loss_scalers[0].loss_scale())
        snaps.append([p.detach().float().clone() for p in model.parameters()])
    device_used = _amp_state.loss_scalers[0].device_mode
    amp.deactivate() if hasattr(amp, "deactivate") else None
    return scales, snaps, device_used


@pytest.mark.gpu
def test_device_scaler_matches_host_without_overflow(monkeypatch):
    s_host, p_host, dev0 = _run(False, 5, monkeypatch=monkeypatch)
    s_dev, p_dev, dev1 = _run(True, 5, monkeypatch=monkeypatch)
    assert not dev0 and dev1
    assert s_host == s_dev and s_host[-1] > s_host[0]  # grew after the window, identically
    # same arithmetic (5 steps from scale 256 with one growth: no step overflows); the device step
    # counter's bias corrections come from fp32 powf instead of the host's double pow: equal to rounding
    for a, b in zip(p_host, p_dev):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_device_scaler_overflow_skips_on_device(monkeypatch):
    s_dev, p_dev, used = _run(True, 4, inf_at=2, monkeypatch=monkeypatch, window=100)
    assert used
    assert s_dev[2] == s_dev[1] / 2  # halved on the overflowing step
    for u, v in zip(p_dev[1], p_dev[2]):  # the skipped step left every parameter unchanged
        assert torch.equal(u, v)
    assert any(not torch.equal(u, v) for u, v in zip(p_dev[2], p_dev[3]))  # and training goes on


@pytest.mark.gpu
def test_device_scaler_matches_host_with_overflow(monkeypatch):
    """An overflowing step is skipped on the host (reference) or on the device (noop flag + device
    step counter): the same parameters afterwards (to the bias-correction rounding) and scales."""
    s_host, p_host, _ = _run(False, 5, inf_at=2, monkeypatch=monkeypatch, window=100)
    s_dev, p_dev, used = _run(True, 5, inf_at=2, monkeypatch=monkeypatch, window=100)
    assert used and s_host == s_dev
    for a, b in zip(p_host, p_dev):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_device_scaler_accumulation_overflow_in_first_micro_batch(monkeypatch):
    """Two micro-batches per step, an Inf in the FIRST one: the device path must still skip the whole
    step (the per-pass flag is cleared by the second pass, the step-level flag is not) and unscale the
    accumulated grads with the device scale -- same trajectory and scales as the host reference."""
    s_host, p_host, _ = _run(False, 5, inf_at=2, monkeypatch=monkeypatch, window=100, micro=2)
    s_dev, p_dev, used = _run(True, 5, inf_at=2, monkeypatch=monkeypatch, window=100, micro=2)
    assert used and s_host == s_dev
    for u, v in zip(p_dev[1], p_dev[2]):
        assert torch.equal(u, v)  # skipped
    for a, b in zip(p_host, p_dev):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_device_scaler_accumulation_after_scale_change(monkeypatch):
    """Accumulated grads after the device scale has grown: unscaled by the device value (the host
    ``_loss_scale`` is stale in device mode)."""
    s_host, p_host, _ = _run(False, 6, monkeypatch=monkeypatch, window=2, micro=2)
    s_dev, p_dev, used = _run(True, 6, monkeypatch=monkeypatch, window=2, micro=2)
    assert used and s_host == s_dev and s_host[-1] > s_host[0]
    for a, b in zip(p_host, p_dev):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_device_scaler_state_dict_roundtrip(monkeypatch):
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp._amp_state import _amp_state

    st_host, st_dev = [], []
    _run(False, 3, monkeypatch=monkeypatch, window=100, state=st_host)
    _run(True, 3, monkeypatch=monkeypatch, window=100, state=st_dev)
    assert st_host[0] == st_dev[0]  # the device counter, not the never-updated host one
    sd = {"loss_scaler0": {"loss_scale": 1024.0, "unskipped": 7}}
    amp.load_state_dict(sd)
    sc = _amp_state.loss_scalers[0]
    assert sc.device_mode and sc.loss_scale() == 1024.0 and sc.unskipped() == 7
