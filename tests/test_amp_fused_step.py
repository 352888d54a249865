"""Fused mixed-precision optimizer step under amp O2 / O5 (amp/_process_optimizer.py, module docstring):
FusedLAMB / FusedAdam read the loss-scaled 16-bit model gradients with the device inverse scale,
update the fp32 masters and write the 16-bit model parameters in the same launches -- no fp32 master
gradients, no master-to-model copy (reference: csrc/multi_tensor_lamb_mp.cu:41,248,367).

Checked on the GPU against the unfused sequence (unscale into fp32 master grads, step, copy back):
parameter and master trajectories and loss scales, with and without an injected overflow, host and
device-resident loss scale, gradient accumulation (a second backward materialises the pending step),
``amp.master_params`` (materialises the master gradients before it yields), and O5 (bf16, no scale)."""
import pytest
import torch

from beforeholiday_amd import config
import torch.nn.functional as F


def _run(monkeypatch, fused, opt_name="lamb", device_mode=True, steps=5, inf_at=None, micro=1, opt_level="O2",
         window=100, probe=None):
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp import _process_optimizer
    from beforeholiday_amd.amp._amp_state import _amp_state
    from beforeholiday_amd.optimizers import FusedAdam, FusedLAMB

    config.set(amp_device_scaler=device_mode)
    config.set(amp_fused_master_step=fused)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.BatchNorm1d(64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 24), torch.nn.ReLU(), torch.nn.Linear(24, 8)).cuda()
    if opt_name == "lamb":
        opt = FusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    else:
        opt = FusedAdam(model.parameters(), lr=1e-2, weight_decay=0.01)
    kw = dict(loss_scale="dynamic") if opt_level == "O2" else {}
    model, opt = amp.initialize(model, opt, opt_level=opt_level, keep_batchnorm_fp32=True, verbosity=0, **kw)
    if opt_level == "O2":
        _amp_state.loss_scalers[0]._scale_seq_len = window
        _amp_state.loss_scalers[0]._loss_scale = 256.0
    dt = torch.half if opt_level == "O2" else torch.bfloat16
    x = torch.randn(16, 32, device="cuda", dtype=dt)
    y = torch.randint(0, 8, (16,), device="cuda")
    plan = opt._amp_stash.plan
    scales, snaps, masters, pending = [], [], [], []
    for i in range(steps):
        for m in range(micro):
            loss = F.cross_entropy(model(x[m::micro]).float(), y[m::micro])
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
                if inf_at == i and m == 0:
                    next(model.parameters()).grad.view(-1)[0] = float("inf")
            pending.append(plan.fused_pending())
        if probe is not None and i == 1:
            probe.append([None if p.grad is None else p.grad.clone() for p in amp.master_params(opt)])
        opt.step()
        opt.zero_grad()
        scales.append(_amp_state.loss_scalers[0].loss_scale())
        snaps.append([p.detach().clone() for p in model.parameters()])
        masters.append([p.detach().clone() for p in amp.master_params(opt)])
    return scales, snaps, masters, pending


def _close(a, b, exact):
    """Trajectories equal (``exact``) or to rounding: the fused kernels are other instantiations of the
    same arithmetic (16-bit gradient operand), so the compiler's FMA contraction may round differently;
    a 16-bit parameter may then land one ulp apart."""
    for u, v in zip(a, b):
        for s, t in zip(u, v):
            if exact:
                assert torch.equal(s, t)
            elif s.dtype == torch.float32:
                torch.testing.assert_close(s, t, rtol=1e-5, atol=1e-6)
            else:
                torch.testing.assert_close(s.float(), t.float(), rtol=0, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["lamb", "adam"])
@pytest.mark.parametrize("device_mode", [True, False])
@pytest.mark.parametrize("inf_at", [None, 2])
def test_fused_step_matches_unfused(monkeypatch, opt_name, device_mode, inf_at):
    s_ref, p_ref, m_ref, pend_ref = _run(monkeypatch, False, opt_name, device_mode, inf_at=inf_at)
    s_fus, p_fus, m_fus, pend_fus = _run(monkeypatch, True, opt_name, device_mode, inf_at=inf_at)
    assert not any(pend_ref) and all(pend_fus)  # the fused path really ran, the reference did not
    assert s_ref == s_fus
    if inf_at is not None:
        assert s_fus[inf_at] == s_fus[inf_at - 1] / 2
        for u, v in zip(p_fus[inf_at - 1], p_fus[inf_at]):  # the overflowing step changed nothing
            assert torch.equal(u, v)
    # equal to rounding: other kernel instantiations, and LAMB's global norm blends the 16-bit and the
    # fp32 (BatchNorm) gradient norms in another order
    _close(m_ref, m_fus, False)
    _close(p_ref, p_fus, False)


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["lamb", "adam"])
def test_fused_step_accumulation(monkeypatch, opt_name):
    """Two micro-batches per step: the second backward materialises the pending fused step into fp32
    master gradients, and the step runs unfused -- identical to the unfused path throughout, including
    an overflow in the first micro-batch."""
    s_ref, p_ref, m_ref, _ = _run(monkeypatch, False, opt_name, True, inf_at=2, micro=2)
    s_fus, p_fus, m_fus, pend = _run(monkeypatch, True, opt_name, True, inf_at=2, micro=2)
    assert pend[0] and not pend[1]  # pending after the first micro-batch, materialised by the second
    assert s_ref == s_fus
    _close(m_ref, m_fus, True)
    _close(p_ref, p_fus, True)


@pytest.mark.gpu
def test_master_params_materialises_master_grads(monkeypatch):
    ref, fus = [], []
    _run(monkeypatch, False, "lamb", True, steps=2, probe=ref)
    _run(monkeypatch, True, "lamb", True, steps=2, probe=fus)
    assert all(g is not None for g in fus[0])
    for a, b in zip(ref[0], fus[0]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_fused_step_o5_bf16(monkeypatch):
    """O5: bf16 model, fp32 masters, static scale 1 -- the step reads the bf16 gradients directly."""
    s_ref, p_ref, m_ref, _ = _run(monkeypatch, False, "adam", False, opt_level="O5")
    s_fus, p_fus, m_fus, pend = _run(monkeypatch, True, "adam", False, opt_level="O5")
    assert all(pend)
    _close(m_ref, m_fus, False)
    _close(p_ref, p_fus, False)


def _cpu_setup():
    from beforeholiday_amd import amp
    from beforeholiday_amd.optimizers import FusedLAMB

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.BatchNorm1d(64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 8))
    opt = FusedLAMB(model.parameters(), lr=1e-2)
    model, opt = amp.initialize(model, opt, opt_level="O2", keep_batchnorm_fp32=True, verbosity=0,
                                loss_scale="dynamic")
    return amp, model, opt


def test_fused_plan_flow_cpu(monkeypatch):
    """The plan's bookkeeping (CPU, the optimizer hooks faked): a backward leaves the step pending with
    no master gradients, the step hands (models, 1/scale, scaled norm) to the optimizer, and
    ``amp.master_params`` materialises exactly the unfused master gradients."""
    from beforeholiday_amd.amp import _process_optimizer

    config.set(amp_device_scaler=False)
    x = torch.randn(16, 32).half()
    y = torch.randint(0, 8, (16,))

    config.set(amp_fused_master_step=False)
    amp, model, opt = _cpu_setup()
    with amp.scale_loss(F.cross_entropy(model(x).float(), y), opt) as s:
        s.backward()
    want = [p.grad.clone() for p in amp.master_params(opt)]

    config.set(amp_fused_master_step=True)
    amp, model, opt = _cpu_setup()
    calls = []
    opt._amp_fused_ok = lambda: True
    opt._amp_fused_step = lambda models, inv, norm: calls.append((models, inv, norm))
    with amp.scale_loss(F.cross_entropy(model(x).float(), y), opt) as s:
        s.backward()
    plan = opt._amp_stash.plan
    assert plan.fused_pending()
    assert all(m.grad is None for m in opt._amp_stash.all_fp32_from_fp16_params)
    lows = [p.grad.float() for p in opt._amp_stash.all_fp16_params]
    scale = 2.0 ** 16
    opt.step()
    (models, inv, norm), = calls
    assert set(models) == {id(m) for m in opt._amp_stash.all_fp32_from_fp16_params}
    assert float(inv) == 1.0 / scale
    torch.testing.assert_close(norm.reshape(()), torch.cat([g.reshape(-1) for g in lows]).norm(), rtol=1e-4, atol=0)
    assert not plan.fused_pending()

    amp, model, opt = _cpu_setup()
    opt._amp_fused_ok = lambda: True
    with amp.scale_loss(F.cross_entropy(model(x).float(), y), opt) as s:
        s.backward()
    got = [p.grad.clone() for p in amp.master_params(opt)]  # materialised
    assert not opt._amp_stash.plan.fused_pending()
    for a, b in zip(want, got):
        assert torch.equal(a, b)


def test_default_populates_param_group_grads_cpu():
    """The fused step is opt-in: by default the fp32 masters in ``optimizer.param_groups``
    carry their gradients when ``scale_loss`` exits, so clipping through the param groups clips what the
    step applies. With the fused step on, ``amp.master_params`` (the documented clipping route)
    materialises the same gradients, and clipping through it changes the step's input."""
    config.set(amp_device_scaler=False)
    assert config.Config().amp_fused_master_step is False
    x = torch.randn(16, 32).half()
    y = torch.randint(0, 8, (16,))

    amp, model, opt = _cpu_setup()
    opt._amp_fused_ok = lambda: True  # even where the fused kernels exist, the default path is unfused
    with amp.scale_loss(F.cross_entropy(model(x).float(), y), opt) as s:
        s.backward()
    group_params = [p for g in opt.param_groups for p in g["params"]]
    assert all(p.grad is not None for p in group_params)
    assert not opt._amp_stash.plan.fused_pending()
    before = torch.cat([p.grad.reshape(-1) for p in group_params]).norm()
    torch.nn.utils.clip_grad_norm_(group_params, max_norm=float(before) / 4)
    after = torch.cat([p.grad.reshape(-1) for p in group_params]).norm()
    torch.testing.assert_close(after, before / 4, rtol=1e-3, atol=0)

    config.set(amp_fused_master_step=True)
    amp, model, opt = _cpu_setup()
    opt._amp_fused_ok = lambda: True
    with amp.scale_loss(F.cross_entropy(model(x).float(), y), opt) as s:
        s.backward()
    assert opt._amp_stash.plan.fused_pending()
    masters = list(amp.master_params(opt))  # materialises: the step falls back to the unfused kernels
    assert all(p.grad is not None for p in masters)
    assert not opt._amp_stash.plan.fused_pending()
    torch.testing.assert_close(torch.cat([p.grad.reshape(-1) for p in masters]).norm(), before, rtol=1e-3, atol=0)
