"""amp: opt-level properties, O1/O4 cast tables, promotion, weight-cast cache, dynamic loss scaling
with injected overflows, multiple losses, gradient accumulation, add_param_group, checkpointing.

Mirrors the reference suites tests/L0/run_amp/{test_basic_casts.py:25-258, test_promotion.py:12-112,
test_cache.py:62-158, test_multiple_models_optimizers_losses.py:45-762, test_checkpointing.py:27-268,
test_add_param_group.py:53}. Every case runs on CPU (the multi-tensor ops fall back to their
PyTorch reference there) and as a gpu-marked case on the MI355X, where the unscale / overflow
flag path is the native multi_tensor_scale / axpby kernel.
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from beforeholiday_amd import amp
from beforeholiday_amd.amp._amp_state import _amp_state
from beforeholiday_amd.optimizers import FusedAdam, FusedSGD

from conftest import devices


@pytest.fixture(autouse=True)
def _reset_amp():
    yield
    amp.deactivate()
    _amp_state.opt_properties = None
    _amp_state.loss_scalers = []
    _amp_state.hard_override = False


def _low(device):
    return torch.float16


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(8, 16)
        self.bn = nn.BatchNorm1d(16)
        self.fc2 = nn.Linear(16, 4)

    def forward(self, x):
        return self.fc2(F.relu(self.bn(self.fc1(x))))


# --------------------------------------------------------------------------------------------- options
def test_opt_level_properties():
    expected = {
        "O0": (torch.float32, False, None, False, 1.0),
        "O1": (None, True, None, None, "dynamic"),
        "O2": (torch.float16, False, True, True, "dynamic"),
        "O3": (torch.float16, False, False, False, 1.0),
        "O4": (None, True, None, None, 1.0),
        "O5": (torch.bfloat16, False, True, True, 1.0),
    }
    for lvl, (cast, patch, keep_bn, master, scale) in expected.items():
        p = amp.opt_levels[lvl](amp.Properties())
        assert p.enabled and p.opt_level == lvl
        assert p.cast_model_type == cast
        assert p.patch_torch_functions == patch
        assert p.keep_batchnorm_fp32 == keep_bn
        assert p.master_weights == master
        assert p.loss_scale == scale


def test_invalid_options_raise():
    m = nn.Linear(4, 4)
    with pytest.raises(RuntimeError, match="Unexpected optimization level"):
        amp.initialize(m, opt_level="02")
    with pytest.raises(RuntimeError, match="keep_batchnorm_fp32"):
        amp.initialize(nn.Linear(4, 4), opt_level="O1", keep_batchnorm_fp32=True, verbosity=0)


def test_string_overrides_parsed():
    m = MLP()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    amp.initialize(m, opt, opt_level="O2", keep_batchnorm_fp32="False", loss_scale="128.0", verbosity=0)
    assert _amp_state.opt_properties.keep_batchnorm_fp32 is False
    assert _amp_state.opt_properties.loss_scale == 128.0
    assert _amp_state.loss_scalers[0].loss_scale() == 128.0 and not _amp_state.loss_scalers[0].dynamic


@pytest.mark.parametrize("device", devices())
def test_o2_casts_model_and_keeps_bn_fp32(device):
    m = MLP().to(device)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    m, opt = amp.initialize(m, opt, opt_level="O2", verbosity=0)
    assert m.fc1.weight.dtype == torch.float16 and m.fc2.bias.dtype == torch.float16
    assert m.bn.weight.dtype == torch.float32 and m.bn.running_mean.dtype == torch.float32
    out = m(torch.randn(6, 8, device=device))  # fp32 input is cast by the patched forward
    assert out.dtype == torch.float32  # outputs are cast back to fp32
    # the saved model state is fp32 (O2StateDictHook)
    assert all(v.dtype == torch.float32 for v in m.state_dict().values() if v.is_floating_point())
    # master weights are created lazily at the first scaled backward (reference behaviour)
    with amp.scale_loss(out.mean(), opt) as scaled:
        scaled.backward()
    opt.step()
    masters = list(amp.master_params(opt))
    assert len(masters) == 6 and all(p.dtype == torch.float32 for p in masters)


# ------------------------------------------------------------------------------------- O1/O4 casting
def _run_layer(fn, dtype, device, *shape):
    x = torch.randn(*shape, device=device, dtype=dtype)
    return fn(x)


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("patch_type", [torch.float16, torch.bfloat16])
def test_o1_basic_casts(device, patch_type):
    amp.init(patch_type=patch_type, enable_caching=True)
    lin = nn.Linear(8, 8).to(device)
    conv = nn.Conv2d(3, 4, 3).to(device)
    for in_dt in (torch.float32, patch_type):
        # whitelist -> low precision regardless of input dtype
        assert _run_layer(lin, in_dt, device, 4, 8).dtype == patch_type
        assert _run_layer(conv, in_dt, device, 1, 3, 8, 8).dtype == patch_type
        assert torch.mm(torch.randn(4, 4, device=device, dtype=in_dt),
                        torch.randn(4, 4, device=device)).dtype == patch_type
        # blacklist -> fp32
        assert _run_layer(lambda t: F.softmax(t, dim=-1), in_dt, device, 4, 8).dtype == torch.float32
        assert _run_layer(lambda t: F.mse_loss(t, t.detach()), in_dt, device, 4, 8).dtype == torch.float32
        assert _run_layer(lambda t: F.layer_norm(t, (8,)), in_dt, device, 4, 8).dtype == torch.float32
        assert _run_layer(lambda t: torch.exp(t), in_dt, device, 4, 8).dtype == torch.float32
        # pass-through ops keep their input type
        assert _run_layer(F.relu, in_dt, device, 4, 8).dtype == in_dt
    # banned function raises on low precision input
    with pytest.raises(NotImplementedError):
        F.binary_cross_entropy(torch.rand(4, device=device, dtype=patch_type),
                               torch.rand(4, device=device, dtype=patch_type))


@pytest.mark.parametrize("device", devices())
def test_o1_promotion_and_inplace(device):
    amp.init(patch_type=torch.float16)
    h = torch.randn(4, device=device, dtype=torch.float16)
    f = torch.randn(4, device=device)
    assert torch.cat([h, f]).dtype == torch.float32
    assert torch.stack([h, h]).dtype == torch.float16
    assert (h + f).dtype == torch.float32
    assert torch.add(h, f).dtype == torch.float32
    assert torch.mul(h, h).dtype == torch.float16
    # in-place op on an fp32 tensor with a half argument casts the argument
    f2 = f.clone()
    f2.add_(h)
    assert f2.dtype == torch.float32
    # an fp32-only in-place op on a half tensor is an error (it would silently lose precision)
    with pytest.raises(NotImplementedError):
        h.clone().exp_()


@pytest.mark.parametrize("device", devices())
def test_o1_weight_cast_cache(device):
    handle = amp.init(patch_type=torch.float16, enable_caching=True)
    lin = nn.Linear(8, 8).to(device)
    x = torch.randn(4, 8, device=device)
    y1 = lin(x)
    y2 = lin(x)
    assert len(handle.cache) >= 1  # the fp16 weight copy is cached and reused
    (y1.float().sum() + y2.float().sum()).backward()
    assert lin.weight.grad is not None and lin.weight.grad.dtype == torch.float32
    # the cached cast is a differentiable view of the param: grads of both uses accumulate
    ref = nn.Linear(8, 8).to(device)
    ref.load_state_dict(lin.state_dict())
    amp.deactivate()
    (ref(x).sum() * 2).backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad, rtol=2e-2, atol=2e-2)
    handle._clear_cache()
    assert len(handle.cache) == 0


@pytest.mark.parametrize("device", devices())
def test_user_registries_and_decorators(device):
    @amp.float_function
    def f32_op(a):
        return a * 2

    @amp.half_function
    def f16_op(a):
        return a * 2

    @amp.promote_function
    def promo(a, b):
        return a + b

    h = torch.randn(3, device=device, dtype=torch.float16)
    f = torch.randn(3, device=device)
    assert f32_op(h).dtype == torch.float16  # no handle yet -> untouched
    amp.init(patch_type=torch.float16)
    assert f32_op(h).dtype == torch.float32
    assert f16_op(f).dtype == torch.float16
    assert promo(h, f).dtype == torch.float32
    with amp.disable_casts():
        assert f16_op(f).dtype == torch.float32


# --------------------------------------------------------------------------------------- loss scaling
def _train(model, opt, xs, ys, opt_level=None, inject=(), loss_scale=None, device="cpu"):
    """Runs len(xs) steps; injects inf into fc1.weight.grad at the iterations in ``inject``."""
    for it, (x, y) in enumerate(zip(xs, ys)):
        out = model(x)
        loss = F.mse_loss(out.float(), y)
        if opt_level is None:
            loss.backward()
            if it in inject:
                opt.zero_grad()  # reference: an overflowing step is skipped entirely
                continue
            opt.step()
            opt.zero_grad()
        else:
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
                if it in inject:
                    model.fc1.weight.grad[0, 0] = float("inf")
            opt.step()
            opt.zero_grad()


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("opt_level", ["O0", "O1", "O2", "O3", "O5"])
@pytest.mark.parametrize("optim", ["sgd", "fused_sgd", "fused_adam"])
def test_dynamic_scaling_skips_overflow_steps(device, opt_level, optim):
    torch.manual_seed(0)
    ref = MLP().to(device)
    ref.bn = nn.Identity()
    model = copy.deepcopy(ref)
    xs = [torch.randn(16, 8, device=device) for _ in range(6)]
    ys = [torch.randn(16, 4, device=device) for _ in range(6)]

    def mk(params):
        if optim == "sgd":
            return torch.optim.SGD(params, lr=0.05, momentum=0.9)
        if optim == "fused_sgd":
            return FusedSGD(params, lr=0.05, momentum=0.9)
        return FusedAdam(params, lr=1e-2)

    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9) if optim != "fused_adam" else \
        torch.optim.Adam(ref.parameters(), lr=1e-2)
    opt = mk(model.parameters())
    loss_scale = "dynamic" if opt_level in ("O3", "O5", "O0") else None
    model, opt = amp.initialize(model, opt, opt_level=opt_level, loss_scale=loss_scale, verbosity=0)
    inject = (2, 4)
    _train(ref, ref_opt, xs, ys, inject=inject)
    _train(model, opt, xs, ys, opt_level=opt_level, inject=inject)
    scaler = _amp_state.loss_scalers[0]
    assert scaler.loss_scale() == 2.0 ** 16 / 4  # halved once per injected overflow
    assert scaler._unskipped == 1
    tol = {"O0": 1e-5, "O1": 3e-2, "O2": 3e-2, "O3": 5e-2, "O5": 8e-2}[opt_level]
    for p_ref, p in zip(ref.parameters(), model.parameters()):
        torch.testing.assert_close(p.float(), p_ref, rtol=tol, atol=tol)
    if opt_level in ("O2", "O5"):
        # model params track the fp32 master params
        for p, m in zip(model.parameters(), amp.master_params(opt)):
            torch.testing.assert_close(p.float(), m, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("device", devices())
def test_scale_growth_window(device):
    model = nn.Linear(4, 4).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=0)
    scaler = _amp_state.loss_scalers[0]
    scaler._scale_seq_len = 3
    for _ in range(3):
        with amp.scale_loss(model(torch.randn(2, 4, device=device)).float().mean(), opt) as s:
            s.backward()
        opt.step()
        opt.zero_grad()
    assert scaler.loss_scale() == 2.0 ** 17 and scaler._unskipped == 0


@pytest.mark.parametrize("device", devices())
def test_min_max_loss_scale(device):
    model = nn.Linear(4, 4).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    model, opt = amp.initialize(model, opt, opt_level="O2", min_loss_scale=2.0 ** 15, max_loss_scale=2.0 ** 15,
                                verbosity=0)
    scaler = _amp_state.loss_scalers[0]
    assert scaler.loss_scale() == 2.0 ** 15
    for _ in range(2):
        with amp.scale_loss(model(torch.randn(2, 4, device=device)).float().mean(), opt) as s:
            s.backward()
            model.weight.grad.fill_(float("nan"))
        opt.step()
        opt.zero_grad()
    assert scaler.loss_scale() == 2.0 ** 15


@pytest.mark.parametrize("device", devices())
def test_multiple_losses_have_independent_scalers(device):
    torch.manual_seed(0)
    m0, m1 = nn.Linear(4, 4).to(device), nn.Linear(4, 4).to(device)
    o0 = torch.optim.SGD(m0.parameters(), lr=0.1)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1)
    [m0, m1], [o0, o1] = amp.initialize([m0, m1], [o0, o1], opt_level="O2", num_losses=2, verbosity=0)
    assert len(_amp_state.loss_scalers) == 2
    w0, w1 = m0.weight.detach().clone(), m1.weight.detach().clone()
    x = torch.randn(3, 4, device=device)
    with amp.scale_loss(m0(x).float().mean(), o0, loss_id=0) as s:
        s.backward()
    with amp.scale_loss(m1(x).float().mean(), o1, loss_id=1) as s:
        s.backward()
        m1.weight.grad[0, 0] = float("inf")
    o0.step()
    o1.step()
    assert _amp_state.loss_scalers[0].loss_scale() == 2.0 ** 16
    assert _amp_state.loss_scalers[1].loss_scale() == 2.0 ** 15
    assert not torch.equal(m0.weight, w0)  # stepped
    assert torch.equal(m1.weight, w1)  # skipped


@pytest.mark.parametrize("device", devices())
def test_delay_unscale_gradient_accumulation(device):
    torch.manual_seed(0)
    ref = nn.Linear(8, 4).to(device)
    model = copy.deepcopy(ref)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=0)
    xs = [torch.randn(5, 8, device=device) for _ in range(3)]
    for x in xs:
        ref(x).mean().backward()
    ref_opt.step()
    for i, x in enumerate(xs):
        with amp.scale_loss(model(x).float().mean(), opt, delay_unscale=i < len(xs) - 1) as s:
            s.backward()
    opt.step()
    torch.testing.assert_close(model.weight.float(), ref.weight, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(model.bias.float(), ref.bias, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("device", devices())
def test_add_param_group_after_initialize(device):
    torch.manual_seed(0)
    a, b = nn.Linear(4, 4).to(device), nn.Linear(4, 4).to(device)
    ref_a, ref_b = copy.deepcopy(a), copy.deepcopy(b)
    opt = torch.optim.SGD(a.parameters(), lr=0.1)
    ref_opt = torch.optim.SGD(ref_a.parameters(), lr=0.1)
    [a, b], opt = amp.initialize([a, b], opt, opt_level="O2", verbosity=0)
    x = torch.randn(3, 4, device=device)
    for it in range(3):
        if it == 1:
            opt.add_param_group({"params": b.parameters(), "lr": 0.05})
            ref_opt.add_param_group({"params": ref_b.parameters(), "lr": 0.05})
        with amp.scale_loss((b(a(x))).float().mean(), opt) as s:
            s.backward()
        opt.step()
        opt.zero_grad()
        ref_b(ref_a(x)).mean().backward()
        ref_opt.step()
        ref_opt.zero_grad()
    assert len(opt.param_groups) == 2
    for p, r in zip(list(a.parameters()) + list(b.parameters()),
                    list(ref_a.parameters()) + list(ref_b.parameters())):
        torch.testing.assert_close(p.float(), r, rtol=2e-2, atol=2e-2)


# -------------------------------------------------------------------------------------- checkpointing
@pytest.mark.parametrize("device", devices())
def test_amp_state_dict_roundtrip(device):
    model = MLP().to(device)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level="O2", num_losses=2, verbosity=0)
    x = torch.randn(4, 8, device=device)
    with amp.scale_loss(model(x).mean(), opt, loss_id=1) as s:
        s.backward()
        model.fc2.weight.grad.fill_(float("inf"))
    opt.step()
    opt.zero_grad()
    sd = amp.state_dict()
    assert list(sd.keys()) == ["loss_scaler0", "loss_scaler1"]
    assert sd["loss_scaler0"] == {"loss_scale": 65536.0, "unskipped": 0}
    assert sd["loss_scaler1"] == {"loss_scale": 32768.0, "unskipped": 0}
    model_sd = model.state_dict()
    opt_sd = opt.state_dict()
    assert all(v.dtype == torch.float32 for v in model_sd.values() if v.is_floating_point())

    # restore into a fresh O2 setup: initialize first, then load model / optimizer / amp state
    amp.deactivate()
    model2 = MLP().to(device)
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.1, momentum=0.9)
    model2, opt2 = amp.initialize(model2, opt2, opt_level="O2", num_losses=2, verbosity=0)
    model2.load_state_dict(model_sd)
    opt2.load_state_dict(opt_sd)
    amp.load_state_dict(sd)
    assert amp.state_dict() == sd
    for p, q in zip(model.parameters(), model2.parameters()):
        assert torch.equal(p, q)
    with pytest.raises(RuntimeError, match="Unexpected key"):
        amp.load_state_dict({"loss_scaler0": sd["loss_scaler0"], "bogus": {}})


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("save_level,load_level", [("O0", "O2"), ("O2", "O0"), ("O2", "O1"), ("O1", "O2"),
                                                   ("O2", "O5"), ("O5", "O2")])
def test_checkpoint_across_opt_levels(device, save_level, load_level):
    torch.manual_seed(0)
    x = torch.randn(8, 8, device=device)
    model = MLP().to(device)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level=save_level, verbosity=0)
    for _ in range(2):
        with amp.scale_loss(model(x).float().mean(), opt) as s:
            s.backward()
        opt.step()
        opt.zero_grad()
    ckpt = {"model": model.state_dict(), "optimizer": opt.state_dict(), "amp": amp.state_dict()}
    assert all(v.dtype == torch.float32 for v in ckpt["model"].values() if v.is_floating_point())
    amp.deactivate()
    _amp_state.loss_scalers = []
    model2 = MLP().to(device)
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.05, momentum=0.9)
    model2, opt2 = amp.initialize(model2, opt2, opt_level=load_level, verbosity=0)
    model2.load_state_dict(ckpt["model"])
    opt2.load_state_dict(ckpt["optimizer"])
    amp.load_state_dict(ckpt["amp"])
    for (k, v), (k2, v2) in zip(ckpt["model"].items(), model2.state_dict().items()):
        assert k == k2
        torch.testing.assert_close(v2.float(), v.float(), rtol=1e-3, atol=1e-3)
    # both continue training without error and stay finite
    with amp.scale_loss(model2(x).float().mean(), opt2) as s:
        s.backward()
    opt2.step()
    assert all(torch.isfinite(p).all() for p in model2.parameters())


def test_optim_wrapper_second_loss_touches_subset_of_params():
    """Legacy multi-loss OptimWrapper: loss 1 reaches only one of two parameters. zero_grad() before
    its backward leaves the other parameter's .grad None; the wrapper must restore loss 0's gradient
    there instead of failing on None.add_()."""
    from beforeholiday_amd.amp.opt import OptimWrapper

    class _Handle:
        def is_active(self):
            return True

        def remove_cache(self, p):
            pass

    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(4))
    b = torch.nn.Parameter(torch.randn(4))
    opt = OptimWrapper(torch.optim.SGD([a, b], lr=0.1), _Handle(), num_loss=2)
    with opt.scale_loss((a * b).sum()) as s:
        s.backward()
    ga, gb = a.grad.clone(), b.grad.clone()
    with opt.scale_loss((a * 3).sum()) as s:
        s.backward()
    torch.testing.assert_close(a.grad, ga + 3)
    torch.testing.assert_close(b.grad, gb)
    a0, b0 = a.detach().clone(), b.detach().clone()
    opt.step()
    torch.testing.assert_close(a.detach(), a0 - 0.1 * (ga + 3))
    torch.testing.assert_close(b.detach(), b0 - 0.1 * gb)
