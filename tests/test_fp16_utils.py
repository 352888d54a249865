"""Legacy fp16_utils (FP16_Optimizer, conversions, master-param helpers) and LARC.

Reference behaviour: apex/fp16_utils/fp16_optimizer.py:13-554 (state_dict :209-228, load :230-271),
apex/fp16_utils/fp16util.py:22-187, apex/parallel/LARC.py; the reference's own LARC test is
tests/L0/run_amp/test_larc.py:31 (it only smoke-tests amp + LARC; here the update is checked
against the closed-form LARC rule).
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from beforeholiday_amd import fp16_utils
from beforeholiday_amd.fp16_utils import (FP16_Optimizer, FP16Model, convert_network, master_params_to_model_params,
                                          model_grads_to_master_grads, network_to_half, prep_param_lists)
from beforeholiday_amd.parallel import LARC

from conftest import devices


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(8, 8)
        self.bn = nn.BatchNorm1d(8)
        self.out = nn.Linear(8, 2)

    def forward(self, x):
        return self.out(F.relu(self.bn(self.fc(x))))


def test_network_to_half_keeps_affine_bn_fp32():
    net = network_to_half(Net())
    assert net[1].fc.weight.dtype == torch.float16
    assert net[1].bn.weight.dtype == torch.float32 and net[1].bn.running_var.dtype == torch.float32
    y = net(torch.randn(4, 8))
    assert y.dtype == torch.float16
    net2 = convert_network(Net(), torch.bfloat16)
    assert net2.fc.weight.dtype == torch.bfloat16 and net2.bn.weight.dtype == torch.float32
    m = FP16Model(Net())
    assert m(torch.randn(4, 8)).dtype == torch.float16


@pytest.mark.parametrize("flat_master", [False, True])
def test_param_list_helpers(flat_master):
    torch.manual_seed(0)
    net = Net().half()
    model_params, master_params = prep_param_lists(net, flat_master=flat_master)
    assert all(p.dtype == torch.float32 for p in master_params)
    if flat_master:
        assert len(master_params) == 1 and master_params[0].numel() == sum(p.numel() for p in model_params)
    net(torch.randn(4, 8).half()).float().sum().backward()
    model_grads_to_master_grads(model_params, master_params, flat_master=flat_master)
    flat_g = torch.cat([p.grad.float().reshape(-1) for p in model_params])
    got = torch.cat([p.grad.reshape(-1) for p in master_params])
    torch.testing.assert_close(got, flat_g)
    for p in master_params:
        p.data.add_(1.0)
    master_params_to_model_params(model_params, master_params, flat_master=flat_master)
    got = torch.cat([p.float().reshape(-1) for p in model_params])
    want = torch.cat([p.data.reshape(-1) for p in master_params])
    torch.testing.assert_close(got, want.half().float())


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("dynamic", [False, True])
def test_fp16_optimizer_tracks_fp32_reference(device, dynamic):
    torch.manual_seed(0)
    ref = Net().to(device)
    model = network_to_half(copy.deepcopy(ref))
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9),
                         static_loss_scale=128.0, dynamic_loss_scale=dynamic,
                         dynamic_loss_args={"init_scale": 2.0 ** 8}, verbose=False)
    for it in range(5):
        x = torch.randn(16, 8, device=device)
        y = torch.randn(16, 2, device=device)
        F.mse_loss(ref(x), y).backward()
        opt.zero_grad()
        loss = F.mse_loss(model(x).float(), y)
        opt.backward(loss, update_master_grads=False)
        if dynamic and it == 2:
            # overflow: the fp16 grads carry an inf, the step must be skipped and the scale halved
            model[1].fc.weight.grad[0, 0] = float("inf")
        opt.update_master_grads()
        if dynamic and it == 2:
            assert opt.overflow
            opt.step()
            ref_opt.zero_grad()
            continue
        opt.step()
        ref_opt.step()
        ref_opt.zero_grad()
    if dynamic:
        assert opt.loss_scale == 2.0 ** 7
    for p, r in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.float(), r, rtol=3e-2, atol=3e-2)
    # masters are fp32 copies of the fp16 weights
    for m, p in zip(opt.fp32_from_fp16_groups[0], opt.fp16_groups[0]):
        torch.testing.assert_close(m.half(), p)


@pytest.mark.parametrize("device", devices())
def test_fp16_optimizer_state_dict_roundtrip(device):
    torch.manual_seed(0)
    model = network_to_half(Net().to(device))
    opt = FP16_Optimizer(torch.optim.Adam(model.parameters(), lr=1e-2), dynamic_loss_scale=True, verbose=False)
    x = torch.randn(8, 8, device=device)
    for _ in range(2):
        opt.zero_grad()
        opt.backward(model(x).float().pow(2).mean())
        opt.step()
    sd = opt.state_dict()
    assert set(sd) == {"loss_scaler", "dynamic_loss_scale", "overflow", "first_closure_call_this_step",
                       "optimizer_state_dict", "fp32_from_fp16"}
    model2 = network_to_half(Net().to(device))
    opt2 = FP16_Optimizer(torch.optim.Adam(model2.parameters(), lr=1e-2), dynamic_loss_scale=True, verbose=False)
    opt2.load_state_dict(sd)
    for a, b in zip(opt.fp32_from_fp16_groups[0], opt2.fp32_from_fp16_groups[0]):
        assert torch.equal(a, b)
    assert opt2.loss_scale == opt.loss_scale


@pytest.mark.parametrize("device", devices())
def test_fp16_optimizer_clip_master_grads(device):
    model = network_to_half(Net().to(device))
    opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=0.1), static_loss_scale=64.0, verbose=False)
    opt.backward(model(torch.randn(8, 8, device=device)).float().sum() * 100)
    norm = opt.clip_master_grads(1.0)
    assert float(norm) > 1.0
    total = torch.sqrt(sum(p.grad.pow(2).sum() for g in opt.optimizer.param_groups for p in g["params"]))
    assert float(total) <= 1.0 + 1e-3


def test_loss_scaler_classes():
    s = fp16_utils.DynamicLossScaler(init_scale=2 ** 8, scale_window=2)
    p = nn.Parameter(torch.ones(3))
    p.grad = torch.tensor([1.0, float("nan"), 2.0])
    assert s.has_overflow([p])
    s.update_scale(True)
    assert s.loss_scale == 2 ** 7
    s.update_scale(False)
    s.update_scale(False)
    assert s.loss_scale == 2 ** 8
    st = fp16_utils.LossScaler(4.0)
    assert st.loss_scale == 4.0 and not st.has_overflow([p])


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("clip", [True, False])
def test_larc_matches_closed_form(device, clip):
    torch.manual_seed(0)
    params = [nn.Parameter(torch.randn(16, 8, device=device)), nn.Parameter(torch.randn(8, device=device))]
    ref = [p.detach().clone() for p in params]
    grads = [torch.randn_like(p) * 10 for p in params]
    for p, g in zip(params, grads):
        p.grad = g.clone()
    lr, wd, tc, eps = 0.1, 1e-4, 0.02, 1e-8
    opt = LARC(torch.optim.SGD(params, lr=lr, weight_decay=wd), trust_coefficient=tc, clip=clip, eps=eps)
    opt.step()
    assert opt.param_groups[0]["weight_decay"] == wd  # restored after the step
    for r, g, p in zip(ref, grads, params):
        pn, gn = r.norm(), g.norm()
        adaptive = tc * pn / (gn + pn * wd + eps)
        if clip:
            adaptive = torch.clamp(adaptive / lr, max=1.0)
        expect = r - lr * (g + wd * r) * adaptive
        torch.testing.assert_close(p.detach(), expect, rtol=1e-5, atol=1e-6)
