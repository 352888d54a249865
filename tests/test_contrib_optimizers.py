"""ZeRO DistributedFusedAdam / DistributedFusedLAMB (gloo CPU ranks) vs single-process optimizers on
the averaged gradient; legacy contrib FusedAdam / FusedSGD / FP16_Optimizer
(reference tests: apex/contrib/test/optimizers/test_dist_adam.py, test_distributed_fused_lamb.py)."""
import pytest
import torch

from tests._dist import run_distributed
from tests.conftest import devices


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 33), torch.nn.Tanh(), torch.nn.Linear(33, 5))


def _data(world, n=8):
    torch.manual_seed(100)
    return torch.randn(world, n, 12), torch.randn(world, n, 5)


def _dist_adam(rank, world, bucket_mb, overlap):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedAdam
    model = _model()
    ref = _model()
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.1, bucket_cap_mb=bucket_mb,
                               overlap_grad_sync=overlap)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1, eps=1e-8)
    X, Y = _data(world)
    for it in range(3):
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(X[rank]), Y[rank])
        loss.backward()
        opt.step()
        ref_opt.zero_grad()
        # reference: gradient of the mean over ranks' losses
        sum(torch.nn.functional.mse_loss(ref(X[r]), Y[r]) for r in range(world)).div(world).backward()
        ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
    # grad norm + clipping path and state dict round trip
    opt.zero_grad()
    torch.nn.functional.mse_loss(model(X[rank]), Y[rank]).backward()
    n = opt.clip_grad_norm(0.01)
    assert torch.isfinite(n).all()
    opt.step()
    sd = opt.state_dict()
    before = [p.detach().clone() for p in model.parameters()]
    opt2 = DistributedFusedAdam(_model(1).parameters(), lr=1e-2, bucket_cap_mb=bucket_mb)
    opt2.load_state_dict(sd)
    assert opt2.state["step"] == opt.state["step"]
    for b1, b2 in zip(opt._buckets, opt2._buckets):
        torch.testing.assert_close(b1.exp_avg, b2.exp_avg)
        torch.testing.assert_close(b1.master, b2.master)
    for p, b in zip(model.parameters(), before):
        torch.testing.assert_close(p.detach(), b)


@pytest.mark.parametrize("bucket_mb,overlap", [(100, True), (0.0005, True), (0.0005, False)])
def test_distributed_fused_adam(bucket_mb, overlap):
    run_distributed(_dist_adam, 2, bucket_mb, overlap)


def _dist_adam_no_sync(rank, world):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedAdam
    model, ref = _model(), _model()
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, bucket_cap_mb=0.001)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    X, Y = _data(world)
    opt.zero_grad()
    with opt.no_sync():
        torch.nn.functional.mse_loss(model(X[rank][:4]), Y[rank][:4]).backward()
    torch.nn.functional.mse_loss(model(X[rank][4:]), Y[rank][4:]).backward()
    opt.step()
    ref_opt.zero_grad()
    sum(torch.nn.functional.mse_loss(ref(X[r][:4]), Y[r][:4]) + torch.nn.functional.mse_loss(ref(X[r][4:]), Y[r][4:])
        for r in range(world)).div(world).backward()
    ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_distributed_fused_adam_grad_accumulation():
    run_distributed(_dist_adam_no_sync, 2)


def _dist_lamb(rank, world):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedLAMB
    from beforeholiday_amd.optimizers import FusedLAMB
    model, ref = _model(), _model()
    opt = DistributedFusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0,
                               bucket_cap_mb=0.0005)
    ref_opt = FusedLAMB(ref.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0, eps=1e-8)
    X, Y = _data(world)
    for it in range(3):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(X[rank]), Y[rank]).backward()
        opt.step()
        ref_opt.zero_grad()
        sum(torch.nn.functional.mse_loss(ref(X[r]), Y[r]) for r in range(world)).div(world).backward()
        ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_distributed_fused_lamb():
    run_distributed(_dist_lamb, 2)


@pytest.mark.parametrize("device", devices())
def test_legacy_contrib_fused_adam_and_fp16_optimizer(device):
    from beforeholiday_amd.contrib.optimizers import FP16_Optimizer, FusedAdam
    torch.manual_seed(0)
    dtype = torch.float16 if device != "cpu" else torch.float32
    model = torch.nn.Linear(16, 8).to(device, dtype)
    ref = torch.nn.Linear(16, 8).to(device)
    with torch.no_grad():
        ref.weight.copy_(model.weight.float())
        ref.bias.copy_(model.bias.float())
    opt = FP16_Optimizer(FusedAdam(model.parameters(), lr=1e-3), static_loss_scale=128.0, verbose=False)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    x = torch.randn(4, 16, device=device)
    for _ in range(3):
        opt.zero_grad()
        opt.backward(model(x.to(dtype)).float().pow(2).mean())
        opt.step()
        ref_opt.zero_grad()
        ref(x).pow(2).mean().backward()
        ref_opt.step()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(model.weight.float(), ref.weight, rtol=tol, atol=tol)


@pytest.mark.parametrize("device", devices())
def test_legacy_contrib_fused_sgd(device):
    from beforeholiday_amd.contrib.optimizers import FP16_Optimizer, FusedSGD
    torch.manual_seed(0)
    model = torch.nn.Linear(16, 8).to(device)
    ref = torch.nn.Linear(16, 8).to(device)
    ref.load_state_dict(model.state_dict())
    opt = FP16_Optimizer(FusedSGD(model.parameters(), lr=0.1, momentum=0.9), static_loss_scale=4.0, verbose=False)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(4, 16, device=device)
    for _ in range(3):
        opt.zero_grad()
        opt.backward(model(x).pow(2).mean())
        opt.step()
        ref_opt.zero_grad()
        ref(x).pow(2).mean().backward()
        ref_opt.step()
    torch.testing.assert_close(model.weight, ref.weight, rtol=1e-5, atol=1e-6)
