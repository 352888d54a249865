"""amp O1 / O4 (fp32 model, 16-bit casts around torch functions) on the fused ResNet: every
convolution runs the own MFMA kernels in amp's 16-bit dtype -- the reference's O1 routes conv2d to the
16-bit tensor cores through its cast lists (apex/amp/lists/functional_overrides.py:18-32); here the
kernels are not torch functions, so the model casts for them (models/resnet.py ``_kx`` / ``_kw``,
amp ``kernel_cast``). Checked against the same fp32 model without amp: loss and gradients, with no
``F.conv2d`` (MIOpen) call in the forward, and fp32 gradients on the fp32 parameters."""
import copy

import pytest
import torch


def _net():
    from beforeholiday_amd.models import resnet50_fused

    torch.manual_seed(0)
    net = resnet50_fused(layers=(1, 1, 1, 1), num_classes=10).cuda().to(memory_format=torch.channels_last)
    return net


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("level,tol", [("O4", 5e-2), ("O1", 2e-2)])
def test_o1_o4_resnet_runs_mfma_kernels(level, tol):
    from beforeholiday_amd import amp
    from beforeholiday_amd.optimizers import FusedAdam

    net = _net()
    ref = copy.deepcopy(net)
    torch.manual_seed(5)
    x = torch.randn(16, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    loss_ref = torch.nn.functional.cross_entropy(ref(x), y)
    loss_ref.backward()

    opt = FusedAdam(net.parameters(), lr=1e-3)
    kw = {"loss_scale": 128.0} if level == "O1" else {}  # (a fixed fp16 scale: no overflow-skipped step)
    net, opt = amp.initialize(net, opt, opt_level=level, verbosity=0, **kw)
    calls = []
    conv2d = torch.nn.functional.conv2d

    def counting(*a, **k):
        calls.append(a[0].shape)
        return conv2d(*a, **k)

    torch.nn.functional.conv2d = counting
    try:
        out = net(x)
        loss = torch.nn.functional.cross_entropy(out, y)
        assert not calls, f"{len(calls)} convolutions fell back to F.conv2d under {level}: {calls[:4]}"
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        assert abs(float(loss) - float(loss_ref)) < tol * abs(float(loss_ref)), (float(loss), float(loss_ref))
        for (n, p), q in zip(net.named_parameters(), ref.parameters()):
            assert p.dtype == torch.float32 and p.grad is not None and p.grad.dtype == torch.float32, n
        # the stem and the classifier: well-conditioned gradients (deep BN chains amplify rounding)
        assert _rel(net.fc.weight.grad, ref.fc.weight.grad) < 10 * tol
        w0 = net.fc.weight.detach().clone()
        opt.step()
        assert not torch.equal(w0, net.fc.weight.detach())
    finally:
        torch.nn.functional.conv2d = conv2d
        amp.deactivate()
