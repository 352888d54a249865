"""contrib conv_bias_relu vs torch conv2d + bias + ReLU (reference test: apex/contrib/test/conv_bias_relu)."""
import pytest
import torch
import torch.nn.functional as F

from tests.conftest import devices


@pytest.mark.parametrize("device", devices())
@pytest.mark.parametrize("variant", ["relu", "mask", "bias", "frozen"])
def test_conv_bias_relu(device, variant):
    from beforeholiday_amd.contrib import conv_bias_relu as cbr
    torch.manual_seed(0)
    dtype = torch.float16 if device != "cpu" else torch.float32
    x = torch.randn(2, 16, 10, 10, device=device).to(dtype).to(memory_format=torch.channels_last).requires_grad_()
    w = (torch.randn(32, 16, 3, 3, device=device) * 0.1).to(dtype).to(memory_format=torch.channels_last)
    w.requires_grad_()
    b = torch.randn(1, 32, 1, 1, device=device).to(dtype).requires_grad_()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    with torch.autocast("cuda", enabled=device != "cpu", dtype=torch.half):
        if variant == "relu":
            y = cbr.ConvBiasReLU(x, w, b, 1, 1)
        elif variant == "mask":
            mask = (torch.rand(2, 32, 10, 10, device=device) > 0.3).to(dtype)
            y = cbr.ConvBiasMaskReLU(x, w, b, mask, 1, 1)
        elif variant == "bias":
            y = cbr.ConvBias(x, w, b, 1, 1)
        else:
            scale = torch.rand(32, device=device) + 0.5
            y = cbr.ConvFrozenScaleBiasReLU(x, w, scale, b, 1, 1)
    c = F.conv2d(xr, wr, None, 1, 1)
    # the ReLU mask of the reference is taken from the kernel's own output: pre-activations within
    # fp16 rounding of 0 may legitimately flip sign between the fp16 kernel and the fp32 reference
    keep = (y.detach().float() > 0).float()
    if variant == "frozen":
        sc = scale.half().float() if dtype == torch.float16 else scale
        pre = c * sc.view(1, -1, 1, 1) + br
        torch.testing.assert_close(y.float(), torch.relu(pre.detach()), rtol=3e-2, atol=3e-2)
        ref = pre * keep
    else:
        ref = c + br
        if variant in ("relu", "mask"):
            torch.testing.assert_close(y.float(), (torch.relu(ref) * (mask.float() if variant == "mask" else 1)).detach(),
                                       rtol=3e-2, atol=3e-2)
            ref = ref * keep
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    g = torch.randn_like(ref)
    y.float().backward(g)
    ref.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol * 5)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=tol, atol=tol * 20)
    if variant != "frozen":
        torch.testing.assert_close(b.grad.float(), br.grad, rtol=tol, atol=tol * 20)
