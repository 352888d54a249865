"""Per-parameter gradient error of the BN-folded and the unfolded fused fp16 ResNet against fp32."""
import sys
import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from beforeholiday_amd.models import resnet as R  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def build(fold, layers):
    torch.manual_seed(0)
    ref = R.ResNet(R.Bottleneck, list(layers), num_classes=10).cuda()
    R._FOLD_BN = fold
    m = R.resnet50_fused(layers=layers, num_classes=10).cuda()
    m.load_state_dict(ref.state_dict())
    m = m.to(memory_format=torch.channels_last).half()
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.float()
    return ref, m


layers = (2, 2, 2, 2)
x = torch.randn(8, 3, 64, 64, device="cuda")
res = {}
for fold in (True, False):
    ref, m = build(fold, layers)
    R._FOLD_BN = fold
    xr = x.clone().requires_grad_()
    xf = x.half().contiguous(memory_format=torch.channels_last).requires_grad_()
    orr, of = ref(xr), m(xf)
    orr.square().sum().backward()
    of.float().square().sum().backward()
    res[fold] = {"out": rel(of, orr), "xgrad": rel(xf.grad, xr.grad)}
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        res[fold][n] = rel(p.grad, q.grad)
    for (n, b), q in zip(m.named_buffers(), ref.buffers()):
        if "running" in n:
            res[fold][n] = rel(b, q)
for k in res[True]:
    print(f"{k:45s} fold {res[True][k]:.4f}   nofold {res[False].get(k, float('nan')):.4f}")
