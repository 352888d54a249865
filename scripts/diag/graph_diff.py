"""Per-step parameter divergence between eager steps and HIP-graph replays of the same step."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
os.environ["BH_AMP_DEVICE_SCALER"] = "1"


def run(graph, steps=5):
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp._amp_state import _amp_state
    from beforeholiday_amd.models import resnet50_fused
    from beforeholiday_amd.optimizers import FusedLAMB
    from beforeholiday_amd.parallel import DistributedDataParallel
    from beforeholiday_amd.utils import GraphedStep

    torch.manual_seed(0)
    model = resnet50_fused(layers=(1, 1, 1, 1), num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = FusedLAMB(model.parameters(), lr=1e-3, weight_decay=0.01)
    model, opt = amp.initialize(model, opt, opt_level="O2", keep_batchnorm_fp32=True, verbosity=0)
    model = DistributedDataParallel(model)
    x = torch.randn(32, 3, 64, 64, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    names = [n for n, _ in model.named_parameters()]

    def step():
        loss = F.cross_entropy(model(x), y)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss.detach()

    hist = []
    sc = _amp_state.loss_scalers[0]

    def snap(loss):
        torch.cuda.synchronize()
        hist.append((float(loss), float(sc._scale_dev) if sc.device_mode else sc._loss_scale,
                     [p.detach().float().clone() for p in model.parameters()]))

    if graph:
        g = GraphedStep(step, warmup=2).capture()
        snap(torch.zeros(()))
        for _ in range(steps - 2):
            snap(g())
    else:
        for i in range(steps):
            l = step()
            if i >= 1:
                snap(l)
    amp.deactivate()
    return names, hist


names, he = run(False)
_, hg = run(True)
for k, ((le, se, pe), (lg, sg, pg)) in enumerate(zip(he, hg)):
    d = sorted(((((a - b).abs().max() / (b.abs().max() + 1e-6)).item(), n) for n, a, b in zip(names, pg, pe)),
               reverse=True)[:4]
    print(f"snap {k}: eager loss {le:.5f} scale {se}; graph loss {lg:.5f} scale {sg}; worst {d}", flush=True)
