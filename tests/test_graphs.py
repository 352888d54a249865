"""Whole-step HIP graph capture (utils/graphs.py): a captured amp O2 + FusedLAMB + fused-SyncBN ResNet
training step, replayed, must produce the same parameters and losses as the same steps run eagerly."""
import pytest
import torch

from beforeholiday_amd import config
import torch.nn.functional as F


def _train(graph: bool, steps: int = 4):
    from beforeholiday_amd import amp
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
    losses = []

    def step():
        loss = F.cross_entropy(model(x), y)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss

    if graph:
        g = GraphedStep(lambda: step().detach(), warmup=2).capture()
        for _ in range(steps - 2):
            losses.append(g().clone())
    else:
        for i in range(steps):
            out = step().detach()
            if i >= 2:
                losses.append(out.clone())
    torch.cuda.synchronize()
    params = [p.detach().float().clone() for p in model.parameters()]
    amp.deactivate()
    return torch.stack(losses), params


@pytest.mark.gpu
def test_graphed_step_matches_eager(monkeypatch):
    config.set(amp_device_scaler=True)  # no host synchronisation inside the step
    l_eager, p_eager = _train(False)
    l_graph, p_graph = _train(True)
    torch.testing.assert_close(l_graph, l_eager, rtol=2e-3, atol=2e-3)
    # LAMB's first steps move every element by about lr whatever the gradient's size, so the sign of a
    # near-zero gradient (BN biases start at 0) decides the direction: compare in absolute terms, a
    # few steps of lr = 1e-3
    worst = max((a - b).abs().max().item() for a, b in zip(p_graph, p_eager))
    assert worst < 1e-2, worst
    # the step actually trained: the replays moved the parameters
    assert l_graph.isfinite().all()
