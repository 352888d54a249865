"""Probe: one amp O2 step with the fused mixed-precision LAMB step vs the unfused sequence; prints the
differences of masters, moments and model params."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["BH_AMP_DEVICE_SCALER"] = sys.argv[2] if len(sys.argv) > 2 else "1"


def run(fused, opt_name):
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp import _process_optimizer
    from beforeholiday_amd.optimizers import FusedAdam, FusedLAMB

    _process_optimizer.fused_master_step = fused
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.BatchNorm1d(64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 8)).cuda()
    opt = (FusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=0.5) if opt_name == "lamb"
           else FusedAdam(model.parameters(), lr=1e-2, weight_decay=0.01))
    model, opt = amp.initialize(model, opt, opt_level="O2", keep_batchnorm_fp32=True, verbosity=0,
                                loss_scale="dynamic")
    x = torch.randn(16, 32, device="cuda", dtype=torch.half)
    y = torch.randint(0, 8, (16,), device="cuda")
    out = []
    for i in range(2):
        loss = F.cross_entropy(model(x).float(), y)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        g16 = [p.grad.clone() if p.grad is not None else None for p in model.parameters()]
        opt.step()
        opt.zero_grad()
        st = [(opt.state[p].get("exp_avg"), opt.state[p].get("exp_avg_sq")) for p in amp.master_params(opt)]
        if any(x[0] is None for x in st):
            print("fused", fused, "step", i, "missing state:",
                  [(tuple(p.shape), p.dtype, p.grad is None, list(opt.state[p].keys())) for p in amp.master_params(opt)],
                  "scale", __import__("beforeholiday_amd.amp._amp_state", fromlist=["x"])._amp_state.loss_scalers[0].loss_scale(), flush=True)
            st = [(torch.zeros_like(p) if a is None else a, torch.zeros_like(p) if b is None else b)
                  for p, (a, b) in zip(amp.master_params(opt), st)]
        out.append(dict(masters=[p.detach().clone() for p in amp.master_params(opt)],
                        model=[p.detach().clone() for p in model.parameters()],
                        m=[s[0].clone() for s in st], v=[s[1].clone() for s in st], g16=g16,
                        step=getattr(opt, "_device_steps", None)))
    return out


for name in [sys.argv[1] if len(sys.argv) > 1 else "lamb"]:
    a, b = run(False, name), run(True, name)
    for i in range(2):
        for k in ("m", "v", "masters", "model", "g16"):
            d = [(u.float() - w.float()).abs().max().item() if u is not None else None for u, w in zip(a[i][k], b[i][k])]
            print(name, "step", i, k, ["%.3g" % x if x is not None else None for x in d])
        print("steps", a[i]["step"], b[i]["step"])
