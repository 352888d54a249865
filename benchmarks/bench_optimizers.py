"""Optimizer step time: fused multi-tensor kernels vs torch.optim (second half of the headline
metric, "FusedLAMB step ms vs torch.optim"; reference harness: tests/L0/run_optimizers/test_lamb.py
math, apex/optimizers/fused_lamb.py).

Parameter sets are the real ResNet-50 (25.6M params, 161 tensors) and BERT-large (335M params,
~390 tensors) shapes, fp32 params + fp32 grads. torch has no LAMB, so the baseline LAMB is a
sync-free ``torch._foreach_*`` implementation of the same math (global grad-norm clip, Adam moments,
per-tensor trust ratio) -- the fastest torch.optim-style formulation. Adam / SGD compare against
``torch.optim.Adam(foreach=True)`` / ``(fused=True)`` and ``torch.optim.SGD(foreach=True)``.

Prints one JSON line per (model, optimizer, implementation) and writes them to --out.
"""
import argparse
import json
import time
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.optimizers import FusedAdam, FusedLAMB, FusedSGD  # noqa: E402


def bert_large_shapes(vocab=30522, hidden=1024, layers=24, ffn=4096, seq=512):
    s = [(vocab, hidden), (seq, hidden), (2, hidden), (hidden,), (hidden,)]
    for _ in range(layers):
        s += [(3 * hidden, hidden), (3 * hidden,), (hidden, hidden), (hidden,), (hidden,), (hidden,),
              (ffn, hidden), (ffn,), (hidden, ffn), (hidden,), (hidden,), (hidden,)]
    s += [(hidden, hidden), (hidden,), (hidden, hidden), (hidden,), (hidden,), (hidden,), (vocab,)]
    return s


def resnet50_shapes():
    from beforeholiday_amd.models import resnet50
    return [tuple(p.shape) for p in resnet50().parameters()]


class ForeachLAMB(torch.optim.Optimizer):
    """LAMB with torch._foreach ops, no host syncs (same math as FusedLAMB, adam_w_mode)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = max_grad_norm

    @torch.no_grad()
    def step(self):
        ps = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        gs = [p.grad for p in ps]
        gn = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(gs)))
        clip = torch.clamp(gn / self.max_grad_norm, min=1.0)
        for group in self.param_groups:
            b1, b2 = group["betas"]
            ps = [p for p in group["params"] if p.grad is not None]
            for p in ps:
                if not self.state[p]:
                    self.state[p].update(step=0, m=torch.zeros_like(p), v=torch.zeros_like(p))
            st = [self.state[p] for p in ps]
            step = st[0]["step"] + 1
            for s in st:
                s["step"] = step
            ms, vs = [s["m"] for s in st], [s["v"] for s in st]
            g = torch._foreach_div([p.grad for p in ps], clip)
            torch._foreach_lerp_(ms, g, 1 - b1)
            torch._foreach_mul_(vs, b2)
            torch._foreach_addcmul_(vs, g, g, 1 - b2)
            den = torch._foreach_sqrt(torch._foreach_div(vs, 1 - b2 ** step))
            torch._foreach_add_(den, group["eps"])
            u = torch._foreach_div(torch._foreach_div(ms, 1 - b1 ** step), den)
            torch._foreach_add_(u, ps, alpha=group["weight_decay"])
            pn = torch.stack(torch._foreach_norm(ps))
            un = torch.stack(torch._foreach_norm(u))
            ratio = torch.where((pn > 0) & (un > 0), pn / un, torch.ones_like(pn)) * group["lr"]
            torch._foreach_mul_(u, list(ratio.unbind(0)))
            torch._foreach_sub_(ps, u)


def make(shapes, device):
    g = torch.Generator(device=device).manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=device, generator=g) * 0.02) for s in shapes]
    for p in ps:
        p.grad = torch.randn(p.shape, device=device, generator=g) * 1e-3
    return ps


def time_opt(opt, iters, warmup):
    for _ in range(warmup):
        opt.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    t0 = time.perf_counter()
    for _ in range(iters):
        opt.step()
    host = (time.perf_counter() - t0) / iters * 1e3  # issue time: ~= ms_per_step when host-bound
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters, host


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--models", default="resnet50,bert_large")
    ap.add_argument("--out", default="gpurun_out/optimizers.jsonl")
    args = ap.parse_args()
    dev = torch.device("cuda")
    shapes = {"resnet50": resnet50_shapes, "bert_large": bert_large_shapes}
    cases = {
        "lamb": [("FusedLAMB", lambda ps: FusedLAMB(ps, lr=1e-3, weight_decay=0.01)),
                 ("torch_foreach_lamb", lambda ps: ForeachLAMB(ps, lr=1e-3, weight_decay=0.01))],
        "adam": [("FusedAdam", lambda ps: FusedAdam(ps, lr=1e-3, weight_decay=0.01)),
                 ("torch.optim.Adam(foreach)", lambda ps: torch.optim.Adam(ps, lr=1e-3, weight_decay=0.01,
                                                                          foreach=True)),
                 ("torch.optim.Adam(fused)", lambda ps: torch.optim.Adam(ps, lr=1e-3, weight_decay=0.01,
                                                                        fused=True))],
        "sgd": [("FusedSGD", lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-4)),
                ("torch.optim.SGD(foreach)", lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-4,
                                                                        foreach=True))],
    }
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    rows = []
    for model in args.models.split(","):
        sh = shapes[model]()
        nparam = sum(torch.Size(s).numel() for s in sh)
        for opt_name, impls in cases.items():
            base = None
            for impl, ctor in impls:
                ps = make(sh, dev)
                try:
                    ms, host_ms = time_opt(ctor(ps), args.iters, args.warmup)
                except Exception as e:  # noqa: BLE001 - report unsupported baselines, keep going
                    print(json.dumps({"model": model, "optimizer": opt_name, "impl": impl, "error": str(e)[:200]}))
                    continue
                # bytes touched per step by an ideal fused kernel: read p,g,m,v + write p,m,v (fp32)
                ideal_gb = nparam * 4 * (7 if opt_name != "sgd" else 5) / 1e9
                row = {"model": model, "params_M": round(nparam / 1e6, 2), "tensors": len(sh), "optimizer": opt_name,
                       "impl": impl, "ms_per_step": round(ms, 4), "host_issue_ms": round(host_ms, 4), "effective_GBps": round(ideal_gb / ms * 1e3, 1)}
                if base is None:
                    base = ms
                else:
                    row["fused_speedup"] = round(ms / base, 2)
                rows.append(row)
                print(json.dumps(row), flush=True)
                del ps
                torch.cuda.empty_cache()
    with open(args.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
