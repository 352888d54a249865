"""Batch-norm kernel bandwidth at the ResNet-50 (batch 256, channels_last, fp16) BN shapes.

Times stats (+finalize), fused forward (BN+ReLU), backward reduce (+finalize) and dgrad for each
distinct layer shape, reports effective HBM GB/s per op and the ResNet-50-weighted total per step,
and the same for torch's native batch norm (MIOpen) as a reference. Launch-geometry knobs are read
from BH_BN_* env vars, so a sweep runs this script once per setting.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import syncbn  # noqa: E402

# (H, C, count in ResNet-50 forward) -- N = 256
SHAPES = [(112, 64, 1), (56, 64, 6), (56, 256, 4), (56, 128, 1), (28, 128, 7), (28, 512, 5), (28, 256, 1),
          (14, 256, 11), (14, 1024, 7), (14, 512, 1), (7, 512, 5), (7, 2048, 4)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    N = int(os.environ.get("BN_BATCH", 256))
    dt = torch.float16
    res = {"knobs": {k: v for k, v in os.environ.items() if k.startswith("BH_BN_")}, "layers": []}
    tot = {"stats": 0.0, "fwd": 0.0, "reduce": 0.0, "dgrad": 0.0, "torch_fwd": 0.0, "torch_bwd": 0.0}
    for H, C, cnt in SHAPES:
        x = torch.randn(N, C, H, H, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        w = torch.rand(C, device="cuda") + 0.5
        b = torch.randn(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbytes = x.numel() * 2
        st = syncbn.stats_single(x, w, b, rm, rv, 0.1, 1e-5)
        mean, invstd, scale, shift, count = st
        t_stats = timeit(lambda: syncbn.stats_single(x, w, b, rm, rv, 0.1, 1e-5))
        t_fwd = timeit(lambda: syncbn.forward(x, None, scale, shift, True))
        t_red = timeit(lambda: syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, True))
        sums = syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, True)[0]
        t_dg = timeit(lambda: syncbn.backward_dgrad(dy, x, None, mean, invstd, w, sums, count, scale, shift, True, False))
        # torch reference: F.batch_norm (+relu) forward, autograd backward
        xr = x.detach().requires_grad_(True)
        wr, br = w.detach().requires_grad_(True), b.detach().requires_grad_(True)

        def tfwd():
            return torch.relu(F.batch_norm(xr, rm, rv, wr, br, True, 0.1, 1e-5))

        t_tf = timeit(tfwd)
        y = tfwd()
        t_tb = timeit(lambda: torch.autograd.grad(y, (xr, wr, br), dy, retain_graph=True))
        row = dict(H=H, C=C, count=cnt, MB=round(nbytes / 1e6, 1),
                   stats_us=round(t_stats * 1e3, 1), stats_GBs=round(nbytes / t_stats / 1e6),
                   fwd_us=round(t_fwd * 1e3, 1), fwd_GBs=round(2 * nbytes / t_fwd / 1e6),
                   reduce_us=round(t_red * 1e3, 1), reduce_GBs=round(2 * nbytes / t_red / 1e6),
                   dgrad_us=round(t_dg * 1e3, 1), dgrad_GBs=round(3 * nbytes / t_dg / 1e6),
                   torch_fwd_us=round(t_tf * 1e3, 1), torch_bwd_us=round(t_tb * 1e3, 1))
        res["layers"].append(row)
        for k, t in (("stats", t_stats), ("fwd", t_fwd), ("reduce", t_red), ("dgrad", t_dg), ("torch_fwd", t_tf),
                     ("torch_bwd", t_tb)):
            tot[k] += cnt * t
        print(json.dumps(row), flush=True)
    res["resnet50_weighted_ms"] = {k: round(v, 3) for k, v in tot.items()}
    res["ours_total_ms"] = round(tot["stats"] + tot["fwd"] + tot["reduce"] + tot["dgrad"], 3)
    res["torch_total_ms"] = round(tot["torch_fwd"] + tot["torch_bwd"], 3)
    print(json.dumps({k: res[k] for k in ("knobs", "resnet50_weighted_ms", "ours_total_ms", "torch_total_ms")}),
          flush=True)


if __name__ == "__main__":
    main()
