"""Host-side cost of one ResNet-50 bench step: wall time of issuing the step's work from Python (no
synchronisation inside the step except amp's one loss-scale read) vs the GPU time of the step.

    python benchmarks/probe_host_overhead.py [--batch 256]

If the host issue time approaches the GPU time, the GPU starves between small kernels and HIP-graph
capture / fewer launches pay; if it is well below, the step is GPU-bound.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    from beforeholiday_amd import amp
    from beforeholiday_amd.models import resnet50_fused
    from beforeholiday_amd.optimizers import FusedLAMB
    from beforeholiday_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    model = resnet50_fused().cuda().to(memory_format=torch.channels_last)
    opt = FusedLAMB(model.parameters(), lr=4e-3 * args.batch / 4096, weight_decay=0.01)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=0, keep_batchnorm_fp32=True)
    model = DistributedDataParallel(model)
    x = torch.randn(args.batch, 3, 224, 224, device="cuda", dtype=torch.float16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device="cuda")

    phases = {}

    def step():
        t0 = time.perf_counter()
        out = model(x)
        loss = F.cross_entropy(out, y)
        t1 = time.perf_counter()
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
            t2 = time.perf_counter()
        t3 = time.perf_counter()  # includes the loss-scale read (waits for the GPU)
        opt.step()
        opt.zero_grad()
        t4 = time.perf_counter()
        for k, v in (("fwd_issue", t1 - t0), ("bwd_issue", t2 - t1), ("unscale_sync", t3 - t2), ("opt_issue", t4 - t3)):
            phases.setdefault(k, []).append(v * 1e3)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    phases.clear()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(args.steps):
        step()
    b.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps * 1e3
    print(json.dumps({"wall_ms_per_step": round(wall, 3), "gpu_ms_per_step": round(a.elapsed_time(b) / args.steps, 3),
                      **{k: round(sum(v) / len(v), 3) for k, v in phases.items()}}), flush=True)


if __name__ == "__main__":
    main()
