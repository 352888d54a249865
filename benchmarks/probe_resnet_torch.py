"""Probe: plain-PyTorch ResNet-50 training-step throughput on one GPU for layout/dtype/batch
variants (guides which configuration the framework's bench should build on)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.models import resnet50  # noqa: E402


def run(dtype, cl, bs, steps, warmup, bench):
    torch.backends.cudnn.benchmark = bench
    m = resnet50().cuda().to(dtype)
    # keep BN fp32 like amp O2 keep_batchnorm_fp32
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            mod.float()
    if cl:
        m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(bs, 3, 224, 224, device="cuda", dtype=dtype)
    if cl:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (bs,), device="cuda")

    def step():
        out = m(x)
        loss = F.cross_entropy(out.float(), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    return bs / dt, dt * 1e3


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variants", type=int, default=5, help="run only the first N variants (1: fp16 channels_last)")
    args = ap.parse_args()
    variants = [
        (torch.float16, True, 256, False), (torch.bfloat16, True, 256, False),
        (torch.float16, False, 256, False), (torch.bfloat16, False, 256, False),
        (torch.bfloat16, True, 128, False),
    ]
    for dt, cl, bs, bench in variants[:args.variants]:
        t0 = time.time()
        try:
            ips, ms = run(dt, cl, bs, args.steps, args.warmup, bench)
            r = dict(dtype=str(dt), channels_last=cl, batch=bs, cudnn_benchmark=bench, img_s=round(ips, 1),
                     ms=round(ms, 2), wall_s=round(time.time() - t0, 1))
        except Exception as e:  # keep probing other variants
            r = dict(dtype=str(dt), channels_last=cl, batch=bs, error=repr(e)[:300])
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()
