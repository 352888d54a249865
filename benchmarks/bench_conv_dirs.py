"""Per-layer A/B of the ResNet-50 (batch 256, fp16, channels_last) convolutions: MIOpen (immediate
mode, as the bench runs it) vs hipBLASLt GEMMs on the [N*H*W, C] view for the 1x1 / stride-1 convs,
separately for forward, data gradient and weight gradient. Prints one JSON line per layer and a
summary of the per-step totals (every layer counted with its multiplicity in ResNet-50).

    python benchmarks/bench_conv_dirs.py [--batch 256]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, k, stride, H_in, count) of ResNet-50 v1.5 at 224x224
LAYERS = [
    (64, 64, 1, 1, 56, 1), (256, 64, 1, 1, 56, 2), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 3),
    (64, 256, 1, 1, 56, 1),  # downsample of stage 1 (stride 1)
    (256, 128, 1, 1, 56, 1), (512, 128, 1, 1, 28, 3), (128, 128, 3, 2, 56, 1), (128, 128, 3, 1, 28, 3),
    (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 256, 1, 1, 28, 1), (1024, 256, 1, 1, 14, 5), (256, 256, 3, 2, 28, 1), (256, 256, 3, 1, 14, 5),
    (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 512, 1, 1, 14, 1), (2048, 512, 1, 1, 7, 2), (512, 512, 3, 2, 14, 1), (512, 512, 3, 1, 7, 2),
    (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
]


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = False
    N = args.batch
    tot = {"miopen_fwd": 0.0, "miopen_dgrad": 0.0, "miopen_wgrad": 0.0, "gemm_fwd": 0.0, "gemm_dgrad": 0.0,
           "gemm_wgrad": 0.0, "gemm_dgrad_accum": 0.0}
    for cin, cout, k, s, H, cnt in LAYERS:
        x = torch.randn(N, cin, H, H, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.float16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=s, padding=k // 2)
        gy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        r = {"cin": cin, "cout": cout, "k": k, "stride": s, "H": H, "count": cnt}
        r["miopen_fwd"] = timeit(lambda: F.conv2d(x, w, stride=s, padding=k // 2))
        r["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [False, True, False]))
        if k == 1 and s == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            w2 = w.view(cout, cin)
            acc = torch.empty_like(x2)
            r["gemm_fwd"] = timeit(lambda: torch.mm(x2, w2.t()))
            r["gemm_dgrad"] = timeit(lambda: torch.mm(gy2, w2))
            r["gemm_dgrad_accum"] = timeit(lambda: torch.addmm(acc, gy2, w2, out=acc))
            r["gemm_wgrad"] = timeit(lambda: torch.mm(gy2.t(), x2))
        for key in tot:
            tot[key] += r.get(key, r.get(key.replace("gemm", "miopen").replace("_accum", ""), 0.0)) * cnt
        print(json.dumps({k2: (round(v, 4) if isinstance(v, float) else v) for k2, v in r.items()}), flush=True)
    print(json.dumps({"per_step_ms": {k2: round(v, 3) for k2, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
