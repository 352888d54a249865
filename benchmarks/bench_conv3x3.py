"""ResNet-50 middle 3x3 convs (batch 256, channels_last, fp16): the direct MFMA kernel
(ops/conv.py) vs MIOpen (F.conv2d / convolution_backward, immediate mode as the bench runs it) for
the forward and the data gradient. One JSON line per shape with ms and TFLOP/s.

    python benchmarks/bench_conv3x3.py [--batch 256] [--dtype fp16]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(64, 56, 3), (128, 28, 3), (256, 14, 5), (512, 7, 2)]  # C = K, H = W, count in ResNet-50


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
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--ab", action="store_true",
                    help="pipeline variants (Config.conv3x3_nb x conv3x3_sw) of OUR kernel, interleaved twice on one box")
    args = ap.parse_args()
    from beforeholiday_amd.ops import conv as bhconv

    if args.ab:
        from beforeholiday_amd import config

        dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
        data = []
        for C, H, cnt in SHAPES:
            x = torch.randn(args.batch, C, H, H, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
            w = (torch.randn(C, C, 3, 3, device="cuda", dtype=dt) * 0.02).contiguous(memory_format=torch.channels_last)
            data.append((x, w, torch.randn_like(x), cnt))
        for rep in range(2):
            for nb, sw in ((3, True), (2, True), (2, False), (3, False)):
                config.set(conv3x3_nb=nb, conv3x3_sw=sw)
                f = sum(timeit(lambda: bhconv.conv3x3(x, w)) * cnt for x, w, dy, cnt in data)
                d = sum(timeit(lambda: bhconv.conv3x3_dgrad(dy, w)) * cnt for x, w, dy, cnt in data)
                print(json.dumps({"rep": rep, "nb": nb, "sw": sw, "fwd_ms": round(f, 3), "dgrad_ms": round(d, 3)}),
                      flush=True)
        return

    torch.backends.cudnn.benchmark = False
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    tot = {"ours_fwd": 0.0, "miopen_fwd": 0.0, "ours_dgrad": 0.0, "miopen_dgrad": 0.0, "miopen_wgrad": 0.0}
    for C, H, cnt in SHAPES:
        N = args.batch
        x = torch.randn(N, C, H, H, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device="cuda", dtype=dt) * 0.02).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        flops = 2.0 * N * H * H * C * C * 9
        r = {"C": C, "H": H, "count": cnt}
        r["ours_fwd"] = timeit(lambda: bhconv.conv3x3(x, w))
        r["miopen_fwd"] = timeit(lambda: F.conv2d(x, w, padding=1))
        r["ours_dgrad"] = timeit(lambda: bhconv.conv3x3_dgrad(dy, w))
        r["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        if hasattr(bhconv, "conv3x3_wgrad"):
            r["ours_wgrad"] = timeit(lambda: bhconv.conv3x3_wgrad(dy, x))
            tot.setdefault("ours_wgrad", 0.0)
        for k in tot:
            tot[k] += r[k] * cnt
            r[k + "_tflops"] = round(flops / r[k] / 1e9, 1)
            r[k] = round(r[k], 4)
        print(json.dumps(r), flush=True)
    print(json.dumps({"resnet50_weighted_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
