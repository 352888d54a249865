"""1x1 weight gradients of ResNet-50 (batch 256, channels_last fp16): the MFMA wgrad kernel
(kernels/conv_wgrad.hip) vs the same product as a library GEMM, dW = dY^T . X on the [pixels, channels]
views (hipBLASLt / rocBLAS through torch.mm, with the per-shape solution table of utils/gemm_tuning.py;
``--gemm-table tune`` searches the solutions of these shapes first). One JSON line per shape.

    python benchmarks/bench_wgrad_gemm.py [--gemm-table auto|tune|off] [--batch 256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, H, count per step) of the stride-1 1x1 convolutions
SHAPES = [(64, 64, 56, 1), (256, 64, 56, 2), (64, 256, 56, 4), (512, 128, 28, 3), (128, 512, 28, 4),
          (1024, 256, 14, 5), (256, 1024, 14, 6), (2048, 512, 7, 2), (512, 2048, 7, 3)]


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
    from beforeholiday_amd.utils import gemm_tuning

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    gemm_tuning.add_argument(ap)
    args = ap.parse_args()
    gemm_tuning.setup(args.gemm_table)
    from beforeholiday_amd.ops import conv as bhconv

    tot = {"mfma": 0.0, "gemm": 0.0, "best": 0.0}
    for cin, cout, H, count in SHAPES:
        n = args.batch
        x = torch.randn(n, cin, H, H, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, H, H, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
        x2d = x.permute(0, 2, 3, 1).reshape(-1, cin)
        d2d = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        t_mfma = timeit(lambda: bhconv.conv_wgrad(x, dy, 1))
        t_gemm = timeit(lambda: torch.mm(d2d.t(), x2d))
        ref = (d2d.float().t() @ x2d.float())
        err_g = float((torch.mm(d2d.t(), x2d).float() - ref).abs().max() / ref.abs().max())
        err_m = float((bhconv.conv_wgrad(x, dy, 1).reshape(cout, cin).float() - ref).abs().max() / ref.abs().max())
        fl = 2.0 * n * H * H * cin * cout
        tot["mfma"] += count * t_mfma
        tot["gemm"] += count * t_gemm
        tot["best"] += count * min(t_mfma, t_gemm)
        print(json.dumps({"cin": cin, "cout": cout, "H": H, "count": count, "mfma_ms": round(t_mfma, 4),
                          "gemm_ms": round(t_gemm, 4), "mfma_tflops": round(fl / t_mfma / 1e9, 1),
                          "gemm_tflops": round(fl / t_gemm / 1e9, 1), "rel_err_mfma": round(err_m, 5),
                          "rel_err_gemm": round(err_g, 5)}), flush=True)
    print(json.dumps({"per_step_ms": {k: round(v, 3) for k, v in tot.items()},
                      "gemm_table": gemm_tuning.status()}), flush=True)
    gemm_tuning.finish(args.gemm_table)


if __name__ == "__main__":
    main()
