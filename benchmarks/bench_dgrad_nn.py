"""Dense-layer data gradients dX = dY @ W at the BERT-large / GPT-2-medium shapes (8192 tokens): the NN layout of
the ping-pong MFMA kernel (``gemm.mm_nn``, kernels/gemm_tn.hip) vs hipBLASLt (``dy @ w``), interleaved rounds in
one process, median us and TFLOP/s. One JSON line per shape.

    python benchmarks/bench_dgrad_nn.py [--tokens 8192] [--dtype fp16] [--resnet]

--resnet: the ResNet-50 (bs 256) 1x1 data gradients that still run on hipBLASLt (stage-3 / stage-4 rows).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]  # (K = layer out, N = layer in)
RESNET = [(50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)]  # (M, K, N)


def timeit(fn, iters=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--resnet", action="store_true")
    args = ap.parse_args()
    from beforeholiday_amd._native import submodule

    gm = submodule("gemm")
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    torch.manual_seed(0)
    shapes = RESNET if args.resnet else [(args.tokens, K, N) for K, N in SHAPES]
    for M, K, N in shapes:
        dy = torch.randn(M, K, device="cuda").to(dt)
        w = (torch.randn(K, N, device="cuda") / K ** 0.5).to(dt)
        flops = 2.0 * M * N * K
        cands = {"nn": lambda: gm.mm_nn(dy, w, 0), "hipblaslt": lambda: dy @ w}
        for s in (1, 2, 4):
            cands[f"nn_s{s}"] = (lambda s=s: gm.mm_nn(dy, w, s))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, f in cands.items():
                times[k].append(timeit(f))
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        ref = dy.float() @ w.float()
        err = float((gm.mm_nn(dy, w, 0).float() - ref).norm() / ref.norm())
        print(json.dumps({"M": M, "K": K, "N": N, "us": {k: round(v, 1) for k, v in med.items()},
                          "tflops_nn": round(flops / med["nn"] / 1e6, 1),
                          "tflops_hipblaslt": round(flops / med["hipblaslt"] / 1e6, 1),
                          "speedup_vs_hipblaslt": round(med["hipblaslt"] / med["nn"], 3), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
