"""Dense-layer weight gradients dW = dY^T X at the BERT-large / GPT-2-medium shapes (8192 tokens): the
transposed-operand ping-pong kernel (``gemm.weight_grad_tn``) vs hipBLASLt (``dy.t() @ x``) vs the 1x1
weight-gradient kernel path (ops/fused_dense.weight_grad's previous route), interleaved rounds in one
process, median us and TFLOP/s. One JSON line per shape.

    python benchmarks/bench_wgrad_tn.py [--tokens 8192] [--dtype fp16]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]  # (out, in): QKV, proj, fc1, fc2
# ResNet-50 1x1 weight gradients of stages 3-4 (tokens = pixels at batch 256): (tokens, out, in)
RESNET = [(50176, 256, 1024), (50176, 1024, 256), (12544, 512, 2048), (12544, 2048, 512), (50176, 512, 1024)]


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
    ap.add_argument("--resnet", action="store_true", help="the ResNet-50 1x1 shapes, against the 1x1 wgrad kernel")
    args = ap.parse_args()
    from beforeholiday_amd._native import submodule

    gm = submodule("gemm")
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    torch.manual_seed(0)
    cc = submodule("conv_cuda")
    shapes = RESNET if args.resnet else [(args.tokens, N, K) for N, K in SHAPES]
    for T, N, K in shapes:
        dy = torch.randn(T, N, device="cuda").to(dt)
        x = torch.randn(T, K, device="cuda").to(dt)
        flops = 2.0 * T * N * K
        cands = {"tn": lambda: gm.weight_grad_tn(dy, x, 0), "hipblaslt": lambda: dy.t() @ x}
        x4, dy4 = x.view(1, 1, T, K).permute(0, 3, 1, 2), dy.view(1, 1, T, N).permute(0, 3, 1, 2)
        cands["wgrad1x1"] = lambda: cc.conv_wgrad(x4, dy4, 1, 1)
        for s in (1, 2, 4, 8):
            cands[f"tn_s{s}"] = (lambda s=s: gm.weight_grad_tn(dy, x, s))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, f in cands.items():
                times[k].append(timeit(f))
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        ref = (dy.float().t() @ x.float())
        err = float((gm.weight_grad_tn(dy, x, 0).float() - ref).norm() / ref.norm())
        print(json.dumps({"T": T, "N": N, "K": K, "us": {k: round(v, 1) for k, v in med.items()},
                          "tflops_tn": round(flops / med["tn"] / 1e6, 1),
                          "tflops_hipblaslt": round(flops / med["hipblaslt"] / 1e6, 1),
                          "speedup_vs_hipblaslt": round(med["hipblaslt"] / med["tn"], 3),
                          "speedup_vs_wgrad1x1": round(med["wgrad1x1"] / med["tn"], 3), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
