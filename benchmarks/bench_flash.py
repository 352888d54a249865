"""Flash attention (kernels/attn.hip) forward / backward throughput at head dim 64 vs PyTorch SDPA.

    python benchmarks/bench_flash.py [--dtype bf16] [--shapes gpt,bert,long]

One JSON line per (shape, dropout): milliseconds and TFLOP/s of our forward and backward (backward
= delta + dK/dV + dQ kernels) and of ``torch.nn.functional.scaled_dot_product_attention`` on the
same [B, H, S, 64] problem (no dropout for SDPA: its dropout path is a different kernel). FLOPs:
4*B*H*Sq*Sk*64 forward, 2.5x that backward, halved for causal masks.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "gpt": (8, 16, 1024, True),    # GPT-2-medium bench: batch 8, 16 heads, seq 1024, causal
    "bert": (16, 16, 512, False),  # BERT-large shape
    "long": (4, 16, 2048, True),
    "long4k": (2, 16, 4096, True),
}


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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--shapes", default="gpt,bert,long")
    ap.add_argument("--dropout", default="0,0.1")
    ap.add_argument("--no-sdpa", action="store_true")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from beforeholiday_amd._native import require_native, submodule

    require_native("bench_flash")
    fa = submodule("fused_attention")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    for name in args.shapes.split(","):
        B, H, S, causal = SHAPES[name]
        BH = B * H
        mode = 5 if causal else 0
        flops = 4.0 * BH * S * S * 64 * (0.5 if causal else 1.0)
        qkv = torch.randn(S, BH, 3, 64, device="cuda", dtype=dt)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        dout = torch.randn(S, BH, 64, device="cuda", dtype=dt)
        dqkv = torch.empty_like(qkv)
        for p in (float(x) for x in args.dropout.split(",")):
            fwd = lambda: fa.flash_forward(q, k, v, mode, None, H, 0.125, p, True, 7, float("-inf"))  # noqa: E731
            o, lse = fwd()

            def bwd():
                fa.flash_backward(dout, q, k, v, o, lse, mode, None, H, 0.125, p, True, 7, float("-inf"),
                                  dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])

            tf, tb = timeit(fwd), timeit(bwd)
            r = {"shape": name, "B": B, "H": H, "S": S, "causal": causal, "dropout": p, "dtype": args.dtype,
                 "tag": args.tag, "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                 "fwd_tflops": round(flops / tf / 1e9, 1), "bwd_tflops": round(2.5 * flops / tb / 1e9, 1)}
            if p == 0.0 and not args.no_sdpa:
                F = torch.nn.functional
                qs, ks, vs = (t.permute(1, 0, 2).reshape(B, H, S, 64).detach().requires_grad_(True) for t in (q, k, v))
                do4 = dout.permute(1, 0, 2).reshape(B, H, S, 64)
                sf = lambda: F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal, scale=0.125)  # noqa: E731
                os_ = sf()

                def sb():
                    torch.autograd.grad(os_, (qs, ks, vs), do4, retain_graph=True)

                try:
                    tsf, tsb = timeit(sf), timeit(sb)
                    r.update({"sdpa_fwd_ms": round(tsf, 4), "sdpa_bwd_ms": round(tsb, 4),
                              "sdpa_fwd_tflops": round(flops / tsf / 1e9, 1),
                              "sdpa_bwd_tflops": round(2.5 * flops / tsb / 1e9, 1)})
                except RuntimeError as e:  # no SDPA kernel for this shape
                    r["sdpa_error"] = str(e)[:120]
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
