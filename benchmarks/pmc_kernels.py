"""Drive the hand-written MFMA kernels for rocprofv3 counter collection (one short process per
counter pass; see scripts/pmc_pass.sh). Each kernel is launched `--iters` times on fixed shapes:
  gemm      : gemm.hip big tile, bf16 4096^3 with the GELU+aux epilogue (gemm.linear_act)
  gemm_bwd  : gemm.hip small tile, bf16 8192x1024x4096 with dGELU + bias-grad epilogue
  attn_fwd / attn_bwd : attn.hip, 120 sequences x 16 heads x 64 tokens, head 64, dropout 0.1
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", choices=["all", "gemm_plain"], default="all",
                    help="gemm_plain: only C = A.B^T at 4096^3 bf16 on the ping-pong kernel (uniform [-1, 1) data)")
    args = ap.parse_args()
    from beforeholiday_amd._native import require_native, submodule

    require_native("pmc_kernels")
    gm, fa = submodule("gemm"), submodule("fused_attention")
    gm.set_force_mfma(True)
    dt = torch.bfloat16
    if args.only == "gemm_plain":
        gm.set_tile_mode(4)
        a = torch.rand(4096, 4096, device="cuda", dtype=dt) * 2 - 1
        bm = torch.rand(4096, 4096, device="cuda", dtype=dt) * 2 - 1
        for _ in range(args.iters):
            gm.linear_act(a, bm, None, 0, False)
        torch.cuda.synchronize()
        return
    x = torch.randn(4096, 4096, device="cuda", dtype=dt)
    w = torch.randn(4096, 4096, device="cuda", dtype=dt) / 64
    b = torch.randn(4096, device="cuda", dtype=dt)
    dy = torch.randn(8192, 4096, device="cuda", dtype=dt)
    w2t = torch.randn(1024, 4096, device="cuda", dtype=dt) / 64
    pre = torch.randn(8192, 1024, device="cuda", dtype=dt)
    qkv = torch.randn(64, 120 * 16, 3, 64, device="cuda", dtype=dt)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    dout = torch.randn(64, 120 * 16, 64, device="cuda", dtype=dt)
    dqkv = torch.empty_like(qkv)
    for _ in range(args.iters):
        gm.linear_act(x, w, b, 3, True)
        gm.linear_dact(dy, w2t, pre, 3, True)
        fa.forward(q, k, v, 0, None, 16, 0.125, 0.1, True, 7)
        fa.backward(dout, q, k, v, 0, None, 16, 0.125, 0.1, True, 7, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
    torch.cuda.synchronize()
    print("pmc_kernels done", flush=True)


if __name__ == "__main__":
    main()
