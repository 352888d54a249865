"""Drive the flash attention kernels (kernels/attn.hip) for rocprofv3 counter passes (scripts/pmc_flash.sh):
BERT-large shape (16 seqs x 16 heads x 512 tokens) or the GPT-2-medium bench shape (8 x 16 x 1024,
causal), head 64, dropout --dropout."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="bert", choices=["bert", "gpt"])
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--fwd-only", action="store_true")
    args = ap.parse_args()
    from beforeholiday_amd._native import require_native, submodule

    require_native("pmc_flash")
    fa = submodule("fused_attention")
    dt = torch.bfloat16
    S, BH = (512, 256) if args.shape == "bert" else (1024, 128)
    mode = 0 if args.shape == "bert" else 5
    p = args.dropout
    qkv = torch.randn(S, BH, 3, 64, device="cuda", dtype=dt)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    dout = torch.randn(S, BH, 64, device="cuda", dtype=dt)
    dqkv = torch.empty_like(qkv)
    for _ in range(10):
        o, lse = fa.flash_forward(q, k, v, mode, None, 16, 0.125, p, True, 7, float("-inf"))
        if not args.fwd_only:
            fa.flash_backward(dout, q, k, v, o, lse, mode, None, 16, 0.125, p, True, 7, float("-inf"),
                              dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
    torch.cuda.synchronize()
    print("pmc_flash done", flush=True)


if __name__ == "__main__":
    main()
