"""Drive the flash attention kernels (kernels/attn.hip) at the BERT-large shape (16 seqs x 16 heads x
512 tokens, head 64, dropout 0.1) for rocprofv3 counter passes (scripts/pmc_flash.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from beforeholiday_amd._native import require_native, submodule

    require_native("pmc_flash")
    fa = submodule("fused_attention")
    dt = torch.bfloat16
    S, BH = 512, 256
    qkv = torch.randn(S, BH, 3, 64, device="cuda", dtype=dt)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    dout = torch.randn(S, BH, 64, device="cuda", dtype=dt)
    dqkv = torch.empty_like(qkv)
    for _ in range(10):
        o, lse = fa.flash_forward(q, k, v, 0, None, 16, 0.125, 0.1, True, 7, float("-inf"))
        fa.flash_backward(dout, q, k, v, o, lse, 0, None, 16, 0.125, 0.1, True, 7, float("-inf"),
                          dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
    torch.cuda.synchronize()
    print("pmc_flash done", flush=True)


if __name__ == "__main__":
    main()
