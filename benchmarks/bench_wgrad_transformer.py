"""The transformer weight gradient dW = dY^T . X (tokens are the reduction) on the 1x1 conv
weight-gradient MFMA kernel (kernels/conv_wgrad.hip, the [tokens, channels] views as a 1 x 1 x tokens
image) vs hipBLASLt (torch.mm). GPT-2-medium / BERT-large shapes at 8192 tokens, bf16. JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import conv as bhconv  # noqa: E402

SHAPES = [  # (tokens, out features K, in features C, role)
    (8192, 3072, 1024, "qkv"), (8192, 1024, 1024, "attn out"), (8192, 4096, 1024, "fc1"), (8192, 1024, 4096, "fc2"),
    (16384, 1024, 1024, "attn out 16k"), (4096, 1024, 1024, "attn out 4k"), (8192, 2048, 1024, "2k x 1k"),
    (8192, 1024, 2048, "1k x 2k"), (8192, 2048, 2048, "2k x 2k"), (8192, 768, 768, "base"), (8192, 512, 512, "512"),
    (8192, 3072, 768, "base fc1"), (8192, 768, 3072, "base fc2"),
]


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dt = torch.bfloat16
    for M, K, C, role in SHAPES:
        dy = torch.randn(M, K, device="cuda", dtype=dt)
        x = torch.randn(M, C, device="cuda", dtype=dt)
        # NHWC views: N = 1, H = 1, W = tokens
        x4 = x.view(1, 1, M, C).permute(0, 3, 1, 2)
        dy4 = dy.view(1, 1, M, K).permute(0, 3, 1, 2)
        r = {"tokens": M, "K": K, "C": C, "role": role, "supported": bool(bhconv.wgrad_supported(x4, dy4, 1))}
        flops = 2.0 * M * K * C
        r["blaslt_ms"] = round(t_ms(lambda: torch.mm(dy.t(), x)), 4)
        if r["supported"]:
            ref = torch.mm(dy.t().float(), x.float())
            got = bhconv.conv_wgrad(x4, dy4, 1).view(K, C).float()
            r["rel_err"] = float((got - ref).norm() / ref.norm())
            r["own_ms"] = round(t_ms(lambda: bhconv.conv_wgrad(x4, dy4, 1)), 4)
            r["own_tflops"] = round(flops / r["own_ms"] / 1e9, 1)
        r["blaslt_tflops"] = round(flops / r["blaslt_ms"] / 1e9, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
