"""Attention core (QK^T -> masked softmax -> dropout -> PV) at BERT-large / GPT shapes, fwd and bwd ms:
MFMA flash kernels (kernels/attn.hip) vs the unfused Megatron path (bmm + fused softmax kernel +
dropout + bmm) vs torch SDPA. One JSON line per (shape, impl)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (batch, heads, seq, causal)
    (16, 16, 512, False),   # BERT-large pretraining, seq 512
    (8, 16, 1024, True),    # GPT-2 medium
    (4, 16, 2048, True),
]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    from beforeholiday_amd import config
    from beforeholiday_amd._native import require_native, submodule
    from beforeholiday_amd.contrib.multihead_attn._core import MASK_CAUSAL, MASK_NONE, FusedSelfAttnFn

    require_native("bench_attention")
    p = float(os.environ.get("ATTN_DROPOUT", "0.1"))
    dt = torch.bfloat16
    for B, H, S, causal in SHAPES:
        qkv = torch.randn(S, B * H, 3, 64, device="cuda", dtype=dt, requires_grad=True)
        g = torch.randn(S, B * H, 64, device="cuda", dtype=dt)
        mode = MASK_CAUSAL if causal else MASK_NONE
        flops = 4 * B * H * S * S * 64 * (0.5 if causal else 1.0)
        config.set(attn_flash_only=True)

        def ours():
            return FusedSelfAttnFn.apply(qkv, H, 0.125, None, mode, p, True, float("-inf"))

        def unfused():
            q, k, v = (qkv[:, :, i].transpose(0, 1) for i in range(3))  # [BH, S, 64]
            s = torch.baddbmm(q.new_empty(B * H, S, S), q, k.transpose(1, 2), beta=0.0, alpha=0.125)
            if causal:
                s = s.masked_fill(torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
            pr = F.dropout(torch.softmax(s, -1), p=p)
            return torch.bmm(pr, v).transpose(0, 1)

        def sdpa():
            q, k, v = (qkv[:, :, i].view(S, B, H, 64).permute(1, 2, 0, 3) for i in range(3))
            return F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=causal)

        for name, fn in (("flash_mfma", ours), ("unfused_bmm_softmax", unfused), ("torch_sdpa", sdpa)):
            try:
                tf = timeit(fn)
                out = fn()
                gg = g if out.shape == g.shape else g.view(S, B, H, 64).permute(1, 2, 0, 3)
                tb = timeit(lambda: torch.autograd.grad(out, qkv, gg, retain_graph=True))
                r = {"B": B, "H": H, "S": S, "causal": causal, "dropout": p, "impl": name, "fwd_ms": round(tf, 3),
                     "bwd_ms": round(tb, 3), "fwd_tflops": round(flops / tf / 1e9, 1),
                     "bwd_tflops": round(2.5 * flops / tb / 1e9, 1)}
            except Exception as e:  # noqa: BLE001 - e.g. SDPA backend unavailable
                r = {"B": B, "H": H, "S": S, "impl": name, "error": repr(e)[:200]}
            print(json.dumps(r), flush=True)
        config.set(attn_flash_only=False)
        del qkv, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
