"""The transformer data gradient dX = dY . W (W [out, in] row-major, so the library runs an NN GEMM)
vs the own NT MFMA GEMM on the transposed weight (gemm.transpose + gemm.mm_nt; the transpose is
timed too). GPT-2-medium / BERT-large shapes at 8192 tokens, bf16. JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (tokens, out, in, role): dX [tokens, in] = dY [tokens, out] . W [out, in]
    (8192, 3072, 1024, "qkv"), (8192, 1024, 1024, "attn out"), (8192, 4096, 1024, "fc1"), (8192, 1024, 4096, "fc2"),
    (8192, 768, 1024, "qkv tp4"), (8192, 1024, 256, "attn out tp4"), (8192, 1024, 1024, "fc1 tp4"),
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
    from beforeholiday_amd._native import submodule

    gm = submodule("gemm")
    dt = torch.bfloat16
    for M, O, I, role in SHAPES:
        dy = torch.randn(M, O, device="cuda", dtype=dt)
        w = torch.randn(O, I, device="cuda", dtype=dt) * 0.02
        r = {"tokens": M, "out": O, "in": I, "role": role}
        r["blaslt_ms"] = round(t_ms(lambda: torch.mm(dy, w)), 4)
        wt = gm.transpose(w)
        r["own_gemm_ms"] = round(t_ms(lambda: gm.mm_nt(dy, wt)), 4)
        r["own_total_ms"] = round(t_ms(lambda: gm.mm_nt(dy, gm.transpose(w))), 4)
        ref = torch.mm(dy.float(), w.float())
        r["rel_err"] = float((gm.mm_nt(dy, wt).float() - ref).norm() / ref.norm())
        r["speedup"] = round(r["blaslt_ms"] / r["own_total_ms"], 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
