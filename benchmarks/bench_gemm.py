"""Fused dense layers: MFMA GEMM + epilogue (kernels/gemm.hip) vs hipBLASLt GEMM + separate pass.

For each shape: forward  y = GELU(x W^T + b) with the pre-activation kept (FusedDenseGeluDense's
first layer) and backward  dH = (dY W) * GELU'(pre), db = colsum(dH) (its DGELU_BGRAD step).
'mfma' = one gemm.hip launch (+ the tiny bias-grad finalize); 'blaslt' = at::addmm / at::mm on
hipBLASLt followed by the dense.hip activation pass (the BH_DENSE_MFMA=0 path). Also times a
plain GEMM of the same shape (torch.mm, hipBLASLt) as the roofline reference. Prints JSON lines.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M tokens, N out, K in)
    (1536, 3072, 1024),   # apex fused_dense test shape (seq 512 x 3, 1024 -> 3072)
    (8192, 4096, 1024),   # BERT-large FFN up-projection, batch 16 x 512
    (8192, 1024, 4096),   # BERT-large FFN down-projection
    (1024, 1024, 480),    # apex MLP test layer sizes [480, 1024, ...], batch 1024
    (4096, 4096, 4096),
]


def timeit(fn, iters=50, warm=10):
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
    from beforeholiday_amd._native import require_native, submodule

    require_native("bench_gemm")
    gm, fd = submodule("gemm"), submodule("fused_dense_cuda")
    gm.set_force_mfma(True)  # time the kernels themselves, not the measured dispatch
    out = []
    # plain C = A.B^T per tile kernel (uniform [-1, 1) operands) vs hipBLASLt
    for dtype in (torch.bfloat16,):
        for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 4096, 1024), (8192, 1024, 4096),
                        (16384, 1024, 1024)]:
            a = torch.rand(M, K, device="cuda", dtype=dtype) * 2 - 1
            bm = torch.rand(N, K, device="cuda", dtype=dtype) * 2 - 1
            flops = 2.0 * M * N * K
            r = {"kind": "plain", "dtype": str(dtype).split(".")[1], "M": M, "N": N, "K": K}
            iters = 20 if M * N * K >= 2 ** 38 else 50
            r["blaslt_tflops"] = round(flops / timeit(lambda: torch.mm(a, bm.t()), iters) / 1e9, 1)
            for mode, name in ((1, "t128"), (2, "t256"), (4, "pingpong")):
                gm.set_tile_mode(mode)
                r[name + "_tflops"] = round(flops / timeit(lambda: gm.linear_act(a, bm, None, 0, False), iters) / 1e9, 1)
            gm.set_tile_mode(0)
            out.append(r)
            print(json.dumps(r), flush=True)
    for dtype in (torch.bfloat16, torch.float16):
        for M, N, K in SHAPES:
            x = torch.randn(M, K, device="cuda", dtype=dtype)
            w = torch.randn(N, K, device="cuda", dtype=dtype) / K ** 0.5
            b = torch.randn(N, device="cuda", dtype=dtype)
            dy = torch.randn(M, K, device="cuda", dtype=dtype)   # grad wrt the GEMM output of [M, K] . W2
            w2t = torch.randn(N, K, device="cuda", dtype=dtype) / K ** 0.5  # W2^T  [N, K]
            pre = torch.randn(M, N, device="cuda", dtype=dtype)
            flops = 2.0 * M * N * K

            t_mfma_f = timeit(lambda: gm.linear_act(x, w, b, 3, True))
            t_lt_f = timeit(lambda: (lambda y: (y, fd.act_forward(y, None, 3)))(torch.addmm(b, x, w.t())))
            t_mfma_b = timeit(lambda: gm.linear_dact(dy, w2t, pre, 3, True))
            t_lt_b = timeit(lambda: fd.act_backward(torch.mm(dy, w2t.t()), pre, 3, True))
            t_mm = timeit(lambda: torch.mm(x, w.t()))
            r = {"dtype": str(dtype).split(".")[1], "M": M, "N": N, "K": K,
                 "fwd_mfma_ms": round(t_mfma_f, 4), "fwd_blaslt_plus_pass_ms": round(t_lt_f, 4),
                 "bwd_mfma_ms": round(t_mfma_b, 4), "bwd_blaslt_plus_pass_ms": round(t_lt_b, 4),
                 "plain_blaslt_mm_ms": round(t_mm, 4),
                 "mfma_fwd_tflops": round(flops / t_mfma_f / 1e9, 1), "blaslt_mm_tflops": round(flops / t_mm / 1e9, 1),
                 "fwd_speedup": round(t_lt_f / t_mfma_f, 3), "bwd_speedup": round(t_lt_b / t_mfma_b, 3)}
            out.append(r)
            print(json.dumps(r), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.environ.get("BENCH_GEMM_OUT", "gpurun_out/gemm.jsonl"), "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
