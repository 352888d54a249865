"""ResNet-50 1x1 convolutions at batch 256 (fp16, NHWC as [pixels, channels]): the conv_bn kernel
(kernels/conv_bn.hip) against what it replaces, per layer shape and direction:

  fwd   : hipBLASLt mm + the separate BatchNorm statistics pass  vs  c1x1 with the statistics epilogue
  pro   : BatchNorm-apply pass + hipBLASLt mm + statistics pass    vs  c1x1 with prologue + statistics
  dgrad : hipBLASLt mm + BatchNorm backward-reduce pass           vs  c1x1 with the backward epilogue
          (weights read transposed, as in the data gradient)
  s2    : strided gather + mm + statistics                        vs  c1x1 stride-2 gather + statistics

One JSON line per (shape, mode) with ms of both sides and the kernel's effective HBM TB/s
(unique bytes of A, B, C, and the epilogue's extra input).

    python benchmarks/bench_conv_bn.py [--batch 256] [--out file.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (K, N, H, W, mode): forward / prologue / dgrad shapes of the bottleneck 1x1 convs
SHAPES = [
    (64, 64, 56, 56, "fwd"), (256, 64, 56, 56, "fwd"), (64, 256, 56, 56, "pro"), (64, 256, 56, 56, "fwd"),
    (256, 128, 56, 56, "fwd"), (512, 128, 28, 28, "fwd"), (128, 512, 28, 28, "pro"),
    (512, 256, 28, 28, "fwd"), (1024, 256, 14, 14, "fwd"), (256, 1024, 14, 14, "pro"),
    (1024, 512, 14, 14, "fwd"), (512, 2048, 7, 7, "pro"),
    (128, 512, 28, 28, "fwd"), (256, 1024, 14, 14, "fwd"), (512, 2048, 7, 7, "fwd"),
    (256, 64, 56, 56, "dgrad"), (512, 128, 28, 28, "dgrad"), (1024, 256, 14, 14, "dgrad"),
    (64, 64, 56, 56, "dgrad"), (64, 256, 56, 56, "dgrad"), (128, 512, 28, 28, "dgrad"), (256, 1024, 14, 14, "dgrad"),
    (512, 2048, 7, 7, "dgrad"), (2048, 512, 7, 7, "dgrad"),
    (64, 256, 56, 56, "plain"), (128, 512, 28, 28, "plain"), (256, 1024, 14, 14, "plain"), (512, 2048, 7, 7, "plain"),
    (256, 512, 56, 56, "s2"), (512, 1024, 28, 28, "s2"), (1024, 2048, 14, 14, "s2"),
]


def timeit(fn, iters=20, warm=3):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from beforeholiday_amd.ops import conv_bn, syncbn

    dt = torch.float16
    lines = []
    for K, N, H, W, mode in SHAPES:
        torch.manual_seed(0)
        rows = args.batch * H * W
        M = rows // 4 if mode == "s2" else rows
        a = torch.randn(rows, K, device="cuda", dtype=dt)
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        rm = torch.zeros(N, device="cuda")
        sc = torch.rand(K, device="cuda") + 0.5
        sh = torch.randn(K, device="cuda") * 0.1
        y = torch.randn(M, N, device="cuda", dtype=dt)
        scn, shn, mn = torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda"), torch.zeros(N, device="cuda")

        def stats(c):  # the unfused statistics pass of the BatchNorm after the conv
            return syncbn.stats_local_sums(c.view(-1, H if mode != "s2" else H // 2, W if mode != "s2" else W // 2,
                                                  N).permute(0, 3, 1, 2), rm)

        if mode == "fwd" or mode == "fwd_n64":
            ours = lambda: conv_bn.sum_parts(conv_bn.c1x1(a, b, epi="stats", kshift=rm)[1], M)  # noqa: E731
            base = lambda: stats(torch.mm(a, b.t()))  # noqa: E731
            extra = 0
        elif mode == "pro":
            ours = lambda: conv_bn.sum_parts(conv_bn.c1x1(a, b, sc, sh, epi="stats", kshift=rm)[1], M)  # noqa: E731
            base = lambda: stats(torch.mm(torch.relu(a * sc.half() + sh.half()), b.t()))  # noqa: E731
            extra = 0
        elif mode == "plain":
            ours = lambda: conv_bn.c1x1(a, b)  # noqa: E731
            base = lambda: torch.mm(a, b.t())  # noqa: E731
            extra = 0
        elif mode == "dgrad":
            x4 = y.view(-1, H, W, N).permute(0, 3, 1, 2)

            def base():
                c = torch.mm(a, b.t())
                return syncbn.backward_reduce(c.view(-1, H, W, N).permute(0, 3, 1, 2), x4, None, mn, mn, scn, shn,
                                              True, None, False)

            bt = b.t().contiguous()  # the data gradient reads the forward weight [K, N] transposed

            def ours():
                return conv_bn.sum_parts(conv_bn.c1x1(a, bt, epi="bwd", by=y, bscale=scn, bshift=shn, bmean=mn,
                                                      b_trans=True)[1])
            extra = M * N * 2
        else:  # s2
            ours = lambda: conv_bn.sum_parts(conv_bn.c1x1(a, b, s2=(H, W), epi="stats", kshift=rm)[1], M)  # noqa: E731
            base = lambda: stats(torch.mm(a.view(-1, H, W, K)[:, ::2, ::2].reshape(-1, K), b.t()))  # noqa: E731
            extra = 0
        if not conv_bn.supported(a, bt if mode == "dgrad" else b, pro=mode == "pro", s2=(H, W) if mode == "s2" else None,
                                 b_trans=mode == "dgrad",
                                 epi={"fwd": "stats", "fwd_n64": "stats", "pro": "stats", "plain": "plain",
                                      "dgrad": "bwd", "s2": "stats"}[mode]):
            lines.append({"K": K, "N": N, "HW": H, "mode": mode, "supported": False})
            print(json.dumps(lines[-1]), flush=True)
            continue
        t_ours, t_base = timeit(ours), timeit(base)
        t_tiled = None  # the tiled GEMM with the same epilogue (kernels/gemm.hip)
        if mode in ("fwd", "plain"):
            t_tiled = timeit(lambda: conv_bn.sum_parts(conv_bn.gemm_bn(a, b, "stats", kshift=rm)[0 + 1], M))
        elif mode == "dgrad":
            t_tiled = timeit(lambda: conv_bn.sum_parts(conv_bn.gemm_bn(a, b, "bwd", by=y, bscale=scn, bshift=shn,
                                                                       bmean=mn)[1]))
        a_bytes = (M if mode == "s2" else rows) * K * 2
        byts = a_bytes + N * K * 2 + M * N * 2 + extra
        rec = {"K": K, "N": N, "HW": H, "M": M, "mode": mode, "ms_ours": round(t_ours, 4), "ms_unfused": round(t_base, 4),
               "speedup": round(t_base / t_ours, 3), "TBps_ours": round(byts / t_ours / 1e9, 2),
               "ms_tiled_gemm_bn": (round(t_tiled, 4) if t_tiled else None),
               "TFLOPs_ours": round(2 * M * K * N / t_ours / 1e9, 1)}
        lines.append(rec)
        print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
