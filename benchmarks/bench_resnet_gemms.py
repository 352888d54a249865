"""The ResNet-50 (batch 256) 1x1-convolution GEMMs that the strip kernel does not take (K or N >= 512,
or fewer than 100k pixel rows): hipBLASLt (torch.mm) vs the own MFMA GEMM per tile configuration
(kernels/gemm.hip: 1 = 128x128, 2 = 256x256, 3 = 256x128, 4 = ping-pong 256x256), plain C = A.B^T, and
the own GEMM with the BatchNorm-statistics epilogue vs hipBLASLt + the statistics pass. us per call,
JSON lines; ``calls`` is the number of such GEMMs per training step."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (M pixels, N out, K in, calls per step, role)
SHAPES = [
    (200704, 128, 512, 3, "s2 conv1 fwd / conv3 dgrad"),
    (50176, 256, 1024, 5, "s3 conv1 fwd / conv3 dgrad"),
    (12544, 512, 2048, 2, "s4 conv1 fwd / conv3 dgrad"),
    (200704, 512, 128, 3, "s2 conv1 dgrad"),
    (50176, 1024, 256, 5, "s3 conv1 dgrad"),
    (12544, 2048, 512, 2, "s4 conv1 dgrad"),
    (50176, 1024, 512, 1, "s3 downsample fwd (gathered)"),
    (12544, 2048, 1024, 1, "s4 downsample fwd (gathered)"),
    (50176, 512, 1024, 1, "s3 downsample dgrad"),
    (12544, 1024, 2048, 1, "s4 downsample dgrad"),
]


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from beforeholiday_amd._native import require_native, submodule
    from beforeholiday_amd.ops import conv_bn

    require_native("bench_resnet_gemms")
    gm = submodule("gemm")
    gm.set_force_mfma(True)
    modes = [int(m) for m in os.environ.get("MODES", "1,2,3,4").split(",")]
    tot = {}
    for M, N, K, calls, role in SHAPES:
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        b = torch.randn(N, K, device="cuda", dtype=torch.float16) * 0.05
        r = {"M": M, "N": N, "K": K, "calls": calls, "role": role}
        r["blaslt"] = timeit(lambda: torch.mm(a, b.t()))
        ks = torch.zeros(N, device="cuda")

        for mode in modes:
            gm.set_tile_mode(mode)
            r[f"t{mode}"] = timeit(lambda: gm.linear_act(a, b, None, 0, False))
            r[f"t{mode}_stats"] = timeit(lambda: conv_bn.gemm_bn(a, b, "stats", kshift=ks))
        gm.set_tile_mode(0)
        r["auto_stats"] = timeit(lambda: conv_bn.gemm_bn(a, b, "stats", kshift=ks))
        tf = 2.0 * M * N * K / 1e6
        r["blaslt_tflops"] = round(tf / r["blaslt"], 1)
        best = min(r[f"t{m}"] for m in modes)
        r["best_own_tflops"] = round(tf / best, 1)
        for k in list(r):
            if isinstance(r[k], float) and k not in ("blaslt_tflops", "best_own_tflops"):
                r[k] = round(r[k], 1)
                if k not in tot:
                    tot[k] = 0.0
                tot[k] += r[k] * calls
        print(json.dumps(r), flush=True)
        del a, b
    print(json.dumps({"weighted_us_per_step": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
