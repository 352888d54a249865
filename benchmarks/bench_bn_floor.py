"""Floor check for the BN reductions at the ResNet-50 shapes: our statistics pass (k_stats_nhwc +
finalize), our backward reduction, torch's channel sum and a plain copy of the same tensor, timed
back-to-back with HIP events (per call). If torch's sum and the copy sit at the same time as ours on
the small (14x14, 7x7) layers the cost is the fixed per-kernel latency, not the kernel body.

    python benchmarks/bench_bn_floor.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import syncbn  # noqa: E402

SHAPES = [(56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 2048)]


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    only = os.environ.get("BN_SHAPE")  # e.g. "14x256": one shape (for rocprofv3 kernel traces)
    for H, C in SHAPES:
        if only and only != f"{H}x{C}":
            continue
        x = torch.randn(256, C, H, H, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        w = torch.rand(C, device="cuda") + 0.5
        b = torch.randn(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        mean, invstd, scale, shift, count = syncbn.stats_single(x, w, b, rm, rv, 0.1, 1e-5)
        y = torch.empty_like(x)
        r = {"H": H, "C": C, "MB": round(x.numel() * 2 / 1e6, 1),
             "stats_us": timeit(lambda: syncbn.stats_single(x, w, b, rm, rv, 0.1, 1e-5)),
             "reduce_us": timeit(lambda: syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, True)),
             "torch_sum_us": timeit(lambda: x.sum(dim=(0, 2, 3), dtype=torch.float32)),
             "copy_us": timeit(lambda: y.copy_(x)),
             "empty_kernel_us": timeit(lambda: rm.add_(0.0))}
        r = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        r["stats_TBs"] = round(r["MB"] / r["stats_us"], 2)
        r["copy_TBs"] = round(2 * r["MB"] / r["copy_us"], 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
