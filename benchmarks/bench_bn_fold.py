"""Microbenchmark of the BatchNorm-fold kernels (ops/bn_fold.py) at the ResNet-50 / batch-256 shapes:
Gram (with / without the BatchNorm prologue, stride-2 rows), mask + column sums. Prints one JSON line per
shape with the time per call and the effective HBM rate of the bytes the kernel must read / write."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from beforeholiday_amd.ops import bn_fold


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for name, M, K, pro, s2 in [("l1_bn2", 802816, 64, True, None), ("l2_bn2", 200704, 128, True, None),
                                ("l1_ds", 802816, 64, False, None), ("l2_ds_s2", 802816, 256, False, (56, 56)),
                                ("l3", 50176, 256, False, None), ("l4", 12544, 512, False, None)]:
        a = torch.randn(M, K, device=dev).half()
        s = torch.rand(K, device=dev) + 0.5 if pro else None
        t = torch.randn(K, device=dev) * 0.1 if pro else None
        us = timed(lambda: bn_fold.gram_partials(a, s, t, s2))
        rows = M // 4 if s2 else M
        gb = rows * K * 2 / 1e9
        print(json.dumps({"kernel": "gram", "shape": name, "M": rows, "K": K, "pro": pro, "us": round(us, 1),
                          "GBps": round(gb / us * 1e6, 1), "TFLOPs": round(2 * rows * K * K / us / 1e6, 1)}))
    for name, M, N in [("l1", 802816, 256), ("l2", 200704, 512)]:
        g = torch.randn(M, N, device=dev).half()
        bits = torch.randint(0, 256, (M, N // 8), dtype=torch.uint8, device=dev)
        us = timed(lambda: bn_fold.mask_colsum_partials(g, bits))
        gb = (2 * M * N * 2 + M * N / 8) / 1e9
        print(json.dumps({"kernel": "mask_colsum", "shape": name, "us": round(us, 1), "GBps": round(gb / us * 1e6, 1)}))


if __name__ == "__main__":
    main()
