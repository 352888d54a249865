"""BatchNorm backward-reduction pass at every ResNet-50 shape (batch 256): us per call, with the
ReLU bit mask (bn3 / downsample BNs: 2 reads + mask) and with the mask recomputed from x (bn1 / bn2:
2 reads). Run once per launch geometry (BH_BN_RED_BLOCKS / BH_BN_RED_ROWS) to pick the default; the
``weighted_ms`` line is the per-step total at ResNet-50's launch counts."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import syncbn  # noqa: E402

# (H, C, calls per step): bn3 / downsample (mask) and bn1 / bn2 (recomputed ReLU) shapes
MASK = [(56, 256, 4), (28, 512, 5), (14, 1024, 7), (7, 2048, 4)]
PLAIN = [(112, 64, 1), (56, 64, 5), (56, 128, 1), (28, 128, 7), (28, 256, 1), (14, 256, 11), (14, 512, 1),
         (7, 512, 5)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    tot = 0.0
    for masked, shapes in ((True, MASK), (False, PLAIN)):
        for H, C, calls in shapes:
            mk = lambda: torch.randn(256, C, H, H, device="cuda", dtype=torch.float16).contiguous(  # noqa: E731
                memory_format=torch.channels_last)
            x, z, dy = mk(), mk(), mk()
            scale = torch.rand(C, device="cuda") + 0.5
            shift = torch.randn(C, device="cuda") * 0.1
            mean = torch.zeros(C, device="cuda")
            invstd = torch.ones(C, device="cuda")
            w = torch.ones(C, device="cuda")
            mask = syncbn.forward_mask(x, z, scale, shift)[1] if masked else None
            us = timeit(lambda: syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, True, mask))
            tot += us * calls
            print(json.dumps({"H": H, "C": C, "mask": masked, "calls": calls, "us": round(us, 1)}), flush=True)
    print(json.dumps({"blocks": os.environ.get("BH_BN_RED_BLOCKS", "256"), "rows": os.environ.get("BH_BN_RED_ROWS", "32"),
                      "cvb": os.environ.get("BH_BN_RED_CVB", "256"), "weighted_ms": round(tot / 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
