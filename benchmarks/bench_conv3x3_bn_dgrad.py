"""3x3 data gradient with the previous BatchNorm's backward sums in its epilogue vs the plain data gradient
followed by the BatchNorm backward-reduce pass (ResNet-50 batch-256 bn1 shapes). One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd._native import submodule  # noqa: E402
from beforeholiday_amd.ops import conv as bhconv  # noqa: E402
from beforeholiday_amd.ops import syncbn  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for n, c, h, w in [(256, 64, 56, 56), (256, 128, 28, 28), (256, 256, 14, 14), (256, 512, 7, 7)]:
    cl = torch.channels_last
    dy = torch.randn(n, c, h, w, device="cuda", dtype=torch.half).contiguous(memory_format=cl)
    wt = (torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).half().contiguous(memory_format=cl)
    y = torch.randn(n, c, h, w, device="cuda", dtype=torch.half).contiguous(memory_format=cl)
    sc, sh = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.3
    mean, invstd = torch.randn(c, device="cuda") * 0.1, torch.rand(c, device="cuda") + 0.5
    dx = bhconv.conv3x3_dgrad(dy, wt)
    t_plain = timed(lambda: bhconv.conv3x3_dgrad(dy, wt))
    t_red = timed(lambda: syncbn.backward_reduce(dx, y, None, mean, invstd, sc, sh, True, None, False, None))
    t_epi = timed(lambda: submodule("conv_cuda").conv3x3_bn_dgrad(dy, wt, y, sc, sh, mean, True))
    print(json.dumps({"shape": [n, c, h, w], "dgrad_us": round(t_plain, 1), "reduce_us": round(t_red, 1),
                      "dgrad_plus_reduce_us": round(t_plain + t_red, 1), "dgrad_bn_epilogue_us": round(t_epi, 1)}),
          flush=True)
