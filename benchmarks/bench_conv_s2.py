"""Stride-2 3x3 convolutions of ResNet-50 at batch 256: the own MFMA kernels (implicit-GEMM forward /
data gradient, strided-halo weight gradient) vs MIOpen, ms per call and TFLOP/s. JSON lines."""
import json
import sys

import torch

sys.path.insert(0, ".")
from beforeholiday_amd.ops import conv as bhconv  # noqa: E402


def t_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


conv_bwd = torch.ops.aten.convolution_backward
dt = torch.float16 if "--bf16" not in sys.argv else torch.bfloat16
for c, hw in ((128, 56), (256, 28), (512, 14)):
    n = 256
    x = torch.randn(n, c, hw, hw, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, c, hw // 2, hw // 2, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    sc = torch.rand(c, device="cuda") + 0.5
    sh = torch.randn(c, device="cuda")
    flop = 2.0 * n * (hw // 2) ** 2 * c * c * 9
    rows = {
        "fwd": (lambda: bhconv.conv3x3_s2(x, w), lambda: torch.nn.functional.conv2d(x, w, stride=2, padding=1)),
        "fwd_pro_stats": (lambda: bhconv.conv3x3_s2(x, w, sc, sh, True), None),
        "dgrad": (lambda: bhconv.conv3x3_s2_dgrad(gy, w, (hw, hw)),
                  lambda: conv_bwd(gy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
        "wgrad": (lambda: bhconv.conv_wgrad(x, gy, 3, stride=2),
                  lambda: conv_bwd(gy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])),
        "wgrad_pro": (lambda: bhconv.conv_wgrad(x, gy, 3, sc, sh, stride=2), None),
    }
    for name, (own, lib) in rows.items():
        a = t_ms(own)
        b = t_ms(lib) if lib is not None else None
        print(json.dumps({"C": c, "K": c, "HW_in": hw, "N": n, "dtype": str(dt).split(".")[1], "dir": name,
                          "own_ms": round(a, 4), "own_tflops": round(flop / a / 1e9, 1),
                          "miopen_ms": None if b is None else round(b, 4),
                          "speedup": None if b is None else round(b / a, 3)}))
        sys.stdout.flush()
