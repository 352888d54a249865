"""Stride-2 3x3 convolutions of ResNet-50 (batch 256) on MIOpen: time and run-to-run repeatability of
forward / data gradient / weight gradient with torch.backends.cudnn.deterministic off and on."""
import json
import sys

import torch

conv_bwd = torch.ops.aten.convolution_backward
for c, hw in ((128, 56), (256, 28), (512, 14)):
    x = torch.randn(256, c, hw, hw, device="cuda").half().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).half().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(256, c, hw // 2, hw // 2, device="cuda").half().contiguous(memory_format=torch.channels_last)
    for det in (False, True):
        with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=det):
            fns = {
                "fwd": lambda: torch.nn.functional.conv2d(x, w, stride=2, padding=1),
                "dgrad": lambda: conv_bwd(gy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0],
                "wgrad": lambda: conv_bwd(gy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1],
            }
            for name, fn in fns.items():
                a = fn().clone()
                same = all(torch.equal(a, fn()) for _ in range(3))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                print(json.dumps({"C": c, "HW": hw, "dir": name, "deterministic": det, "repeatable": same,
                                  "ms": round(s.elapsed_time(e) / 10, 4)}))
                sys.stdout.flush()
