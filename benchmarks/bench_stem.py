"""ResNet-50 stem conv (7x7 / stride 2, 3 -> 64 channels, batch 256, fp16 channels_last) on MIOpen:
the input as it is (C = 3) vs zero-padded to C = 4 / 8 channels (aligned pixels), forward and
weight gradient. Probe for the stem's input layout."""
import json
import os

import torch
import torch.nn.functional as F


def t_ms(fn, reps=10):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    for c in (3,) if os.environ.get("STEM_ONLY") else (3, 4, 8):
        x = torch.randn(256, c, 224, 224, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
        w = torch.randn(64, c, 7, 7, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=2, padding=3)
        gy = torch.randn_like(y)
        fwd = t_ms(lambda: F.conv2d(x, w, stride=2, padding=3))
        wgrad = t_ms(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0],
                                                                 1, [False, True, False]))
        pad = t_ms(lambda: F.pad(x[:, :3], (0, 0, 0, 0, 0, c - 3)).contiguous(memory_format=torch.channels_last)) \
            if c > 3 else 0.0
        rec = {"C": c, "fwd_ms": round(fwd, 4), "wgrad_ms": round(wgrad, 4), "pad_copy_ms": round(pad, 4)}
        if c == 3:
            import sys

            sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            from beforeholiday_amd.ops import conv as bhconv

            if bhconv.stem_supported(x, w):
                t = t_ms(lambda: bhconv.stem_conv(x, w))
                err = ((bhconv.stem_conv(x, w).float() - y.float()).abs().max() / y.float().abs().max()).item()
                tw = t_ms(lambda: bhconv.stem_wgrad(x, gy))
                ref_w = torch.ops.aten.convolution_backward(gy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                            [False, True, False])[1].float()
                werr = ((bhconv.stem_wgrad(x, gy).float() - ref_w).abs().max() / ref_w.abs().max()).item()
                rec.update(mfma_stem_fwd_ms=round(t, 4), mfma_stem_tflops=round(2 * 256 * 112 * 112 * 64 * 147 / t / 1e9, 1),
                           rel_err_vs_miopen=round(err, 5), mfma_stem_wgrad_ms=round(tw, 4),
                           wgrad_rel_err_vs_miopen=round(werr, 5))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
