"""Conv weight gradient at the ResNet-50 (batch 256) shapes (stride 1, and the 1x1 / stride-2
downsample layers): the MFMA kernel of kernels/conv_wgrad.hip vs MIOpen (torch.ops.aten.convolution_backward), fp16 channels_last.
One JSON line per shape plus a per-step total weighted by how often the shape occurs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import conv as bhconv  # noqa: E402

# (C_in, C_out, H, R, occurrences per ResNet-50 step)
SHAPES = [
    (64, 64, 56, 3, 3), (128, 128, 28, 3, 3), (256, 256, 14, 3, 5), (512, 512, 7, 3, 2),
    (64, 64, 56, 1, 1), (256, 64, 56, 1, 2), (64, 256, 56, 1, 4), (256, 128, 56, 1, 1),
    (512, 128, 28, 1, 3), (128, 512, 28, 1, 4), (512, 256, 28, 1, 1), (1024, 256, 14, 1, 5),
    (256, 1024, 14, 1, 6), (1024, 512, 14, 1, 1), (2048, 512, 7, 1, 2), (512, 2048, 7, 1, 3),
]
# 1x1 / stride 2 downsample layers: (C_in, C_out, H_in, R, occurrences), dY is H_in / 2 wide
S2_SHAPES = [(256, 512, 56, 1, 1), (512, 1024, 28, 1, 1), (1024, 2048, 14, 1, 1)]


def time_ms(fn, reps=10):
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
    n = int(os.environ.get("BATCH", "256"))
    tot = {"mfma": 0.0, "miopen": 0.0, "best": 0.0}
    only_r = int(os.environ.get("ONLY_R", "0"))  # e.g. ONLY_R=3 for counter passes over the 3x3 kernels
    only_s2 = os.environ.get("ONLY_S2", "0") == "1"
    shapes = [] if only_s2 else [sh + (1,) for sh in SHAPES if not only_r or sh[3] == only_r]
    if not only_r:
        shapes += [sh + (2,) for sh in S2_SHAPES]
    for cin, cout, h, r, cnt, st in shapes:
        ho = h // st
        x = torch.randn(n, cin, h, h, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, ho, ho, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
        w = torch.empty(cout, cin, r, r, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
        p = (r - 1) // 2
        mi = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [p, p], [1, 1], False, [0, 0], 1,
                                                         [False, True, False])[1]
        ours = (lambda: bhconv.conv_wgrad_s2(x, dy)) if st == 2 else (lambda: bhconv.conv_wgrad(x, dy, r))
        t_mi = time_ms(mi)
        rec = {"cin": cin, "cout": cout, "H": h, "R": r, "stride": st, "count": cnt, "miopen_ms": round(t_mi, 4)}
        if bhconv.wgrad_supported(x, dy, r, st):
            t_k = time_ms(ours)
            ref = mi().float()
            err = ((ours().float() - ref).abs().max() / ref.abs().max()).item()
            flop = 2.0 * n * ho * ho * cin * cout * r * r
            rec.update(mfma_ms=round(t_k, 4), mfma_tflops=round(flop / t_k / 1e9, 1), rel_err_vs_miopen=round(err, 5),
                       speedup=round(t_mi / t_k, 2))
        else:
            t_k = float("inf")
        tot["miopen"] += cnt * t_mi
        tot["mfma"] += cnt * (t_k if t_k != float("inf") else t_mi)
        tot["best"] += cnt * min(t_k, t_mi)
        print(json.dumps(rec), flush=True)
        del x, dy
    print(json.dumps({"per_step_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
