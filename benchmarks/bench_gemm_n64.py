"""The 64-channel side of ResNet-50's 56x56 1x1 convolutions (batch 256): kernels/gemm_n64.hip vs
torch.mm (hipBLASLt) and the MIOpen convolution it replaces, fp16 channels_last. One JSON line per
op with the HBM floor at the bytes moved."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import conv as bhconv  # noqa: E402


def time_ms(fn, reps=20):
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
    n, h = int(os.environ.get("BATCH", "256")), 56
    M = n * h * h
    cl = torch.channels_last
    for name, cin, cout in [("fwd 256->64", 256, 64), ("fwd 64->64", 64, 64), ("dgrad 64->256", 64, 256),
                            ("dgrad 64->64", 64, 64)]:
        if name.startswith("fwd"):
            x = torch.randn(n, cin, h, h, device="cuda", dtype=torch.half).contiguous(memory_format=cl)
            w = torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.half) * cin ** -0.5
            a2, b2 = x.permute(0, 2, 3, 1).reshape(M, cin), w.view(cout, cin)
            mi = lambda: torch.nn.functional.conv2d(x, w)  # noqa: E731
        else:
            dy = torch.randn(n, cout, h, h, device="cuda", dtype=torch.half).contiguous(memory_format=cl)
            w = torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.half) * cout ** -0.5
            a2, b2 = dy.permute(0, 2, 3, 1).reshape(M, cout), w.view(cout, cin).t().contiguous()
            mi = lambda: torch.ops.aten.convolution_backward(dy, dy.new_empty(n, cin, h, h).contiguous(memory_format=cl),  # noqa: E731
                                                             w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                             [True, False, False])[0]
        k = a2.size(1)
        t_k = time_ms(lambda: bhconv.gemm_n64(a2, b2))
        t_mm = time_ms(lambda: torch.mm(a2, b2.t()))
        t_mi = time_ms(mi)
        err = (bhconv.gemm_n64(a2, b2).float() - torch.mm(a2, b2.t()).float()).abs().max().item()
        gb = (M * k + M * 64) * 2 / 1e9
        print(json.dumps({"op": name, "M": M, "K": k, "n64_ms": round(t_k, 4), "hipblaslt_ms": round(t_mm, 4),
                          "miopen_ms": round(t_mi, 4), "n64_TBps": round(gb / t_k, 2), "max_abs_diff": err}),
              flush=True)


if __name__ == "__main__":
    main()
