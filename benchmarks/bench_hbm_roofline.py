"""HBM roofline check for the BatchNorm passes at the largest ResNet-50 shape (batch 256, 56x56x256
fp16 = 411 MB per tensor): achieved GB/s of torch's copy / add / channel sum (read-write, 2-read-1-write,
read-only references) next to the BatchNorm forward (+residual +ReLU mask), backward reduce and backward
dgrad (+dz) kernels of kernels/batchnorm.hip, moving the same bytes. JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd.ops import syncbn  # noqa: E402


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
    H, C, N = 56, 256, 256
    mk = lambda: torch.randn(N, C, H, H, device="cuda", dtype=torch.float16).contiguous(  # noqa: E731
        memory_format=torch.channels_last)
    x, z, dy, out = mk(), mk(), mk(), mk()
    nb = x.numel() * 2
    scale = torch.rand(C, device="cuda") + 0.5
    shift = torch.randn(C, device="cuda") * 0.1
    mean = torch.zeros(C, device="cuda")
    invstd = torch.ones(C, device="cuda")
    w = torch.ones(C, device="cuda")
    count = torch.full((1,), float(N * H * H), device="cuda")
    (y, mask) = syncbn.forward_mask(x, z, scale, shift)
    sums, _, _ = syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, False, mask)
    rows = [
        ("torch_copy", lambda: out.copy_(x), 2 * nb),
        ("torch_add", lambda: torch.add(x, z, out=out), 3 * nb),
        ("torch_sum_channels", lambda: x.sum(dim=(0, 2, 3)), nb),
        ("bn_fwd_residual_relu_mask", lambda: syncbn.forward_mask(x, z, scale, shift), 3 * nb + nb // 16),
        ("bn_fwd_residual_relu_nomask", lambda: syncbn.forward(x, z, scale, shift, True), 3 * nb),
        ("bn_fwd_plain", lambda: syncbn.forward(x, None, scale, shift, True), 2 * nb),
        ("bn_bwd_reduce_z_nomask", lambda: syncbn.backward_reduce(dy, x, z, mean, invstd, scale, shift, True, w, False,
                                                                   None), 3 * nb),
        ("bn_bwd_reduce_plain_relu", lambda: syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w,
                                                                     False, None), 2 * nb),
        ("bn_bwd_dgrad_plain_relu", lambda: syncbn.backward_dgrad(dy, x, None, mean, invstd, w, sums, count, scale,
                                                                   shift, True, False, None), 3 * nb),
        ("bn_bwd_reduce_mask", lambda: syncbn.backward_reduce(dy, x, None, mean, invstd, scale, shift, True, w, False,
                                                               mask), 2 * nb + nb // 16),
        ("bn_bwd_dgrad_mask_dz", lambda: syncbn.backward_dgrad(dy, x, None, mean, invstd, w, sums, count, scale, shift,
                                                                True, True, mask), 4 * nb + nb // 16),
        ("bn_bwd_dgrad_mask", lambda: syncbn.backward_dgrad(dy, x, None, mean, invstd, w, sums, count, scale, shift,
                                                             True, False, mask), 3 * nb + nb // 16),
    ]
    for name, fn, nbytes in rows:
        us = timeit(fn)
        print(json.dumps({"kernel": name, "shape": [N, C, H, H], "us": round(us, 1), "MB": round(nbytes / 1e6, 1),
                          "GB_s": round(nbytes / us / 1e3, 0)}), flush=True)


if __name__ == "__main__":
    main()
