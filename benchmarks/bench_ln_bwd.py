"""FusedLayerNorm backward at the transformer shape (8192 tokens x 1024, fp16): us per backward
(data gradient + gamma / beta gradients), for sweeping BH_LN_WGRAD_ROWS / BH_LN_WGRAD_WGS; the one-pass
fused backward (Config.ln_bwd_fused) and the two-pass one, interleaved in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from beforeholiday_amd import config

    for rep in range(2):
        for fused in (True, False):
            with config.override(ln_bwd_fused=fused):
                run({"rep": rep, "ln_bwd_fused": fused})


def run(out):
    from beforeholiday_amd.normalization import FusedLayerNorm

    out.update({"rows": os.environ.get("BH_LN_WGRAD_ROWS", "8"), "wgs": os.environ.get("BH_LN_WGRAD_WGS", "512")})
    for dtype in (torch.float16, torch.bfloat16):
        ln = FusedLayerNorm(1024).cuda().to(dtype)
        x = torch.randn(8192, 1024, device="cuda", dtype=dtype, requires_grad=True)
        y = ln(x)
        dy = torch.randn_like(y)
        for _ in range(5):
            torch.autograd.grad(y, [x, ln.weight, ln.bias], dy, retain_graph=True)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(50):
            torch.autograd.grad(y, [x, ln.weight, ln.bias], dy, retain_graph=True)
        e.record()
        torch.cuda.synchronize()
        out[str(dtype).split(".")[-1]] = round(s.elapsed_time(e) / 50 * 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
