"""Compare the loss trajectories of an L1 run with the fused extension (``True_*``) and the
python-only path (``False_*``) (reference: tests/L1/common/compare.py:37-56). Exact equality per
iteration, as in the reference; ``--rtol`` relaxes it for runs with non-deterministic kernels."""
import argparse
import os
import sys

import torch


def trajectory_name(has_ext, opt_level, loss_scale, keep_bn, fused_adam=False):
    return "{}_{}_{}_{}_{}".format(bool(has_ext), opt_level, loss_scale, keep_bn, bool(fused_adam))


def compare(dir_, opt_level, loss_scale=None, keep_bn=None, fused_adam=False, rtol=0.0, baseline_dir=None):
    e = torch.load(os.path.join(dir_, trajectory_name(True, opt_level, loss_scale, keep_bn, fused_adam)),
                   weights_only=True)
    p = torch.load(os.path.join(dir_, trajectory_name(False, opt_level, loss_scale, keep_bn, fused_adam)),
                   weights_only=True)
    others = [p]
    if baseline_dir:
        others.append(torch.load(os.path.join(baseline_dir, trajectory_name(True, opt_level, loss_scale, keep_bn,
                                                                             fused_adam)), weights_only=True))
    assert len(e["Loss"]) > 0, "empty trajectory"
    for o in others:
        assert e["Iteration"] == o["Iteration"], (e["Iteration"], o["Iteration"])
        for it, le, lo in zip(e["Iteration"], e["Loss"], o["Loss"]):
            ok = le == lo if rtol == 0.0 else abs(le - lo) <= rtol * max(abs(le), abs(lo))
            assert ok, "iteration {}: loss_e = {!r}, loss_p = {!r}".format(it, le, lo)
    return e["Loss"], p["Loss"]


def main(argv=None):
    ap = argparse.ArgumentParser(description="L1 trajectory compare")
    ap.add_argument("--dir", default=".")
    ap.add_argument("--opt-level", required=True)
    ap.add_argument("--keep-batchnorm-fp32", default=None)
    ap.add_argument("--loss-scale", default=None)
    ap.add_argument("--fused-adam", action="store_true")
    ap.add_argument("--rtol", type=float, default=0.0)
    ap.add_argument("--baseline-dir", default=None)
    a = ap.parse_args(argv)
    le, lp = compare(a.dir, a.opt_level, a.loss_scale, a.keep_batchnorm_fp32, a.fused_adam, a.rtol, a.baseline_dir)
    for i, (x, y) in enumerate(zip(le, lp)):
        print("{:4} {:15.10f} {:15.10f}".format(i, x, y))
    return 0


if __name__ == "__main__":
    sys.exit(main())
