"""Which Python call sites still hand GEMMs to the library (hipBLASLt / rocBLAS) in a bench.py step:
wraps torch.mm / addmm / matmul / F.linear, runs bench.main() eagerly (--graph off) and prints
(call site, op, operand shapes, strides) x calls per step. C++ at::mm calls are not seen.

usage: python scripts/probes/mm_shapes.py [bench.py args ...]
"""
import collections
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
_calls = collections.Counter()


def _wrap(name, fn):
    def inner(*args, **kw):
        f = sys._getframe(1)
        site = f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}"
        ts = [a for a in args if isinstance(a, torch.Tensor)]
        sig = " ".join(f"{tuple(t.shape)}{'' if t.is_contiguous() else 's' + str(t.stride())}" for t in ts)
        _calls[(site, name, sig)] += 1
        return fn(*args, **kw)

    return inner


torch.mm = _wrap("mm", torch.mm)
torch.addmm = _wrap("addmm", torch.addmm)
torch.matmul = _wrap("matmul", torch.matmul)
F.linear = _wrap("linear", F.linear)

import bench  # noqa: E402

steps, warmup = 2, 1
sys.argv = ["bench.py", "--steps", str(steps), "--warmup", str(warmup), "--graph", "off"] + sys.argv[1:]
bench.main()
for (site, name, sig), n in sorted(_calls.items(), key=lambda kv: -kv[1]):
    print(f"{n:4d} calls ({n / (steps + warmup):5.2f}/step)  {site:28s} {name:7s} {sig}")
