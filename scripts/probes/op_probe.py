"""Probe: which aten ops launch the small elementwise / copy kernels of an eager bench step (torch.profiler
over bench.py --graph off; table of aten::copy_ / add / mul / to / contiguous ... with input shapes and
the Python stack)."""
import os
import runpy
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
out = sys.argv[1]
sys.argv = ["bench.py", "--steps", "1", "--warmup", "3", "--graph", "off"]
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    try:
        runpy.run_path("bench.py", run_name="__main__")
    except SystemExit:
        pass
keys = ("aten::copy_", "aten::add", "aten::add_", "aten::mul", "aten::mul_", "aten::maximum", "aten::where",
        "aten::clamp", "aten::fill_", "aten::zero_", "aten::reciprocal", "aten::div", "aten::eq", "aten::to",
        "aten::contiguous", "aten::cat", "aten::index", "aten::sum")
with open(out, "w") as f:
    tab = prof.key_averages(group_by_input_shape=True, group_by_stack_n=6)
    rows = [e for e in tab if e.key in keys and e.device_time_total > 0]
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:60]:
        f.write(f"{e.key} calls={e.count} dev_us={e.device_time_total:.0f} shapes={e.input_shapes}\n")
        for fr in (e.stack or [])[:6]:
            f.write(f"    {fr}\n")
print("wrote", out)
