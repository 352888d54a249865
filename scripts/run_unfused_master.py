"""A/B helper: run a bench script with amp's fused mixed-precision optimizer step turned off
(amp/_process_optimizer.py ``fused_master_step``). Usage: python scripts/run_unfused_master.py SCRIPT ARGS..."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import beforeholiday_amd.amp._process_optimizer as _po  # noqa: E402

_po.fused_master_step = False
script = sys.argv[1]
sys.argv = sys.argv[1:]
runpy.run_path(script, run_name="__main__")
