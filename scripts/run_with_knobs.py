"""A/B helper: run a script with native knobs set (``python scripts/run_with_knobs.py name=value ... -- SCRIPT ARGS``)."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beforeholiday_amd import _native  # noqa: E402

i = sys.argv.index("--")
kv = dict(a.split("=") for a in sys.argv[1:i])
_native.module().set_knobs({k: int(v) for k, v in kv.items()})
sys.argv = sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
