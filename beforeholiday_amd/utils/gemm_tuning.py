"""Per-shape hipBLASLt / rocBLAS solution choice for the library GEMMs that stay on the hot path.

The 1x1 convolutions of ResNet-50's layers 2-4 (and their data gradients) run as plain library GEMMs
on the ``[pixels, channels]`` view of the NHWC activation (models/resnet.py). hipBLASLt's default
heuristic picks tiles such as 256x256 for ``M = 200704, N = 128`` -- half of every tile is padding --
and reaches 250-430 TFLOP/s on shapes whose HBM bound is 2-4x higher. PyTorch's TunableOp can time
every hipBLASLt / rocBLAS solution of a GEMM signature and keep the fastest; this module runs that
search OFFLINE (``scripts/tune_gemms.py`` on an MI355X, once per library version) and ships the result
as a CSV next to this file, so a training run only LOADS the table (no timing on its first step).

TunableOp rejects a table whose validator lines (PyTorch / ROCm / hipBLASLt / rocBLAS versions) do
not match the running libraries; the GEMMs then take the default heuristic, so a stale table costs
speed, never correctness. Signatures absent from the table also take the default.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_TABLE = os.path.join(_HERE, "tuned", "tunableop_gfx950.csv")


def _tunable():
    import torch.cuda.tunable as tunable

    return tunable


def table_path(path: Optional[str] = None) -> str:
    from .. import config

    return path or config.get().gemm_table or DEFAULT_TABLE


def enable_tuned_gemms(path: Optional[str] = None, tune: bool = False, max_tuning_ms: int = 20,
                       max_tuning_iters: int = 40) -> bool:
    """Route torch's GEMMs through TunableOp with the shipped per-shape table. ``tune=True`` also times
    every solution of each new signature (seconds per shape: tuning runs only, see
    scripts/tune_gemms.py). Returns whether TunableOp is active (False without ROCm or a table)."""
    if not torch.cuda.is_available() or torch.version.hip is None:
        return False
    path = table_path(path)
    if not tune and not os.path.exists(path):
        return False
    t = _tunable()
    t.enable(True)
    t.tuning_enable(tune)
    t.record_untuned_enable(False)
    if tune:
        t.set_max_tuning_duration(max_tuning_ms)
        t.set_max_tuning_iterations(max_tuning_iters)
    # one shared table for every rank (the device ordinal is not part of the name)
    t.set_filename(path, False)
    if os.path.exists(path):
        t.read_file(path)
    return True


def write_table(path: Optional[str] = None) -> int:
    """Write the validators and every tuned signature of this process to ``path`` (TunableOp's CSV
    format); returns the number of signatures."""
    t = _tunable()
    path = table_path(path)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    rows = list(t.get_results())
    with open(path, "w") as f:
        for key, val in t.get_validators():
            f.write(f"Validator,{key},{val}\n")
        for op, params, solution, ms in rows:
            f.write(f"{op},{params},{solution},{float(ms):.6f}\n")
    return len(rows)


def status() -> dict:
    """Diagnostics for bench output: whether TunableOp is on and how many signatures it holds."""
    if not torch.cuda.is_available() or torch.version.hip is None:
        return {"enabled": False}
    t = _tunable()
    return {"enabled": bool(t.is_enabled()), "tuning": bool(t.tuning_is_enabled()),
            "signatures": len(list(t.get_results())) if t.is_enabled() else 0}


def add_argument(ap) -> None:
    """The ``--gemm-table {auto,off,tune}`` option shared by bench.py and benchmarks/*.py."""
    ap.add_argument("--gemm-table", default="auto", choices=["auto", "off", "tune"],
                    help="library GEMMs: auto loads the shipped per-shape hipBLASLt / rocBLAS solution table "
                         "(utils/gemm_tuning.py), tune times every solution of each new shape and rewrites the "
                         "table (offline only), off keeps hipBLASLt's default heuristic")


def setup(mode: str) -> bool:
    """Apply ``--gemm-table``; call before the first GEMM. Returns whether a table is in use."""
    return mode != "off" and enable_tuned_gemms(tune=mode == "tune")


def finish(mode: str, rank: int = 0) -> None:
    """After a ``--gemm-table tune`` run, rank 0 writes the merged table (shipped + new signatures)."""
    if mode == "tune" and rank == 0:
        import sys

        n = write_table()
        print(f"[gemm-table] wrote {n} tuned GEMM signatures to {table_path()}", file=sys.stderr, flush=True)
