"""The shipped per-shape GEMM solution table (utils/gemm_tuning.py): format, coverage of the
benchmark shapes, and the CPU no-op path. GPU: loading it routes torch.mm through TunableOp
without changing results beyond fp16 rounding."""
import csv
import os

import pytest
import torch

from beforeholiday_amd.utils import gemm_tuning


def _rows():
    with open(gemm_tuning.DEFAULT_TABLE) as f:
        return list(csv.reader(f))


def test_table_has_validators_and_signatures():
    rows = _rows()
    validators = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    for key in ("PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"):
        assert key in validators, key
    assert validators["GCN_ARCH_NAME"].startswith("gfx950")
    sigs = [r for r in rows if r[0] != "Validator"]
    assert len(sigs) >= 40
    for op, params, solution, ms in sigs:
        assert op.startswith(("GemmTunableOp", "GemmAndBiasTunableOp", "GemmStridedBatchedTunableOp")), op
        assert solution == "Default" or solution.startswith(("Gemm_Hipblaslt_", "Gemm_Rocblas_")), solution
        assert float(ms) > 0


def test_table_covers_resnet50_layer2_to_4_1x1_gemms():
    """Every stride-1 1x1 convolution of layers 2-4 at batch 256 (M = pixels) that stays on the library
    GEMM has a tuned fp16 signature (forward NN, data gradient TN, in TunableOp's column-major naming)."""
    params = {r[1] for r in _rows() if r[0].startswith("GemmTunableOp_Half")}
    for M, cin, cout in [(200704, 512, 128), (200704, 128, 512), (50176, 1024, 256), (50176, 256, 1024),
                         (12544, 2048, 512), (12544, 512, 2048)]:
        assert any(f"_{cout}_{M}_{cin}_" in p or f"_{cin}_{M}_{cout}_" in p for p in params), (M, cin, cout)


def test_cpu_is_a_no_op():
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    assert gemm_tuning.enable_tuned_gemms() is False
    assert gemm_tuning.setup("auto") is False
    assert gemm_tuning.status() == {"enabled": False}


@pytest.mark.gpu
def test_loaded_table_keeps_mm_results(tmp_path):
    assert gemm_tuning.enable_tuned_gemms()
    try:
        a = torch.randn(200704 // 16, 512, device="cuda", dtype=torch.float16)
        b = torch.randn(128, 512, device="cuda", dtype=torch.float16)
        ref = a.float() @ b.float().t()
        out = torch.mm(a, b.t()).float()
        assert float((out - ref).abs().max() / ref.abs().max()) < 2e-3
        assert gemm_tuning.status()["enabled"]
        path = os.path.join(tmp_path, "t.csv")
        n = gemm_tuning.write_table(path)
        assert n >= 40 and os.path.getsize(path) > 0
    finally:
        torch.cuda.tunable.enable(False)
