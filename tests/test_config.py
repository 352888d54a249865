"""The typed run-time configuration (beforeholiday_amd/config.py): parsing and validation of the
environment, overrides, module globals refreshed on change, native knobs pushed to the extension, and
the cross-rank agreement check (2 gloo ranks: equal passes, a differing rank raises)."""
import dataclasses

import pytest

from beforeholiday_amd import config
from tests._dist import run_distributed


def test_from_env_parses_and_validates():
    c = config.Config.from_env({"BH_FOLD_BN": "0", "BH_DS_FOLD": "all", "BH_GEMM_TILE": "4", "BH_OWN_GEMM": "all",
                                "BH_BN_RES_FOLD": "0", "BH_MASK_PRODUCER": "1"})
    assert c.fold_bn is False and c.ds_fold == "all" and c.gemm_tile == 4
    assert c.own_gemm == "fwd,bwd,plain,resid" and c.bn_res_fold == "off" and c.mask_producer == "any"
    assert config.Config.from_env({}) == config.Config()
    with pytest.raises(ValueError):
        config.Config.from_env({"BH_DS_FOLD": "sometimes"})
    with pytest.raises(ValueError):
        config.Config.from_env({"BH_FOLD_BN": "maybe"})
    with pytest.raises(ValueError):
        config.Config(own_gemm="fwd,oops")
    with pytest.raises(TypeError):
        config.Config(gemm_tile=True)
    assert config.Config().native_knobs() == {"dense_wgrad": 1, "dense_mfma": 1, "dense_tune": 0, "gemm_tile": 0,
                                             "conv3x3_nb": 2, "conv3x3_sw": 0, "ln_bwd_fused": 0, "igemm_lds": 0, "gemm_log": 0}


def test_set_override_and_module_globals():
    import beforeholiday_amd.amp._process_optimizer as po
    import beforeholiday_amd.models.resnet as R

    base = config.get()
    with config.override(ds_fold="off", bn_res_fold="all", mask_producer="fast", amp_fused_master_step=True):
        assert R._DS_FOLD is False and R._BN_RES_FOLD == "all"
        assert R._MASK_PRODUCER and not R._MASK_PRODUCER_ANY
        assert po.fused_master_step is True
        assert config.get().digest() != base.digest()
    assert config.get() == base and R._DS_FOLD is True and po.fused_master_step is False
    with pytest.raises(ValueError):
        config.set(fold_apply="sideways")
    assert config.get() == base


def test_native_knobs_pushed():
    from beforeholiday_amd import _native

    if not _native.available() or not hasattr(_native.module(), "get_knob"):
        pytest.skip("native extension not built")
    mod = _native.module()
    config.set(gemm_log=True, dense_mfma=False)
    assert mod.get_knob("gemm_log", 0) == 1 and mod.get_knob("dense_mfma", 1) == 0
    config.set(gemm_log=False, dense_mfma=True)
    assert mod.get_knob("gemm_log", 1) == 0 and mod.get_knob("dense_mfma", 0) == 1


def _ranks(rank, world):
    import torch.distributed as dist

    d = config.check_ranks()
    assert d == config.get().digest()
    if rank == 1:
        config.set(fold_apply="none")
    try:
        config.check_ranks()
    except RuntimeError as e:
        assert "differs between ranks" in str(e)
    else:
        raise AssertionError("a differing rank must raise")
    dist.barrier()


def test_check_ranks_two_gloo_ranks():
    run_distributed(_ranks, 2)


def test_digest_ignores_diagnostics_and_table_path(tmp_path):
    """a rank that only turns GEMM logging on, or reads the same GEMM table from another
    path, computes the same numbers and must pass check_ranks; a different table must not."""
    base = config.Config()
    assert dataclasses.replace(base, gemm_log=True).digest() == base.digest()
    a, b, c = tmp_path / "a.csv", tmp_path / "sub_b.csv", tmp_path / "c.csv"
    a.write_text("Validator,x\nGemm,1\n")
    b.write_text("Validator,x\nGemm,1\n")
    c.write_text("Validator,x\nGemm,2\n")
    da, db, dc = (dataclasses.replace(base, gemm_table=str(p)).digest() for p in (a, b, c))
    assert da == db and da != dc
    assert dataclasses.replace(base, fold_apply="none").digest() != base.digest()


def test_python_scaler_flag_follows_config():
    from beforeholiday_amd.amp.scaler import LossScaler

    with config.override(amp_python_scaler=True):
        assert LossScaler.has_fused_kernel is False
    assert LossScaler.has_fused_kernel is (not config.get().amp_python_scaler)
