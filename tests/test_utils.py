"""utils: logging formatter, profiling ranges / timers, checkpoint round trip; package imports."""
import importlib

import pytest
import torch


def test_all_subpackages_import():
    import beforeholiday_amd as bh
    for name in bh._SUBMODULES:
        importlib.import_module(f"beforeholiday_amd.{name}")
    for sub in ["contrib.bottleneck", "contrib.clip_grad", "contrib.conv_bias_relu", "contrib.fmha",
                "contrib.focal_loss", "contrib.groupbn", "contrib.index_mul_2d", "contrib.layer_norm",
                "contrib.multihead_attn", "contrib.nccl_p2p", "contrib.optimizers", "contrib.peer_memory",
                "contrib.sparsity", "contrib.transducer", "contrib.xentropy", "transformer.amp",
                "transformer.pipeline_parallel", "transformer.tensor_parallel", "transformer.testing.commons",
                "transformer.testing.standalone_gpt", "transformer.testing.standalone_bert", "transformer._data",
                "transformer.layers", "transformer.microbatches"]:
        importlib.import_module(f"beforeholiday_amd.{sub}")


def test_logging_and_profiling(caplog):
    from beforeholiday_amd.utils import EventTimer, get_logger, profile_range, report_memory
    log = get_logger("beforeholiday_amd.test")
    log.warning("hello")
    with profile_range("region"):
        t = EventTimer().start()
        torch.ones(10).sum()
        t.stop()
    assert t.elapsed_ms() >= 0
    assert "memory" in report_memory("x")


def test_checkpoint_round_trip(tmp_path):
    from beforeholiday_amd.optimizers import FusedAdam
    from beforeholiday_amd.utils import load_checkpoint, save_checkpoint
    m = torch.nn.Linear(4, 3)
    opt = FusedAdam(m.parameters(), lr=0.1)
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    p = save_checkpoint(str(tmp_path / "c.pt"), m, opt, epoch=3)
    m2 = torch.nn.Linear(4, 3)
    opt2 = FusedAdam(m2.parameters(), lr=0.1)
    st = load_checkpoint(p, m2, opt2)
    assert st["epoch"] == 3
    torch.testing.assert_close(m2.weight, m.weight)
    assert opt2.state_dict()["state"].keys() == opt.state_dict()["state"].keys()


def test_install_apex_aliases():
    import sys
    import beforeholiday_amd as bh
    bh.install_apex_aliases()
    import apex  # noqa: F401
    from apex.optimizers import FusedLAMB  # noqa: F401
    assert "amp_C" in sys.modules and "apex_C" in sys.modules


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_pipeline_timers(device, capsys):
    """_Timers: accumulate over start/stop pairs, cut a running interval in elapsed(), reset, log."""
    import time

    from beforeholiday_amd.transformer.pipeline_parallel._timers import _Timers

    if device == "cuda":
        torch.cuda.init()
        x = torch.randn(2048, 2048, device="cuda")
    timers = _Timers()
    t = timers("fwd")
    for _ in range(2):
        t.start()
        if device == "cuda":
            for _ in range(20):
                x = x @ x / 2048
        else:
            time.sleep(0.01)
        t.stop()
    with pytest.raises(RuntimeError):
        t.stop()
    v = t.elapsed(reset=False)
    assert v > (0.015 if device == "cpu" else 0.0)
    assert t.elapsed(reset=True) == pytest.approx(v)
    assert t.elapsed() == 0.0
    t.start()
    assert t.elapsed() >= 0.0 and t.running  # cut and restarted
    t.stop()
    timers("bwd").start()
    timers("bwd").stop()
    timers.log(["fwd", "bwd"])
    assert capsys.readouterr().out.startswith("time (ms) | fwd:")

    class _W:
        def __init__(self):
            self.rows = []

        def add_scalar(self, k, v, it):
            self.rows.append((k, it))

    w = _W()
    timers.write(["fwd"], w, 7)
    assert w.rows == [("fwd-time", 7)]


def test_pipeline_timers_fold_and_sync_mode():
    """Closed intervals are folded once more than _FOLD_AT pile up (the total is unchanged), and the
    sync-mode timers (reference wall-clock semantics) accumulate like the event timers."""
    import time

    from beforeholiday_amd.transformer.pipeline_parallel import _timers as tm

    timers = tm._Timers(sync=True)
    t = timers("step")
    for _ in range(tm._FOLD_AT + 5):
        t.start()
        t.stop()
    assert len(t._done) <= tm._FOLD_AT
    t.start()
    time.sleep(0.005)
    t.stop()
    assert t.elapsed() >= 0.005


@pytest.mark.gpu
def test_pipeline_timer_rejects_cross_stream_stop():
    """An interval started on one stream and stopped on another raises instead of timing nothing."""
    from beforeholiday_amd.transformer.pipeline_parallel._timers import _Timers

    torch.cuda.init()
    t = _Timers()("x")
    t.start()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError, match="across streams"):
            t.stop()
    t.stop()
    assert t.elapsed() >= 0.0
