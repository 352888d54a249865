"""L1 cross-product (reference: tests/L1/common/run_test.sh + compare.py): train the same model
under opt level x loss scale x keep-batchnorm, once with the fused multi-tensor unscale
(``--has-ext``) and once with the per-tensor python scaler, and require IDENTICAL loss
trajectories. CPU: a tiny conv net; GPU: the bottleneck ResNet through MIOpen + the HIP kernels."""
import importlib.util
import itertools
import os

import pytest
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(_ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


main_amp = _load("examples/imagenet/main_amp.py", "bh_main_amp")
compare = _load("tests/L1/compare.py", "bh_l1_compare")

LOSS_SCALES = [None, "1.0", "128.0", "dynamic"]
KEEP_BN = [None, "True", "False"]


def _configs(levels):
    for o, ls, kb in itertools.product(levels, LOSS_SCALES, KEEP_BN):
        if o in ("O1", "O4") and kb is not None:
            continue  # the reference skips keep-batchnorm with O1 (it is implied)
        yield o, ls, kb


def _run(out, o, ls, kb, ext, common):
    argv = common + ["--opt-level", o, "--out-dir", str(out), "--quiet", "--deterministic"]
    if ls is not None:
        argv += ["--loss-scale", ls]
    if kb is not None:
        argv += ["--keep-batchnorm-fp32", kb]
    if ext:
        argv.append("--has-ext")
    return main_amp.run(argv)


@pytest.mark.parametrize("opt_level", ["O0", "O2", "O3", "O5"])
def test_l1_cross_product_cpu(tmp_path, opt_level):
    common = ["-a", "tiny", "--device", "cpu", "-b", "8", "--image-size", "16", "--synthetic-images", "32",
              "--num-classes", "10", "--prints-to-process", "3", "--lr", "0.4"]
    for o, ls, kb in _configs([opt_level]):
        for ext in (True, False):
            rec = _run(tmp_path, o, ls, kb, ext, common)
            assert len(rec["Loss"]) == 3
        le, lp = compare.compare(str(tmp_path), o, ls, kb)
        assert all(torch.isfinite(torch.tensor(le)))


def test_l1_loss_scale_1_vs_dynamic_differ_only_by_scale(tmp_path):
    """O0 with any loss scale is the same fp32 computation up to rounding of the scale product."""
    common = ["-a", "tiny", "--device", "cpu", "-b", "8", "--image-size", "16", "--synthetic-images", "32",
              "--num-classes", "10", "--prints-to-process", "3"]
    a = _run(tmp_path, "O0", "1.0", None, True, common)["Loss"]
    b = _run(tmp_path, "O0", "128.0", None, True, common)["Loss"]
    torch.testing.assert_close(torch.tensor(a), torch.tensor(b), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("opt_level", ["O0", "O1", "O2", "O3", "O4", "O5"])
def test_l1_cross_product_gpu(tmp_path, opt_level):
    common = ["-a", "resnet18_like", "--device", "cuda", "-b", "32", "--image-size", "64",
              "--synthetic-images", "192", "--num-classes", "100", "--prints-to-process", "4"]
    for o, ls, kb in _configs([opt_level]):
        for ext in (True, False):
            _run(tmp_path, o, ls, kb, ext, common)
        le, _ = compare.compare(str(tmp_path), o, ls, kb)
        assert all(torch.isfinite(torch.tensor(le))), (o, ls, kb, le)


def test_dcgan_example_multiple_losses_cpu():
    dcgan = _load("examples/dcgan/main_amp.py", "bh_dcgan")
    hist = dcgan.run(["--device", "cpu", "--opt_level", "O0", "--iters", "2", "--batchSize", "4", "--ngf", "8",
                      "--ndf", "8"])
    assert len(hist) == 2 and all(torch.isfinite(torch.tensor(hist)).flatten())


def test_simple_ddp_example_two_ranks_gloo():
    import subprocess
    import sys
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29547", os.path.join(_ROOT, "examples/simple/distributed/distributed_data_parallel.py"),
           "--backend", "gloo", "--device", "cpu", "--opt-level", "O0", "--steps", "10"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "final loss" in r.stdout


@pytest.mark.gpu
def test_dcgan_example_o1_gpu():
    dcgan = _load("examples/dcgan/main_amp.py", "bh_dcgan_gpu")
    hist = dcgan.run(["--device", "cuda", "--opt_level", "O1", "--iters", "3", "--batchSize", "16", "--fused-adam"])
    assert len(hist) == 3 and all(torch.isfinite(torch.tensor(hist)).flatten())
