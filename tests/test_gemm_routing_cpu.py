"""CPU checks of the GEMM routing helpers (the GPU paths are covered by the gpu-marked tests):
``ops.fused_dense.weight_grad`` falls back to ``dY^T @ X`` off the GPU, the ResNet 1x1 own-GEMM
kind switch parses its setting, ``_tr`` transposes, and ``ops.conv_bn.gemm_bn`` on CPU matches the
fp32 reference with a residual."""
import pytest
import torch

from beforeholiday_amd.models import resnet as R
from beforeholiday_amd.ops import conv_bn
from beforeholiday_amd.ops import fused_dense as fd


def test_weight_grad_cpu_fallback():
    torch.manual_seed(0)
    dy, x = torch.randn(64, 24), torch.randn(64, 40)
    torch.testing.assert_close(fd.weight_grad(dy, x), dy.t() @ x)


@pytest.mark.parametrize("setting,kinds", [("all", {"fwd", "bwd", "plain", "resid"}), ("1", {"fwd", "bwd", "plain", "resid"}),
                                           ("none", set()), ("0", set()), ("fwd,plain", {"fwd", "plain"}),
                                           (" bwd ", {"bwd"})])
def test_own_gemm_kinds(setting, kinds):
    from beforeholiday_amd import config

    c = config.Config.from_env({"BH_OWN_GEMM": setting})
    with config.override(own_gemm=c.own_gemm):
        assert R._OWN_GEMM_KINDS == kinds and R._OWN_GEMM == bool(kinds)


def test_own_gemm_kinds_rejects_unknown():
    from beforeholiday_amd import config

    with pytest.raises(ValueError):
        config.Config.from_env({"BH_OWN_GEMM": "fwd,bogus"})


def test_tr_cpu():
    t = torch.randn(16, 24)
    assert torch.equal(R._tr(t), t.t().contiguous())


def test_gemm_bn_cpu_plain_resid_and_bwd():
    torch.manual_seed(1)
    a, b, r = torch.randn(32, 16), torch.randn(8, 16), torch.randn(32, 8)
    c, part = conv_bn.gemm_bn(a, b, "plain", resid=r)
    assert part is None
    torch.testing.assert_close(c, a @ b.t() + r)
    y = torch.randn(32, 8)
    sc, sh, mu = torch.rand(8) + 0.5, torch.randn(8), torch.randn(8)
    c2, p2 = conv_bn.gemm_bn(a, b, "bwd", by=y, bscale=sc, bshift=sh, bmean=mu)
    dz = c2 * ((y * sc + sh) > 0).float()
    torch.testing.assert_close(conv_bn.sum_parts(p2), torch.cat([dz.sum(0), (dz * (y - mu)).sum(0)]))
