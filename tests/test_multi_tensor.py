"""multi-tensor apply ops: GPU kernels vs the fp32 PyTorch reference, CPU reference vs torch.

Modelled on the reference's tests/L0/run_amp/test_multi_tensor_{scale,axpby,l2norm}.py: sizes that
straddle chunk boundaries, repeated tensors, dtype cross products and Inf/NaN injection.
"""
import math

import pytest
import torch

from beforeholiday_amd.ops import amp_C
from beforeholiday_amd.ops._ref import multi_tensor as ref

SIZES = [1, 7, 8, 9, 1023, 16384, 16385, 33331, 65536 + 9, 130001]
CHUNKS = [16384, 2048 * 32, 333 * 8]


def _lists(n_lists, dtypes, device, sizes=SIZES, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for li in range(n_lists):
        dt = dtypes[li] if isinstance(dtypes, (list, tuple)) else dtypes
        out.append([(torch.randn(s, generator=g) * scale).to(dt).to(device) for s in sizes])
    return out


def _clone(lists, device="cpu"):
    return [[t.detach().clone().to(device) for t in l] for l in lists]


def _assert_lists_close(a, b, rtol, atol):
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            torch.testing.assert_close(u.float().cpu(), v.float().cpu(), rtol=rtol, atol=atol)


# ------------------------------------------------------------------------------ CPU reference


def test_ref_scale_and_flag():
    ins, outs = _lists(2, torch.float32, "cpu")
    noop = torch.zeros(1, dtype=torch.int)
    ref.multi_tensor_scale(16384, noop, [ins, outs], 0.5)
    assert int(noop) == 0
    for i, o in zip(ins, outs):
        torch.testing.assert_close(o, i * 0.5)
    ins[3][5] = float("inf")
    ref.multi_tensor_scale(16384, noop, [ins, outs], 0.5)
    assert int(noop) == 1


def test_ref_l2norm_matches_torch():
    (xs,) = _lists(1, torch.float32, "cpu")
    noop = torch.zeros(1, dtype=torch.int)
    tot, per = ref.multi_tensor_l2norm(65536, noop, [xs], True)
    expect = torch.cat([x.reshape(-1) for x in xs]).norm()
    torch.testing.assert_close(tot[0], expect, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(per, torch.stack([x.norm() for x in xs]), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------ GPU kernels

DT = [torch.float32, torch.float16, torch.bfloat16]
TOL = {torch.float32: (1e-6, 1e-6), torch.float16: (1e-3, 1e-3), torch.bfloat16: (1e-2, 1e-2),
       torch.float64: (1e-6, 1e-6)}


@pytest.mark.gpu
@pytest.mark.parametrize("din", DT)
@pytest.mark.parametrize("dout", DT)
@pytest.mark.parametrize("chunk", CHUNKS)
def test_scale_gpu(din, dout, chunk):
    ins, = _lists(1, din, "cuda")
    outs = [torch.empty_like(x, dtype=dout) for x in ins]
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    amp_C.multi_tensor_scale(chunk, noop, [ins, outs], 4.0)
    torch.cuda.synchronize()
    assert int(noop.item()) == 0
    for i, o in zip(ins, outs):
        torch.testing.assert_close(o.float(), (i.float() * 4.0).to(dout).float(), rtol=TOL[dout][0], atol=TOL[dout][1])


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["first", "middle", "last"])
@pytest.mark.parametrize("val", [float("inf"), float("nan")])
def test_scale_overflow_flag_gpu(where, val):
    ins, = _lists(1, torch.float16, "cuda")
    t = ins[-1]
    idx = {"first": 0, "middle": t.numel() // 2, "last": t.numel() - 1}[where]
    t[idx] = val
    outs = [torch.empty_like(x, dtype=torch.float32) for x in ins]
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    amp_C.multi_tensor_scale(16384, noop, [ins, outs], 1.0)
    assert int(noop.item()) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("dx,dy,do", [(torch.float32,) * 3, (torch.float16, torch.float32, torch.float16),
                                      (torch.bfloat16, torch.bfloat16, torch.float32)])
@pytest.mark.parametrize("check", [-1, 0, 1])
def test_axpby_gpu(dx, dy, do, check):
    xs, ys = _lists(2, [dx, dy], "cuda")
    outs = [torch.empty_like(x, dtype=do) for x in xs]
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    amp_C.multi_tensor_axpby(16384, noop, [xs, ys, outs], 2.0, -0.5, check)
    assert int(noop.item()) == 0
    for x, y, o in zip(xs, ys, outs):
        torch.testing.assert_close(o.float(), (2.0 * x.float() - 0.5 * y.float()).to(do).float(),
                                   rtol=TOL[do][0], atol=TOL[do][1])
    ys[2][0] = float("inf")
    amp_C.multi_tensor_axpby(16384, noop, [xs, ys, outs], 2.0, -0.5, check)
    assert int(noop.item()) == (0 if check == 0 else 1)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DT + [torch.float64])
@pytest.mark.parametrize("chunk", CHUNKS)
@pytest.mark.parametrize("per_tensor", [False, True])
def test_l2norm_gpu(dt, chunk, per_tensor):
    xs, = _lists(1, dt, "cuda", sizes=SIZES * 3)
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    tot, per = amp_C.multi_tensor_l2norm(chunk, noop, [xs], per_tensor)
    exp_per = torch.stack([x.double().norm() for x in xs])
    torch.testing.assert_close(tot.double()[0], exp_per.norm(), rtol=1e-5, atol=1e-5)
    if per_tensor:
        torch.testing.assert_close(per.double(), exp_per, rtol=1e-5, atol=1e-5)
    else:
        assert per.numel() == 0
    xs[1][0] = float("nan")
    amp_C.multi_tensor_l2norm(chunk, noop, [xs], per_tensor)
    assert int(noop.item()) == 1


@pytest.mark.gpu
def test_l2norm_mp_skips_on_flag_gpu():
    xs, = _lists(1, torch.float32, "cuda")
    noop = torch.ones(1, dtype=torch.int, device="cuda")
    tot, per = amp_C.multi_tensor_l2norm_mp(65536, noop, [xs], True)
    assert float(tot.item()) == 0.0 and float(per.abs().sum()) == 0.0
    noop.zero_()
    tot, per = amp_C.multi_tensor_l2norm_mp(65536, noop, [xs], True)
    torch.testing.assert_close(tot[0], torch.cat(xs).norm(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_l2norm_scale_gpu():
    xs, = _lists(1, torch.float16, "cuda")
    outs = [torch.empty_like(x, dtype=torch.float32) for x in xs]
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    tot, per = amp_C.multi_tensor_l2norm_scale(65536, noop, [xs, outs], 0.25, True)
    torch.testing.assert_close(tot[0], torch.cat([x.float() for x in xs]).norm(), rtol=1e-5, atol=1e-4)
    for x, o in zip(xs, outs):
        torch.testing.assert_close(o, x.float() * 0.25)


def _run_both(fn_name, lists_gpu, *args, chunk=16384, rtol=1e-5, atol=1e-6, flag=0, **kw):
    """Run the op on GPU (native) and on CPU copies (reference), compare every list."""
    lists_cpu = _clone(lists_gpu)
    conv = lambda a: a.cpu() if isinstance(a, torch.Tensor) else a
    noop_g = torch.full((1,), flag, dtype=torch.int, device="cuda")
    noop_c = torch.full((1,), flag, dtype=torch.int)
    rg = getattr(amp_C, fn_name)(chunk, noop_g, lists_gpu, *args, **kw)
    rc = getattr(ref, fn_name)(chunk, noop_c, lists_cpu, *[conv(a) for a in args],
                               **{k: conv(v) for k, v in kw.items()})
    torch.cuda.synchronize()
    _assert_lists_close(lists_gpu, lists_cpu, rtol, atol)
    return rg, rc


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("mode", [0, 1])
def test_adam_gpu(dt, mode):
    g, p, m, v = _lists(4, dt, "cuda", seed=1)
    v = [x.abs() for x in v]
    tol = TOL[dt]
    _run_both("multi_tensor_adam", [g, p, m, v], 1e-3, 0.9, 0.999, 1e-8, 3, mode, 1, 0.01,
              rtol=tol[0], atol=tol[1])


@pytest.mark.gpu
@pytest.mark.parametrize("gdt", [torch.float16, torch.bfloat16])
def test_adam_master_copy_gpu(gdt):
    g, = _lists(1, gdt, "cuda", seed=2)
    p, m, v = _lists(3, torch.float32, "cuda", seed=3)
    v = [x.abs() for x in v]
    cp = [x.to(gdt) for x in p]
    _run_both("multi_tensor_adam", [g, p, m, v, cp], 1e-3, 0.9, 0.999, 1e-8, 1, 1, 1, 0.0,
              rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("nesterov,first_run,wd_after", [(False, True, False), (True, False, False),
                                                         (False, False, True)])
@pytest.mark.parametrize("copy", [False, True])
def test_sgd_gpu(nesterov, first_run, wd_after, copy):
    g, = _lists(1, torch.float16 if copy else torch.float32, "cuda", seed=4)
    p, mom = _lists(2, torch.float32, "cuda", seed=5)
    lists = [g, p, mom] + ([[x.half() for x in p]] if copy else [])
    _run_both("multi_tensor_sgd", lists, 1e-4, 0.9, 0.0, 0.1, nesterov, first_run, wd_after, 0.5,
              rtol=1e-3 if copy else 1e-5, atol=1e-3 if copy else 1e-6)


@pytest.mark.gpu
def test_sgd_noop_skips_gpu():
    g, p, mom = _lists(3, torch.float32, "cuda", seed=6)
    p0 = [x.clone() for x in p]
    noop = torch.ones(1, dtype=torch.int, device="cuda")
    amp_C.multi_tensor_sgd(16384, noop, [g, p, mom], 0.0, 0.9, 0.0, 0.1, False, False, False, 1.0)
    for a, b in zip(p, p0):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("mode,nvlamb,decay", [(1, False, 0.01), (0, False, 0.01), (1, True, 0.0), (1, False, 0.0)])
@pytest.mark.parametrize("gnorm", [0.5, 5.0])
def test_lamb_gpu(dt, mode, nvlamb, decay, gnorm):
    g, p, m, v = _lists(4, dt, "cuda", seed=7)
    v = [x.abs() for x in v]
    gn = torch.tensor([gnorm], device="cuda")
    # trust ratios come from norms summed in a different order: allow 1-2 ulp flips in 16-bit
    tol = {torch.float32: (2e-5, 2e-5), torch.float16: (4e-3, 4e-3), torch.bfloat16: (2e-2, 2e-2)}[dt]
    _run_both("multi_tensor_lamb", [g, p, m, v], 1e-2, 0.9, 0.999, 1e-6, 2, 1, decay, 1, mode, gn, 1.0, nvlamb,
              rtol=tol[0], atol=tol[1])


@pytest.mark.gpu
@pytest.mark.parametrize("skip", [0.0, 1.0])
def test_lamb_mp_gpu(skip):
    g, = _lists(1, torch.float16, "cuda", seed=8)
    p, m, v = _lists(3, torch.float32, "cuda", seed=9)
    v = [x.abs() for x in v]
    half = [x.half() for x in p]
    dev = "cuda"
    args = (torch.tensor([1e-2], device=dev), 0.9, 0.999, 1e-6, torch.tensor([3], dtype=torch.int, device=dev), 1,
            0.01, 1, 1, torch.tensor([4.0], device=dev), torch.tensor([2.0], device=dev), False,
            torch.tensor([skip], device=dev), torch.tensor([0.5], device=dev))
    _run_both("multi_tensor_lamb_mp", [g, p, m, v, half], *args, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("norm_type", [0, 2])
@pytest.mark.parametrize("mode", [0, 1])
def test_novograd_gpu(norm_type, mode):
    g, p, m = _lists(3, torch.float32, "cuda", seed=10)
    norms = torch.rand(len(g), device="cuda") + 0.5
    norms_c = norms.cpu().clone()
    lists_c = _clone([g, p, m])
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    amp_C.multi_tensor_novograd(16384, noop, [g, p, m], norms, 1e-2, 0.95, 0.98, 1e-8, 2, 1, 0.001, 1, mode, norm_type)
    ref.multi_tensor_novograd(16384, noop.cpu(), lists_c, norms_c, 1e-2, 0.95, 0.98, 1e-8, 2, 1, 0.001, 1, mode, norm_type)
    torch.testing.assert_close(norms.cpu(), norms_c, rtol=1e-5, atol=1e-5)
    _assert_lists_close([g, p, m], lists_c, 1e-5, 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_adagrad_gpu(mode):
    g, p, h = _lists(3, torch.float32, "cuda", seed=11)
    h = [x.abs() for x in h]
    _run_both("multi_tensor_adagrad", [g, p, h], 1e-2, 1e-10, mode, 0.01)


@pytest.mark.gpu
@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("skipped", [False, True])
def test_lars_gpu(nesterov, skipped):
    g, p, mom = _lists(3, torch.float32, "cuda", seed=12)
    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    gn = amp_C.multi_tensor_l2norm(65536, noop, [g], True)[1]
    pn = amp_C.multi_tensor_l2norm(65536, noop, [p], True)[1]
    _run_both("multi_tensor_lars", [g, p, mom], gn, pn, 0.1, 0.001, 0.0, 1e-4, 0.9, 0.0, nesterov, False,
              False, 1.0, skipped)


@pytest.mark.gpu
def test_empty_and_plan_cache_gpu():
    from beforeholiday_amd._native import submodule

    noop = torch.zeros(1, dtype=torch.int, device="cuda")
    tot, per = amp_C.multi_tensor_l2norm(65536, noop, [[torch.empty(0, device="cuda")]], True)
    assert float(tot.item()) == 0.0
    xs, = _lists(1, torch.float32, "cuda")
    n0 = submodule("amp_C").plan_cache_size()
    for _ in range(3):
        amp_C.multi_tensor_l2norm(65536, noop, [xs], False)
    assert submodule("amp_C").plan_cache_size() == n0 + 1


@pytest.mark.gpu
def test_native_module_is_loaded_gpu():
    import sys

    import beforeholiday_amd._native as nat

    assert nat.available(), nat.import_error()
    assert "beforeholiday_amd._C" in sys.modules
