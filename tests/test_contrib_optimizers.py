"""ZeRO DistributedFusedAdam / DistributedFusedLAMB (gloo CPU ranks) vs single-process optimizers on
the averaged gradient; legacy contrib FusedAdam / FusedSGD / FP16_Optimizer
(reference tests: apex/contrib/test/optimizers/test_dist_adam.py, test_distributed_fused_lamb.py)."""
import pytest
import torch

from tests._dist import run_distributed
from tests.conftest import devices


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 33), torch.nn.Tanh(), torch.nn.Linear(33, 5))


def _data(world, n=8):
    torch.manual_seed(100)
    return torch.randn(world, n, 12), torch.randn(world, n, 5)


def _dist_adam(rank, world, bucket_mb, overlap):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedAdam
    model = _model()
    ref = _model()
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.1, bucket_cap_mb=bucket_mb,
                               overlap_grad_sync=overlap)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1, eps=1e-8)
    X, Y = _data(world)
    for it in range(3):
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(X[rank]), Y[rank])
        loss.backward()
        opt.step()
        ref_opt.zero_grad()
        # reference: gradient of the mean over ranks' losses
        sum(torch.nn.functional.mse_loss(ref(X[r]), Y[r]) for r in range(world)).div(world).backward()
        ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
    # grad norm + clipping path and state dict round trip
    opt.zero_grad()
    torch.nn.functional.mse_loss(model(X[rank]), Y[rank]).backward()
    n = opt.clip_grad_norm(0.01)
    assert torch.isfinite(n).all()
    opt.step()
    sd = opt.state_dict()
    assert (sd is not None) == (rank == 0)
    box = [sd]
    torch.distributed.broadcast_object_list(box, src=0)  # as if every rank torch.load-ed the file
    sd = box[0]
    assert set(sd) == {"gathered_states"} and len(sd["gathered_states"]) == world
    before = [p.detach().clone() for p in model.parameters()]
    opt2 = DistributedFusedAdam(_model(1).parameters(), lr=1e-2, bucket_cap_mb=bucket_mb)
    opt2.load_state_dict(sd)
    assert opt2.state["step"] == opt.state["step"]
    for b1, b2 in zip(opt._buckets, opt2._buckets):
        torch.testing.assert_close(b1.exp_avg, b2.exp_avg)
        torch.testing.assert_close(b1.master, b2.master)
    for p, b in zip(model.parameters(), before):
        torch.testing.assert_close(p.detach(), b)


@pytest.mark.parametrize("bucket_mb,overlap", [(100, True), (0.0005, True), (0.0005, False)])
def test_distributed_fused_adam(bucket_mb, overlap):
    run_distributed(_dist_adam, 2, bucket_mb, overlap)


def _dist_adam_resize(rank, world):
    """Checkpoint written by 2 shards (tiny buckets) loads into 1 shard (one big bucket) and into 2
    shards again; continuing training matches the uninterrupted optimizer (reference format:
    distributed_fused_adam.py:1123-1280, whose own loader needs the same distributed size)."""
    from beforeholiday_amd.contrib.optimizers import DistributedFusedAdam
    X, Y = _data(1)  # identical data on every rank: the averaged gradient equals the local one
    model = _model()
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.1, bucket_cap_mb=0.0005)

    def step(m, o):
        o.zero_grad()
        torch.nn.functional.mse_loss(m(X[0]), Y[0]).backward()
        o.step()

    for _ in range(2):
        step(model, opt)
    box = [opt.state_dict()]
    torch.distributed.broadcast_object_list(box, src=0)
    sd = box[0]
    snapshot = [p.detach().clone() for p in model.parameters()]
    step(model, opt)  # uninterrupted reference
    single = torch.distributed.new_group([rank])
    for group, cap in ((single, 100), (None, 0.0003)):
        m2 = _model(7)
        with torch.no_grad():
            for p, s in zip(m2.parameters(), snapshot):
                p.copy_(s)
        o2 = DistributedFusedAdam(m2.parameters(), lr=5.0, bucket_cap_mb=cap, process_group=group)
        o2.load_state_dict(sd)
        assert o2.param_groups[0]["lr"] == 1e-2 and o2.state["step"] == 2
        step(m2, o2)
        for p, q in zip(m2.parameters(), model.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)


def test_distributed_fused_adam_checkpoint_across_sizes():
    run_distributed(_dist_adam_resize, 2)


def _dist_adam_no_sync(rank, world):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedAdam
    model, ref = _model(), _model()
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, bucket_cap_mb=0.001)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    X, Y = _data(world)
    opt.zero_grad()
    with opt.no_sync():
        torch.nn.functional.mse_loss(model(X[rank][:4]), Y[rank][:4]).backward()
    torch.nn.functional.mse_loss(model(X[rank][4:]), Y[rank][4:]).backward()
    opt.step()
    ref_opt.zero_grad()
    sum(torch.nn.functional.mse_loss(ref(X[r][:4]), Y[r][:4]) + torch.nn.functional.mse_loss(ref(X[r][4:]), Y[r][4:])
        for r in range(world)).div(world).backward()
    ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_distributed_fused_adam_grad_accumulation():
    run_distributed(_dist_adam_no_sync, 2)


def _dist_lamb(rank, world):
    from beforeholiday_amd.contrib.optimizers import DistributedFusedLAMB
    from beforeholiday_amd.optimizers import FusedLAMB
    model, ref = _model(), _model()
    opt = DistributedFusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0,
                               bucket_cap_mb=0.0005)
    ref_opt = FusedLAMB(ref.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0, eps=1e-8)
    X, Y = _data(world)
    for it in range(3):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(X[rank]), Y[rank]).backward()
        opt.step()
        ref_opt.zero_grad()
        sum(torch.nn.functional.mse_loss(ref(X[r]), Y[r]) for r in range(world)).div(world).backward()
        ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_distributed_fused_lamb():
    run_distributed(_dist_lamb, 2)


@pytest.mark.parametrize("device", devices())
def test_legacy_contrib_fused_adam_and_fp16_optimizer(device):
    from beforeholiday_amd.contrib.optimizers import FP16_Optimizer, FusedAdam
    torch.manual_seed(0)
    dtype = torch.float16 if device != "cpu" else torch.float32
    model = torch.nn.Linear(16, 8).to(device, dtype)
    ref = torch.nn.Linear(16, 8).to(device)
    with torch.no_grad():
        ref.weight.copy_(model.weight.float())
        ref.bias.copy_(model.bias.float())
    opt = FP16_Optimizer(FusedAdam(model.parameters(), lr=1e-3), static_loss_scale=128.0, verbose=False)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    x = torch.randn(4, 16, device=device)
    for _ in range(3):
        opt.zero_grad()
        opt.backward(model(x.to(dtype)).float().pow(2).mean())
        opt.step()
        ref_opt.zero_grad()
        ref(x).pow(2).mean().backward()
        ref_opt.step()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(model.weight.float(), ref.weight, rtol=tol, atol=tol)


@pytest.mark.parametrize("device", devices())
def test_legacy_contrib_fused_sgd(device):
    from beforeholiday_amd.contrib.optimizers import FP16_Optimizer, FusedSGD
    torch.manual_seed(0)
    model = torch.nn.Linear(16, 8).to(device)
    ref = torch.nn.Linear(16, 8).to(device)
    ref.load_state_dict(model.state_dict())
    opt = FP16_Optimizer(FusedSGD(model.parameters(), lr=0.1, momentum=0.9), static_loss_scale=4.0, verbose=False)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(4, 16, device=device)
    for _ in range(3):
        opt.zero_grad()
        opt.backward(model(x).pow(2).mean())
        opt.step()
        ref_opt.zero_grad()
        ref(x).pow(2).mean().backward()
        ref_opt.step()
    torch.testing.assert_close(model.weight, ref.weight, rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------------------------------------
# deprecated fused_adam_cuda ops (reference: apex/contrib/csrc/optimizers/fused_adam_cuda.cpp:79-85)
# ------------------------------------------------------------------------------------------------
def _legacy_state(device, n=3000, gdt=torch.float16, seed=0):
    g = torch.Generator().manual_seed(seed)
    p = torch.randn(n, generator=g).to(device)
    m = (torch.randn(n, generator=g) * 0.1).to(device)
    v = (torch.rand(n, generator=g) * 0.01).to(device)
    grad = (torch.randn(n, generator=g) * 64).to(device, gdt)
    return p, m, v, grad


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("copy_dt", [None, torch.float16, torch.uint8])
def test_fused_adam_cuda_adam_matches_reference(mode, copy_dt):
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    args = (1e-3, 0.9, 0.999, 1e-6, 64.0, 3, mode, 1, 0.01)
    p, m, v, g = _legacy_state("cuda")
    rp, rm, rv, rg = (t.cpu().clone() for t in (p, m, v, g))
    pc = torch.empty(0, device="cuda") if copy_dt is None else torch.empty_like(p, dtype=copy_dt)
    rpc = torch.empty(0) if copy_dt is None else torch.empty_like(rp, dtype=copy_dt)
    fac.adam(p, pc, m, v, g, *args)
    fac._ref_adam(rp, rpc, rm, rv, rg, *args)
    for a, b in ((p, rp), (m, rm), (v, rv)):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-6)
    if copy_dt is not None:
        assert torch.equal(pc.cpu(), rpc) if copy_dt == torch.uint8 else torch.allclose(pc.cpu().float(), rpc.float())


@pytest.mark.gpu
def test_fused_adam_cuda_adam_mt_matches_single():
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    args = (1e-3, 0.9, 0.999, 1e-8, 1.0, 5, 1, 1, 0.0)
    sizes = [7, 65536 + 5, 1000]
    single = [_legacy_state("cuda", n, torch.float32, seed=i) for i, n in enumerate(sizes)]
    multi = [tuple(t.clone() for t in s) for s in single]
    outs = [torch.empty_like(s[0], dtype=torch.float16) for s in single]
    for p, m, v, g in single:
        fac.adam(p, torch.empty(0, device="cuda"), m, v, g, *args)
    flag = torch.zeros(1, dtype=torch.int, device="cuda")
    fac.adam_mt(2048, flag, [[s[0] for s in multi], [s[1] for s in multi], [s[2] for s in multi],
                             [s[3] for s in multi], outs], *args)
    for s, t, o in zip(single, multi, outs):
        for a, b in zip(s[:3], t[:3]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
        torch.testing.assert_close(o.float(), t[0].half().float(), rtol=0, atol=0)


@pytest.mark.parametrize("device", devices())
def test_reversible_adam_then_undo_restores_state(device):
    """reversible_adam skips non-finite grads and flags p_copy[0] = inf; maybe_adam_undo then reverts
    the step for every other element (reference kernels :571, :657)."""
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    args = (1e-2, 0.9, 0.999, 1e-8, 8.0, 1, 1, 1, 0.01)
    p, m, v, g = _legacy_state(device, 1024, torch.float32, seed=3)
    g[17] = float("inf")
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    pc = torch.empty_like(p, dtype=torch.float16)
    fac.reversible_adam(p, pc, m, v, g, *args)
    assert torch.isinf(pc[0].float())
    assert p[17] == p0[17] and m[17] == m0[17]
    assert not torch.equal(p, p0)
    flag = torch.zeros(1, dtype=torch.int, device=device)
    fac.strided_check_finite(flag, pc, 1, 1)
    assert int(flag) == 1
    fac.maybe_adam_undo(flag, p, m, v, g, *args)
    torch.testing.assert_close(p, p0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, m0, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(v, v0, rtol=1e-3, atol=1e-7)
    flag.zero_()
    p1 = p.clone()
    fac.maybe_adam_undo(flag, p, m, v, g, *args)  # no overflow -> untouched
    assert torch.equal(p, p1)


@pytest.mark.parametrize("device", devices())
def test_e5m2_casts(device):
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    x = torch.tensor([0.0, 1.0, -1.5, 1.75, 1.8, 3.0e4, -2.0 ** -14, float("inf"), 0.3], device=device)
    b = torch.empty_like(x, dtype=torch.uint8)
    fac.maybe_cast(torch.zeros(1, dtype=torch.int, device=device), x, b)
    back = torch.empty_like(x)
    fac.maybe_cast(None, b, back)
    # e5m2: 2 mantissa bits -> representable 1.0, 1.25, 1.5, 1.75, 2.0 ...
    want = torch.tensor([0.0, 1.0, -1.5, 1.75, 1.75, 28672.0, -2.0 ** -14, float("inf"), 0.3125])
    torch.testing.assert_close(back.cpu(), want, rtol=0, atol=0)
    flag = torch.ones(1, dtype=torch.int, device=device)
    b2 = torch.zeros_like(b)
    fac.maybe_cast(flag, x, b2)  # overflow set -> skipped
    assert int(b2.sum()) == 0
    lists = [[x, x[:3]], [torch.empty_like(x, dtype=torch.float16), torch.empty(3, dtype=torch.float16, device=device)]]
    fac.maybe_cast_mt(2048, torch.zeros(1, dtype=torch.int, device=device), lists)
    torch.testing.assert_close(lists[1][0].float(), x.half().float())


@pytest.mark.gpu
def test_e5m2_gpu_matches_cpu_reference():
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    x = torch.randn(100000) * torch.exp(torch.randn(100000) * 4)
    ref = fac.to_e5m2(x)
    out = torch.empty(100000, dtype=torch.uint8, device="cuda")
    fac.maybe_cast(None, x.cuda(), out)
    assert torch.equal(out.cpu(), ref)


def _dist_lamb_e5m2_and_overflow(rank, world):
    """e5m2 parameter all-gather: the masters follow the uncompressed run exactly after one step and
    the model parameters are their e5m2 rounding; a non-finite gradient on ONE rank skips the step
    everywhere through the device noop flag (reference: distributed_fused_lamb.py e5m2_allgather,
    multi_tensor_distopt_lamb_kernel.cu:109-506)."""
    from beforeholiday_amd.contrib.optimizers import DistributedFusedLAMB
    from beforeholiday_amd.ops import fused_adam_cuda as fac
    X, Y = _data(world)
    runs = {}
    for e5 in (False, True):
        model = _model()
        opt = DistributedFusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0,
                                   bucket_cap_mb=0.0005, e5m2_allgather=e5)
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(X[rank]), Y[rank]).backward()
        opt.step()
        runs[e5] = (model, opt)
    for b0, b1 in zip(runs[False][1]._buckets, runs[True][1]._buckets):
        torch.testing.assert_close(b0.master, b1.master, rtol=0, atol=0)
    for p0, p1 in zip(runs[False][0].parameters(), runs[True][0].parameters()):
        torch.testing.assert_close(p1.detach(), fac.from_e5m2(fac.to_e5m2(p0.detach())), rtol=0, atol=0)
    # overflow on rank 1 only -> both ranks skip
    model, opt = runs[False]
    masters = [b.master.clone() for b in opt._buckets]
    moments = [b.exp_avg.clone() for b in opt._buckets]
    opt.zero_grad()
    loss = torch.nn.functional.mse_loss(model(X[rank]), Y[rank])
    (loss * (float("inf") if rank == 1 else 1.0)).backward()
    opt.step()
    assert int(opt.has_overflow) == 1
    for b, m0, e0 in zip(opt._buckets, masters, moments):
        assert torch.equal(b.master, m0) and torch.equal(b.exp_avg, e0)
    assert int(opt._step_t) == 1
    sd = opt.state_dict()
    assert rank != 0 or sd is not None


def test_distributed_fused_lamb_e5m2_and_overflow_skip():
    run_distributed(_dist_lamb_e5m2_and_overflow, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("copy_dt", [torch.bfloat16, torch.uint8])
def test_distributed_lamb_cuda_stages_match_reference(mode, copy_dt):
    from beforeholiday_amd.ops import distributed_lamb_cuda as dl
    torch.manual_seed(0)
    sizes = [5, 4099, 70000]
    T = len(sizes)

    def make(dev):
        torch.manual_seed(1)
        g = [torch.randn(n).to(dev, torch.float16) * 8 for n in sizes]
        p = [torch.randn(n).to(dev) for n in sizes]
        m = [torch.randn(n).to(dev) * 0.01 for n in sizes]
        v = [torch.rand(n).to(dev) * 0.01 for n in sizes]
        u = [torch.zeros(n, device=dev) for n in sizes]
        c = [torch.empty(n, dtype=copy_dt, device=dev) for n in sizes]
        vec = lambda x, dt=torch.float32: torch.tensor(x, dtype=dt, device=dev)  # noqa: E731
        hp = dict(b1=vec([0.9] * T), b2=vec([0.999] * T), b3=vec([0.1] * T), bc=vec([1, 0, 1], torch.int),
                  step=vec([3], torch.int), eps=vec([1e-6] * T), decay=vec([0.01, 0.0, 0.02]), gs=vec([8.0]),
                  gn=vec([40.0]), lr=vec([1e-2]), off=vec([0, 1, 2], torch.long))
        return [g, p, m, v, u, c], hp

    out = {}
    for dev in ("cuda", "cpu"):
        (g, p, m, v, u, c), hp = make(dev)
        noop = torch.zeros(1, dtype=torch.int, device=dev)
        dl.multi_tensor_lamb_compute_update_term(65536, noop, [g, p, m, v, u], hp["b1"], hp["b2"], hp["b3"], hp["bc"],
                                                 hp["step"], hp["eps"], mode, hp["decay"], hp["gs"], hp["gn"], 1.0)
        pn = torch.stack([t.norm() for t in p])
        un = torch.stack([t.norm() for t in u])
        dl.multi_tensor_lamb_update_weights(65536, noop, [p, u, c], pn, un, hp["off"], hp["lr"], hp["decay"], hp["gn"],
                                            False)
        out[dev] = [t.cpu() for t in p + m + v + u + c]
    for a, b in zip(out["cuda"], out["cpu"]):
        if a.dtype == torch.uint8:
            assert (a.int() - b.int()).abs().max() <= 1
        else:
            torch.testing.assert_close(a.float(), b.float(), rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_distributed_adam_cuda_matches_reference(mode):
    from beforeholiday_amd.ops import distributed_adam_cuda as da
    sizes = [3, 5000, 65537]
    T = len(sizes)
    out = {}
    for dev in ("cuda", "cpu"):
        torch.manual_seed(4)
        p = [torch.randn(n).to(dev) for n in sizes]
        m = [torch.randn(n).to(dev) * 0.01 for n in sizes]
        v = [torch.rand(n).to(dev) * 0.01 for n in sizes]
        g = [(torch.randn(n) * 16).to(dev, torch.float16) for n in sizes]
        c = [torch.empty(n, dtype=torch.float16, device=dev) for n in sizes]
        vec = lambda x, dt=torch.float32: torch.tensor(x, dtype=dt, device=dev)  # noqa: E731
        da.multi_tensor_fused_adam(65536, torch.zeros(1, dtype=torch.int, device=dev), [p, m, v, g, c],
                                   vec([0.9, 0.8, 0.9]), vec([0.999] * T), vec([1, 1, 0], torch.int),
                                   vec([1e-8, 1e-6, 1e-8]), vec([0.0, 0.01, 0.1]), 1e-3, 16.0, 4, mode)
        out[dev] = [t.cpu().float() for t in p + m + v + c]
    for a, b in zip(out["cuda"], out["cpu"]):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-6)
