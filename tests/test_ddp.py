"""DistributedDataParallel / Reducer on gloo world_size=2 (the BASELINE "plumbing" config:
2-layer MLP wrapped in DDP, CPU). Race-style check modelled on
tests/distributed/DDP/ddp_race_condition_test.py: analytic gradient sums every iteration."""
import pytest
import torch
import torch.distributed as dist

from beforeholiday_amd.parallel import DistributedDataParallel as DDP, Reducer

from _dist import run_distributed


class MLP(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = torch.nn.Linear(32, 64)
        self.fc2 = torch.nn.Linear(64, 8)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


def _mlp_ddp(rank, world, kwargs):
    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's params
    model = MLP()
    ddp = DDP(model, **kwargs)
    ref = MLP()
    torch.manual_seed(100)
    ref_state = MLP().state_dict()
    ref.load_state_dict(ref_state)
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    for it in range(4):
        torch.manual_seed(it)
        x = torch.randn(8 * world, 32)
        y = torch.randn(8 * world, 8)
        xs, ys = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
        loss = torch.nn.functional.mse_loss(ddp(xs), ys)
        opt.zero_grad()
        loss.backward()
        # reference: full batch on one process == average of per-rank mean losses
        ref_opt.zero_grad()
        rl = sum(torch.nn.functional.mse_loss(ref(x[r * 8:(r + 1) * 8]), y[r * 8:(r + 1) * 8]) for r in range(world)) / world
        rl.backward()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-6)
        opt.step()
        ref_opt.step()


@pytest.mark.parametrize("kwargs", [
    {},
    {"message_size": 1},
    {"message_size": 100, "num_allreduce_streams": 2},
    {"delay_allreduce": True},
    {"allreduce_always_fp32": True, "gradient_predivide_factor": 2.0},
    {"retain_allreduce_buffers": True, "message_size": 500},
])
def test_ddp_mlp_gloo(kwargs):
    run_distributed(_mlp_ddp, 2, kwargs)


def _race(rank, world):
    # two large params, tiny buckets, trigger params: grads must equal the analytic sum each iter
    a = torch.nn.Parameter(torch.ones(100000))
    b = torch.nn.Parameter(torch.ones(100000))

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a, self.b = a, b

        def forward(self, x):
            return self.a * x, self.b * x

    m = DDP(M(), message_size=1, allreduce_trigger_params=[b], num_allreduce_streams=3)
    for it in range(5):
        x = torch.full((100000,), float(rank + 1 + it))
        ya, yb = m(x)
        a.grad = None
        b.grad = None
        (ya.sum() + yb.sum()).backward()
        expect = sum(r + 1 + it for r in range(world)) / world
        assert torch.all(a.grad == expect), (a.grad[:3], expect)
        assert torch.all(b.grad == expect)


def test_ddp_race_gloo():
    run_distributed(_race, 2)


def _reducer(rank, world):
    torch.manual_seed(rank)
    model = MLP()
    red = Reducer(model)
    x = torch.randn(4, 32) * (rank + 1)
    model(x).sum().backward()
    grads = [p.grad.clone() for p in model.parameters()]
    red.reduce()
    for g, p in zip(grads, model.parameters()):
        tot = g.clone()
        dist.all_reduce(tot)
        torch.testing.assert_close(p.grad, tot / world)


def test_reducer_gloo():
    run_distributed(_reducer, 2)


def _no_sync(rank, world):
    torch.manual_seed(0)
    m = DDP(MLP())
    x = torch.randn(4, 32) * (rank + 1)
    with m.no_sync():
        m(x).sum().backward()
    local = [p.grad.clone() for p in m.parameters()]
    for p in m.parameters():
        p.grad = None
    m(x).sum().backward()
    for g, p in zip(local, m.parameters()):
        tot = g.clone()
        dist.all_reduce(tot)
        torch.testing.assert_close(p.grad, tot / world, rtol=1e-5, atol=1e-6)


def test_ddp_no_sync_gloo():
    run_distributed(_no_sync, 2)


def _amp_master_params(rank, world, opt_level):
    # reference: tests/distributed/amp_master_params/amp_master_params.py:1-71 + compare.py:1-31 —
    # O2 training under DDP, then every rank must hold identical model AND master params, and the
    # fp16 model params must equal the fp32 masters rounded to fp16.
    from beforeholiday_amd import amp
    from beforeholiday_amd.amp._amp_state import _amp_state

    torch.manual_seed(rank)
    model = MLP()
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level=opt_level, verbosity=0)
    ddp = DDP(model, message_size=300)
    for it in range(12):
        torch.manual_seed(1000 * rank + it)
        x, y = torch.randn(8, 32), torch.randn(8, 8)
        loss = torch.nn.functional.mse_loss(ddp(x).float(), y)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
    low = next(model.parameters()).dtype
    for p, m in zip(model.parameters(), amp.master_params(opt)):
        assert m.dtype == torch.float32
        assert torch.equal(p, m.to(low))
        for t in (p.detach().float(), m.detach()):
            gathered = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(gathered, t)
            for g in gathered[1:]:
                assert torch.equal(g, gathered[0])
    assert _amp_state.loss_scalers[0].loss_scale() > 0
    amp.deactivate()


@pytest.mark.parametrize("opt_level", ["O2", "O5"])
def test_amp_master_params_ddp_gloo(opt_level):
    run_distributed(_amp_master_params, 2, opt_level)


def _bucket_view(rank, world):
    """Gradient-as-bucket-view: after the first backward every gradient IS a view of its bucket's flat
    buffer (no gather copy before, no scatter copy after the all-reduce), and stays correct; zeroing
    those view gradients in place (torch, amp and FP16_Optimizer zero_grad) works."""
    from beforeholiday_amd.fp16_utils import FP16_Optimizer
    from beforeholiday_amd.parallel.distributed import grad_is_bucket_view

    torch.manual_seed(100 + rank)
    model = MLP()
    ddp = DDP(model, message_size=1000, gradient_as_bucket_view=True)
    for it in range(3):
        torch.manual_seed(it)
        x = torch.randn(8 * world, 32)
        xs = x[rank * 8:(rank + 1) * 8]
        ddp.zero_grad(set_to_none=it == 0)
        ddp(xs).square().sum().backward()
        flats = {id(b): b.flat for b in ddp._buckets}
        for p in model.parameters():
            assert grad_is_bucket_view(p) and not hasattr(p, "_bh_grad_slot")
            assert any(f.data_ptr() <= p.grad.data_ptr() < f.data_ptr() + f.numel() * f.element_size()
                       for f in flats.values())
        # all ranks hold the same (averaged) gradient
        g = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
        gs = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(gs, g)
        for other in gs:
            torch.testing.assert_close(other, g)
    ddp.zero_grad(set_to_none=False)  # in place on the view gradients: no "can't detach views in-place"
    assert all(p.grad is not None and not p.grad.any() for p in model.parameters())
    ddp(torch.randn(4, 32)).sum().backward()
    fopt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=0.1), static_loss_scale=1.0, verbose=False)
    fopt.zero_grad()  # the reference's default set_grads_to_None=False
    assert all(not p.grad.any() for p in model.parameters())


def test_ddp_gradient_as_bucket_view():
    run_distributed(_bucket_view, 2)


def _default_copies_back(rank, world):
    """Without gradient_as_bucket_view (the default, as in torch) param.grad stays its own tensor and
    receives the average."""
    from beforeholiday_amd.parallel.distributed import grad_is_bucket_view

    torch.manual_seed(rank)
    model = MLP()
    ddp = DDP(model, message_size=1000)
    x = torch.randn(4, 32) * (rank + 1)
    for _ in range(2):
        ddp.zero_grad(set_to_none=True)
        local = []
        out = ddp(x).sum()
        grads = torch.autograd.grad(out, list(model.parameters()), retain_graph=True)
        local = [g.clone() for g in grads]
        out.backward()
        for g, p in zip(local, model.parameters()):
            assert not grad_is_bucket_view(p)
            assert all(p.grad.data_ptr() != b.flat.data_ptr() for b in ddp._buckets)
            tot = g.clone()
            dist.all_reduce(tot)
            torch.testing.assert_close(p.grad, tot / world, rtol=1e-5, atol=1e-6)


def test_ddp_default_copies_back():
    run_distributed(_default_copies_back, 2)


def _amp_accumulate(rank, world, opt_level, view):
    """amp with two ``scale_loss`` micro-batches per step (no delay_unscale) under DDP: the gradient
    stashed after the first micro-batch must survive the second backward, also when it is a bucket view
    (advisor round 3: it was overwritten by the second backward's copy into the slot)."""
    import copy

    from beforeholiday_amd import amp

    torch.manual_seed(0)
    ref = MLP()
    model = copy.deepcopy(ref)
    opt = torch.optim.SGD(model.parameters(), lr=0.0)
    model, opt = amp.initialize(model, opt, opt_level=opt_level, loss_scale=128.0, verbosity=0)
    ddp = DDP(model, message_size=300, gradient_as_bucket_view=view)
    micro = [(torch.randn(4 * world, 32), torch.randn(4 * world, 8)) for _ in range(2)]
    try:
        for step in range(2):
            for x, y in micro:
                xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
                loss = torch.nn.functional.mse_loss(ddp(xs).float(), ys)
                with amp.scale_loss(loss, opt) as scaled:
                    scaled.backward()
            got = [p.grad.float().clone() for p in amp.master_params(opt)]
            opt.zero_grad()
        for p in ref.parameters():
            p.grad = None
        for x, y in micro:  # fp32, one process: the sum over micro-batches of the rank-averaged loss
            sum(torch.nn.functional.mse_loss(ref(x[r * 4:(r + 1) * 4]), y[r * 4:(r + 1) * 4])
                for r in range(world)).div(world).backward()
        for g, q in zip(got, ref.parameters()):
            torch.testing.assert_close(g, q.grad, rtol=3e-2, atol=3e-3)
    finally:
        amp.deactivate()


@pytest.mark.parametrize("opt_level", ["O1", "O2"])
@pytest.mark.parametrize("view", [False, True])
def test_amp_accumulation_under_ddp(opt_level, view):
    run_distributed(_amp_accumulate, 2, opt_level, view)


def test_lr_scheduler_after_scale_loss():
    """A torch LR scheduler built after the first scale_loss (amp has already installed its step gate)
    wraps optimizer.step through ``__func__`` (advisor round 3)."""
    from beforeholiday_amd import amp

    model = MLP()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=0)
    try:
        loss = model(torch.randn(2, 32)).float().sum()
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
        opt.step()
        sched.step()
        assert abs(opt.param_groups[0]["lr"] - 0.05) < 1e-12
    finally:
        amp.deactivate()
