"""Locate the first non-repeatable op of the fused ResNet forward: run the same forward twice and
compare every op output (the autograd Functions of models/resnet.py, SyncBatchNorm.forward_from_stats,
nn.Conv2d / nn.Linear forwards) in call order."""
import sys

import torch

sys.path.insert(0, ".")
from beforeholiday_amd.models import resnet as R  # noqa: E402
from beforeholiday_amd.parallel import SyncBatchNorm  # noqa: E402

LOG = []


def _flat(o):
    if torch.is_tensor(o):
        return [o]
    if isinstance(o, (tuple, list)):
        return [t for x in o for t in _flat(x)]
    return []


def wrap_fn(cls):
    orig = cls.apply

    def apply(*a, **k):
        out = orig(*a, **k)
        LOG.append((cls.__name__, [t.detach().clone() for t in _flat(out)]))
        return out
    cls.apply = apply


for name in ("_Conv1DsFn", "_Conv1x1BNFn", "_BNConvFn", "_Conv3x3BNFn", "_StemStatsFn", "_GlobalAvgPoolFn"):
    wrap_fn(getattr(R, name))


def wrap_method(cls, meth):
    orig = getattr(cls, meth)

    def f(self, *a, **k):
        out = orig(self, *a, **k)
        LOG.append((f"{cls.__name__}.{meth}", [t.detach().clone() for t in _flat(out)]))
        return out
    setattr(cls, meth, f)


wrap_method(SyncBatchNorm, "forward_from_stats")
wrap_method(SyncBatchNorm, "forward")
wrap_method(torch.nn.Conv2d, "forward")
wrap_method(torch.nn.Linear, "forward")

torch.manual_seed(0)
net = R.resnet50_fused(layers=(1, 1, 1, 1), num_classes=10).cuda().to(memory_format=torch.channels_last).half()
for m in net.modules():
    if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
        m.float()
state = {k: v.clone() for k, v in net.state_dict().items()}
torch.manual_seed(11)
import os
B = int(os.environ.get("DIAG_BATCH", "16"))
x = torch.randn(B, 3, 224, 224, device="cuda").half().contiguous(memory_format=torch.channels_last)
def poison(fill):
    """Fill the caching allocator's free blocks with ``fill`` (grab them with tensors of decreasing
    size, write, release): an op that reads memory it never wrote then sees other values."""
    held = []
    free = torch.cuda.memory_reserved() - torch.cuda.memory_allocated()
    size = 1 << 30
    while size >= 512 and free > 0:
        try:
            t = torch.empty(size // 4, dtype=torch.float32, device="cuda")
        except RuntimeError:
            size //= 2
            continue
        if torch.cuda.memory_reserved() - torch.cuda.memory_allocated() < 0:
            break
        t.fill_(fill)
        held.append(t)
        free -= size
        if torch.cuda.memory_reserved() - torch.cuda.memory_allocated() < size:
            size //= 2
    del held
    torch.cuda.synchronize()


REPS = int(os.environ.get("DIAG_REPS", "3"))
pre = os.environ.get("DIAG_PRE")  # "0" / "1": first a step on that half of the batch (like a 2-rank run)
if pre is not None:
    half = x[: B // 2] if pre == "0" else x[B // 2:]
    net.load_state_dict(state)
    (net(half).float().square().sum() / B).backward()
    net.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
BWD = os.environ.get("DIAG_BWD") == "1"
runs = []
for rep in range(REPS):
    if os.environ.get("DIAG_POISON") and rep > 0:
        poison(float("nan") if rep % 2 else 12345.0)
    net.load_state_dict(state)
    LOG.clear()
    net.zero_grad(set_to_none=True)
    out = net(x)
    if BWD:  # then every parameter gradient too, in parameter order
        (out.float().square().sum() / x.shape[0]).backward()
        for n, p in net.named_parameters():
            LOG.append((f"grad {n}", [p.grad.detach().clone()]))
    torch.cuda.synchronize()
    runs.append(list(LOG))
for rep in range(1, REPS):
    bad = None
    for i, ((n0, t0), (n1, t1)) in enumerate(zip(runs[0], runs[rep])):
        for j, (a, b) in enumerate(zip(t0, t1)):
            if not torch.equal(a, b):
                d = (a.float() - b.float()).abs()
                print(f"run {rep}: op #{i} {n0} output {j} shape {tuple(a.shape)} differs: max |d| {d.max().item():.3e}, "
                      f"{(d > 0).sum().item()} of {d.numel()} elements")
                bad = i
                break
        if bad is not None:
            break
    if bad is None:
        print(f"run {rep}: all {len(runs[0])} ops bitwise identical")
print("ops:", [n for n, _ in runs[0]])
dump = os.environ.get("DIAG_DUMP")
if dump:  # per-op output checksums, to compare two processes (python diag_determinism.py a; ... b; diff)
    import hashlib

    with open(dump, "w") as f:
        for i, (n, ts) in enumerate(runs[0]):
            hs = [hashlib.sha1(t.detach().contiguous().reshape(-1).view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12] for t in ts]
            f.write(f"{i} {n} {' '.join(hs)}\n")
