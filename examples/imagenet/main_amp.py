"""ImageNet training with amp, DDP and SyncBatchNorm (reference workload:
examples/imagenet/main_amp.py and tests/L1/common/main_amp.py).

One process per GPU (``torchrun --nproc-per-node N main_amp.py ...``; RCCL over xGMI). The input
pipeline is a stream prefetcher: the next batch is copied host->device and normalised on a side HIP
stream while the current step runs, and the compute stream waits on an event, not the host.

Data: an ImageFolder tree when ``DIR`` is given (needs torchvision); otherwise a fixed synthetic
uint8 image set generated from ``--seed`` (this container has no datasets), so runs are
reproducible and the L1 cross-product harness (``tests/L1``) can compare loss trajectories.

``--has-ext`` selects the fused multi-tensor loss-scale unscale; without it the same run uses the
per-tensor python scaler, i.e. the reference's "python-only install". Both use ``torch.optim.SGD``
unless ``--fused-sgd`` / ``--fused-adam`` is given, as in the reference harness. The per-iteration losses are saved to
``<out-dir>/<has_ext>_<opt>_<loss_scale>_<keep_bn>_<fused_adam>`` as a dict of lists (the
reference's L1 file format, ``tests/L1/common/main_amp.py:500-526``).
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(_HERE, "..", "..")))

from beforeholiday_amd import amp  # noqa: E402
from beforeholiday_amd.models import resnet as bh_resnet  # noqa: E402

MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


def _str2bool(v):
    if v is None or isinstance(v, bool):
        return v
    return {"true": True, "false": False}[v.lower()]


def parser():
    p = argparse.ArgumentParser(description="beforeholiday_amd ImageNet training (amp / DDP / SyncBN)")
    p.add_argument("data", nargs="?", default=None, help="ImageFolder root (train/ val/); synthetic if absent")
    p.add_argument("-a", "--arch", default="resnet50", choices=["resnet50", "resnet18_like", "tiny"])
    p.add_argument("-j", "--workers", default=4, type=int)
    p.add_argument("--epochs", default=1, type=int)
    p.add_argument("--start-epoch", default=0, type=int)
    p.add_argument("-b", "--b", "--batch-size", dest="batch_size", default=128, type=int, help="per-GPU batch")
    p.add_argument("--lr", "--learning-rate", dest="lr", default=0.1, type=float, help="for 256 images")
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--wd", "--weight-decay", dest="weight_decay", default=1e-4, type=float)
    p.add_argument("--print-freq", "-p", default=10, type=int)
    p.add_argument("--resume", default="", type=str, help="checkpoint to resume from")
    p.add_argument("--save", default="", type=str, help="checkpoint path written at each epoch end")
    p.add_argument("-e", "--evaluate", action="store_true")
    p.add_argument("--prof", default=-1, type=int, help="stop after this many iterations (profiling)")
    p.add_argument("--deterministic", action="store_true")
    p.add_argument("--sync_bn", action="store_true")
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--opt-level", default="O2", type=str)
    p.add_argument("--keep-batchnorm-fp32", default=None, type=str)
    p.add_argument("--loss-scale", default=None, type=str)
    p.add_argument("--fused-adam", action="store_true")
    p.add_argument("--fused-sgd", action="store_true")
    p.add_argument("--has-ext", action="store_true")
    p.add_argument("--prints-to-process", default=-1, type=int,
                   help="L1 mode: record this many iterations, save the trajectory and exit")
    p.add_argument("--image-size", default=224, type=int)
    p.add_argument("--num-classes", default=1000, type=int)
    p.add_argument("--synthetic-images", default=2048, type=int)
    p.add_argument("--iters-per-epoch", default=0, type=int, help="cap (0 = the whole data set)")
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--device", default="cuda")
    p.add_argument("--out-dir", default=".")
    p.add_argument("--quiet", action="store_true")
    return p


# ------------------------------------------------------------------------------------ models
class _Tiny(nn.Module):
    """Conv-BN-ReLU x2 + linear head: the CPU-sized model of the L1 harness tests."""

    def __init__(self, num_classes):
        super().__init__()
        self.c1, self.b1 = nn.Conv2d(3, 16, 3, 2, 1, bias=False), nn.BatchNorm2d(16)
        self.c2, self.b2 = nn.Conv2d(16, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32)
        self.fc = nn.Linear(32, num_classes)

    def forward(self, x):
        x = F.relu(self.b1(self.c1(x)))
        x = F.relu(self.b2(self.c2(x)))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def build_model(args):
    if args.arch == "tiny":
        return _Tiny(args.num_classes)
    return getattr(bh_resnet, args.arch)(num_classes=args.num_classes)


# ------------------------------------------------------------------------------------ data
class SyntheticImages(torch.utils.data.Dataset):
    """Deterministic uint8 CHW images + labels, generated once from the seed."""

    def __init__(self, n, size, num_classes, seed):
        g = torch.Generator().manual_seed(seed)
        self.images = torch.randint(0, 256, (n, 3, size, size), dtype=torch.uint8, generator=g)
        self.labels = torch.randint(0, num_classes, (n,), generator=g)

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        return self.images[i], self.labels[i]


def _collate_u8(batch):
    imgs = torch.stack([b[0] for b in batch])
    return imgs, torch.tensor([int(b[1]) for b in batch], dtype=torch.int64)


def build_loader(args, train, world, rank):
    if args.data:
        import torchvision.datasets as datasets  # only for real data
        import torchvision.transforms as transforms

        tf = (transforms.Compose([transforms.RandomResizedCrop(args.image_size), transforms.RandomHorizontalFlip(),
                                  transforms.PILToTensor()]) if train else
              transforms.Compose([transforms.Resize(int(args.image_size * 256 / 224)),
                                  transforms.CenterCrop(args.image_size), transforms.PILToTensor()]))
        ds = datasets.ImageFolder(os.path.join(args.data, "train" if train else "val"), tf)
    else:
        ds = SyntheticImages(args.synthetic_images, args.image_size, args.num_classes,
                             args.seed + (0 if train else 1))
    sampler = None
    if world > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world, rank=rank,
                                                                  shuffle=train and not args.deterministic)
    shuffle = train and sampler is None and not args.deterministic
    workers = 0 if (args.deterministic or not args.data) else args.workers
    return torch.utils.data.DataLoader(ds, batch_size=args.batch_size, shuffle=shuffle, num_workers=workers,
                                       pin_memory=bool(args.data) and args.device != "cpu", sampler=sampler, collate_fn=_collate_u8,
                                       drop_last=train)


class Prefetcher:
    """Overlaps the H2D copy + normalisation of batch i+1 with step i on a side stream."""

    def __init__(self, loader, device, channels_last, dtype):
        self.it = iter(loader)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.mean = torch.tensor(MEAN, device=self.device).view(1, 3, 1, 1)
        self.std = torch.tensor(STD, device=self.device).view(1, 3, 1, 1)
        self.fmt = torch.channels_last if channels_last else torch.contiguous_format
        self.dtype = dtype
        self._preload()

    def _preload(self):
        try:
            x, y = next(self.it)
        except StopIteration:
            self.next = None
            return
        if self.cuda:
            with torch.cuda.stream(self.stream):
                x = x.to(self.device, non_blocking=True)
                y = y.to(self.device, non_blocking=True)
                x = ((x.float() - self.mean) / self.std).to(self.dtype).contiguous(memory_format=self.fmt)
        else:
            x = ((x.float() - self.mean) / self.std).to(self.dtype).contiguous(memory_format=self.fmt)
        self.next = (x, y)

    def __iter__(self):
        return self

    def __next__(self):
        if self.next is None:
            raise StopIteration
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.stream)
            for t in self.next:
                t.record_stream(cur)
        out = self.next
        self._preload()
        return out


# ------------------------------------------------------------------------------------ training
class AverageMeter:
    def __init__(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, v, n=1):
        self.val = v
        self.sum += v * n
        self.count += n
        self.avg = self.sum / max(self.count, 1)


def accuracy(output, target, topk=(1,)):
    maxk = max(topk)
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1))
    return [correct[:k].reshape(-1).float().sum() * (100.0 / target.size(0)) for k in topk]


def adjust_learning_rate(optimizer, base_lr, epoch, step, steps_per_epoch):
    """5-epoch linear warmup, then /10 at epochs 30, 60, 80 (reference schedule)."""
    factor = epoch // 30 + (1 if epoch >= 80 else 0)
    lr = base_lr * (0.1 ** factor)
    if epoch < 5:
        lr = lr * float(1 + step + epoch * steps_per_epoch) / (5.0 * steps_per_epoch)
    for g in optimizer.param_groups:
        g["lr"] = lr


def _loss_scale_arg(v):
    if v is None or v == "dynamic":
        return v
    return float(v)


def run(argv=None):
    """Train; returns ``{"Iteration": [...], "Loss": [...], "Speed": [...], "top1": float}``."""
    args = parser().parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if args.device == "cuda":
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
        device = f"cuda:{torch.cuda.current_device()}"
    else:
        device = "cpu"
    if distributed and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("nccl" if device != "cpu" else "gloo")
    if args.deterministic:
        torch.manual_seed(args.seed)
        torch.backends.cudnn.benchmark = False
        torch.backends.cudnn.deterministic = True
    else:
        torch.backends.cudnn.benchmark = True

    from beforeholiday_amd.amp.scaler import LossScaler
    LossScaler.has_fused_kernel = bool(args.has_ext)

    torch.manual_seed(args.seed)
    model = build_model(args)
    if args.sync_bn:
        from beforeholiday_amd.parallel import convert_syncbn_model
        model = convert_syncbn_model(model)
    model = model.to(device)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)

    lr = args.lr * float(args.batch_size * world) / 256.0
    if args.fused_adam:
        from beforeholiday_amd.optimizers import FusedAdam
        optimizer = FusedAdam(model.parameters(), lr=lr, weight_decay=args.weight_decay)
    elif args.fused_sgd:
        from beforeholiday_amd.optimizers import FusedSGD
        optimizer = FusedSGD(model.parameters(), lr, momentum=args.momentum, weight_decay=args.weight_decay)
    else:
        optimizer = torch.optim.SGD(model.parameters(), lr, momentum=args.momentum, weight_decay=args.weight_decay)

    model, optimizer = amp.initialize(model, optimizer, opt_level=args.opt_level,
                                      keep_batchnorm_fp32=_str2bool(args.keep_batchnorm_fp32),
                                      loss_scale=_loss_scale_arg(args.loss_scale), verbosity=0)
    if distributed:
        from beforeholiday_amd.parallel import DistributedDataParallel
        model = DistributedDataParallel(model, delay_allreduce=True)
    criterion = nn.CrossEntropyLoss().to(device)

    if args.resume:
        from beforeholiday_amd.utils.checkpoint import load_checkpoint
        ck = load_checkpoint(args.resume, model.module if distributed else model, optimizer, amp,
                             map_location=device)
        args.start_epoch = ck.get("epoch", 0)

    in_dtype = {"O3": torch.float16, "O2": torch.float16, "O5": torch.bfloat16}.get(args.opt_level, torch.float32)
    train_loader = build_loader(args, True, world, rank)
    record = {"Iteration": [], "Loss": [], "Speed": []}
    say = (lambda *a: None) if (args.quiet or rank != 0) else (lambda *a: print(*a, flush=True))
    if args.evaluate:
        top1 = validate(args, model, criterion, device, in_dtype, world, rank, say)
        amp.deactivate()
        return {**record, "top1": top1}

    total_iters = 0
    for epoch in range(args.start_epoch, args.epochs):
        if distributed and hasattr(train_loader.sampler, "set_epoch"):
            train_loader.sampler.set_epoch(epoch)
        model.train()
        steps = len(train_loader) if not args.iters_per_epoch else min(len(train_loader), args.iters_per_epoch)
        batch_time, losses = AverageMeter(), AverageMeter()
        end = time.time()
        for i, (x, y) in enumerate(Prefetcher(train_loader, device, args.channels_last, in_dtype)):
            if i >= steps:
                break
            adjust_learning_rate(optimizer, lr, epoch, i, steps)
            out = model(x)
            loss = criterion(out, y)
            optimizer.zero_grad()
            with amp.scale_loss(loss, optimizer) as scaled:
                scaled.backward()
            optimizer.step()
            total_iters += 1
            if i % args.print_freq == 0 or args.prints_to_process > 0:
                # the only host syncs of the step, at print cadence
                lv = loss.detach().float()
                if distributed:
                    torch.distributed.all_reduce(lv)
                    lv /= world
                if device != "cpu":
                    torch.cuda.synchronize()
                dt = (time.time() - end) / (args.print_freq if i and args.prints_to_process <= 0 else 1)
                end = time.time()
                batch_time.update(dt)
                losses.update(float(lv), x.size(0))
                speed = world * args.batch_size / max(dt, 1e-9)
                record["Iteration"].append(i)
                record["Loss"].append(float(lv))
                record["Speed"].append(speed)
                say(f"Epoch [{epoch}][{i}/{steps}] time {batch_time.val:.3f} ({batch_time.avg:.3f}) "
                    f"speed {speed:.1f} img/s loss {losses.val:.10f} ({losses.avg:.4f}) "
                    f"scale {amp._amp_state.loss_scalers[0].loss_scale() if amp._amp_state.loss_scalers else 1}")
            if args.prints_to_process > 0 and len(record["Iteration"]) >= args.prints_to_process:
                break
            if args.prof > 0 and total_iters >= args.prof:
                break
        if args.prints_to_process > 0 or (args.prof > 0 and total_iters >= args.prof):
            break
        if args.save and rank == 0:
            from beforeholiday_amd.utils.checkpoint import save_checkpoint
            save_checkpoint(args.save, model.module if distributed else model, optimizer, amp, epoch=epoch + 1,
                            extra={"arch": args.arch})

    if args.prints_to_process > 0 and rank == 0:
        name = "{}_{}_{}_{}_{}".format(bool(args.has_ext), args.opt_level, args.loss_scale,
                                       args.keep_batchnorm_fp32, bool(args.fused_adam))
        os.makedirs(args.out_dir, exist_ok=True)
        torch.save(record, os.path.join(args.out_dir, name))
    amp.deactivate()
    return record


@torch.no_grad()
def validate(args, model, criterion, device, in_dtype, world, rank, say):
    model.eval()
    loader = build_loader(args, False, world, rank)
    top1, n = torch.zeros((), device=device), 0
    for x, y in Prefetcher(loader, device, args.channels_last, in_dtype):
        out = model(x)
        top1 += accuracy(out.float(), y)[0] * y.size(0) / 100.0
        n += y.size(0)
    stats = torch.stack([top1.float(), torch.tensor(float(n), device=device)])
    if world > 1:
        torch.distributed.all_reduce(stats)
    acc = float(stats[0] / stats[1].clamp_min(1)) * 100.0
    say(f" * Acc@1 {acc:.3f}")
    return acc


if __name__ == "__main__":
    r = run()
    if not math.isfinite(r["Loss"][-1] if r.get("Loss") else 0.0):
        sys.exit(1)
