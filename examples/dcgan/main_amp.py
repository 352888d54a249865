"""DCGAN with amp: two models, two optimizers, three losses each with its own loss scaler
(reference workload: examples/dcgan/main_amp.py — ``amp.initialize([netD, netG], [optD, optG],
num_losses=3)`` and ``amp.scale_loss(..., loss_id=k)``).

Data: synthetic images (``--dataset fake``, the default; this container has no datasets) or an
ImageFolder root via torchvision when installed. The generator output and discriminator loss use
``binary_cross_entropy_with_logits`` (amp-safe; plain BCE is banned under O1 as in the reference).
"""
import argparse
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")))
from beforeholiday_amd import amp  # noqa: E402
from beforeholiday_amd.optimizers import FusedAdam  # noqa: E402


def parser():
    p = argparse.ArgumentParser()
    p.add_argument("--dataset", default="fake", help="fake | folder")
    p.add_argument("--dataroot", default="./")
    p.add_argument("--batchSize", type=int, default=64)
    p.add_argument("--imageSize", type=int, default=64)
    p.add_argument("--nz", type=int, default=100)
    p.add_argument("--ngf", type=int, default=64)
    p.add_argument("--ndf", type=int, default=64)
    p.add_argument("--niter", type=int, default=1)
    p.add_argument("--iters", type=int, default=0, help="cap iterations per epoch (0 = all)")
    p.add_argument("--lr", type=float, default=0.0002)
    p.add_argument("--beta1", type=float, default=0.5)
    p.add_argument("--netG", default="")
    p.add_argument("--netD", default="")
    p.add_argument("--outf", default="")
    p.add_argument("--manualSeed", type=int, default=1234)
    p.add_argument("--opt_level", default="O1")
    p.add_argument("--device", default="cuda")
    p.add_argument("--fused-adam", action="store_true")
    return p


def weights_init(m):
    name = m.__class__.__name__
    if "Conv" in name:
        nn.init.normal_(m.weight, 0.0, 0.02)
    elif "BatchNorm" in name:
        nn.init.normal_(m.weight, 1.0, 0.02)
        nn.init.zeros_(m.bias)


class Generator(nn.Module):
    def __init__(self, nz, ngf, nc=3):
        super().__init__()

        def up(i, o, k=4, s=2, p=1):
            return [nn.ConvTranspose2d(i, o, k, s, p, bias=False), nn.BatchNorm2d(o), nn.ReLU(True)]

        self.main = nn.Sequential(*up(nz, ngf * 8, 4, 1, 0), *up(ngf * 8, ngf * 4), *up(ngf * 4, ngf * 2),
                                  *up(ngf * 2, ngf), nn.ConvTranspose2d(ngf, nc, 4, 2, 1, bias=False), nn.Tanh())

    def forward(self, z):
        return self.main(z)


class Discriminator(nn.Module):
    def __init__(self, ndf, nc=3):
        super().__init__()

        def down(i, o, bn=True):
            layers = [nn.Conv2d(i, o, 4, 2, 1, bias=False)]
            if bn:
                layers.append(nn.BatchNorm2d(o))
            return layers + [nn.LeakyReLU(0.2, inplace=True)]

        self.main = nn.Sequential(*down(nc, ndf, bn=False), *down(ndf, ndf * 2), *down(ndf * 2, ndf * 4),
                                  *down(ndf * 4, ndf * 8), nn.Conv2d(ndf * 8, 1, 4, 1, 0, bias=False))

    def forward(self, x):
        return self.main(x).view(-1)  # logits


def batches(args, device):
    if args.dataset == "folder":
        import torchvision.datasets as dset
        import torchvision.transforms as T
        ds = dset.ImageFolder(args.dataroot, T.Compose([T.Resize(args.imageSize), T.CenterCrop(args.imageSize),
                                                        T.ToTensor(), T.Normalize((0.5,) * 3, (0.5,) * 3)]))
        for x, _ in torch.utils.data.DataLoader(ds, batch_size=args.batchSize, shuffle=True, drop_last=True):
            yield x.to(device, non_blocking=True)
    else:
        g = torch.Generator(device="cpu").manual_seed(args.manualSeed)
        n = args.iters or 50
        for _ in range(n):
            yield (torch.rand(args.batchSize, 3, args.imageSize, args.imageSize, generator=g) * 2 - 1).to(device)


def run(argv=None):
    args = parser().parse_args(argv)
    device = torch.device(args.device)
    torch.manual_seed(args.manualSeed)
    netG = Generator(args.nz, args.ngf).to(device)
    netD = Discriminator(args.ndf).to(device)
    netG.apply(weights_init)
    netD.apply(weights_init)
    if args.netG:
        netG.load_state_dict(torch.load(args.netG, map_location=device, weights_only=True))
    if args.netD:
        netD.load_state_dict(torch.load(args.netD, map_location=device, weights_only=True))
    Opt = FusedAdam if args.fused_adam else torch.optim.Adam
    optD = Opt(netD.parameters(), lr=args.lr, betas=(args.beta1, 0.999))
    optG = Opt(netG.parameters(), lr=args.lr, betas=(args.beta1, 0.999))
    [netD, netG], [optD, optG] = amp.initialize([netD, netG], [optD, optG], opt_level=args.opt_level,
                                                num_losses=3, verbosity=0)
    fixed_noise = torch.randn(args.batchSize, args.nz, 1, 1, device=device)
    hist = []
    for epoch in range(args.niter):
        for i, real in enumerate(batches(args, device)):
            if args.iters and i >= args.iters:
                break
            b = real.size(0)
            ones = torch.ones(b, device=device)
            zeros = torch.zeros(b, device=device)
            # (1) D: maximise log D(x) + log(1 - D(G(z)))
            optD.zero_grad()
            errD_real = F.binary_cross_entropy_with_logits(netD(real), ones)
            with amp.scale_loss(errD_real, optD, loss_id=0) as s:
                s.backward()
            fake = netG(torch.randn(b, args.nz, 1, 1, device=device))
            errD_fake = F.binary_cross_entropy_with_logits(netD(fake.detach()), zeros)
            with amp.scale_loss(errD_fake, optD, loss_id=1) as s:
                s.backward()
            optD.step()
            # (2) G: maximise log D(G(z))
            optG.zero_grad()
            errG = F.binary_cross_entropy_with_logits(netD(fake), ones)
            with amp.scale_loss(errG, optG, loss_id=2) as s:
                s.backward()
            optG.step()
            hist.append((float((errD_real + errD_fake).detach()), float(errG.detach())))
            if i % 10 == 0:
                print(f"[{epoch}/{args.niter}][{i}] Loss_D {hist[-1][0]:.4f} Loss_G {hist[-1][1]:.4f}", flush=True)
        if args.outf:
            os.makedirs(args.outf, exist_ok=True)
            with torch.no_grad():
                torch.save(netG(fixed_noise).float().cpu(), os.path.join(args.outf, f"fake_samples_epoch_{epoch:03d}.pt"))
            torch.save(netG.state_dict(), os.path.join(args.outf, f"netG_epoch_{epoch}.pth"))
            torch.save(netD.state_dict(), os.path.join(args.outf, f"netD_epoch_{epoch}.pth"))
    amp.deactivate()
    return hist


if __name__ == "__main__":
    run()
