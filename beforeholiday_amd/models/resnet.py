"""ResNet-50 (v1.5: stride on the 3x3 conv), the reference's headline ImageNet workload
(examples/imagenet/main_amp.py, ``-a resnet50``). Written here because torchvision is not part of
the stack; layer shapes and init follow torchvision's ``resnet50`` so parameter counts (25.56 M)
and FLOPs match.
"""
from __future__ import annotations

from typing import List, Optional, Type

import torch
import torch.nn as nn

from .. import config as _config


def conv3x3(cin, cout, stride=1):
    if _CONV3X3_MODE != "miopen" and stride in (1, 2):
        return Conv3x3(cin, cout, 3, stride=stride, padding=1, bias=False, mode=_CONV3X3_MODE)
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def _time_ms(fn, reps=3):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def _kx(x):
    """x as the own kernels consume it: under amp O1 / O4 (fp32 model, torch functions patched to
    cast to 16 bits) an fp32 activation is cast to amp's dtype here, since the kernel paths below are
    not torch functions the cast lists could see. Otherwise x unchanged."""
    from ..amp.amp import kernel_cast_dtype

    dt = kernel_cast_dtype()
    if dt is not None and x.is_cuda and x.dtype == torch.float32:
        return x.to(dt)
    return x


def _kw(weight, x):
    """``weight`` in x's dtype for the kernel paths: the weight itself for a 16-bit model (O2 / O5 / a
    .half() model), amp's per-iteration 16-bit copy of an fp32 weight under O1 / O4 (differentiable:
    the fp32 parameter gets an fp32 gradient), None when the kernel paths do not apply."""
    if weight.dtype == x.dtype:
        return weight
    from ..amp.amp import kernel_cast, kernel_cast_dtype

    if weight.dtype == torch.float32 and x.dtype == kernel_cast_dtype():
        return kernel_cast(weight)
    return None


def _like(g, weight):
    return g if g.stride() == weight.stride() else g.contiguous()


def _conv_wgrad(x, gy, r, weight, scale=None, shift=None, stride=1):
    """``ops.conv.conv_wgrad`` in ``weight``'s layout. (Rounds 3-4 also tried the weight gradients and
    their split-partial sums on a second HIP stream; both lost on the same box --
    profiles/resnet50_wgrad_side_stream_ab.txt, profiles/resnet50_wgrad_reduce_side_ab.txt -- and were
    removed.)"""
    from ..ops import conv as bhconv

    return _like(bhconv.conv_wgrad(x, gy, r, scale, shift, stride=stride), weight)


# per-shape choice of the 1x1 / stride-1 convolution paths: {(N, Cin, H, W, Cout, dtype, dir): "gemm" | "miopen"}
_CONV1X1_CHOICE = {}


def choice_table():
    """The per-shape kernel choices this process has made so far (sorted, printable): identical on
    every rank by construction (tests/test_determinism.py checks it)."""
    return sorted((tuple(str(v) for v in k), c) for k, c in _CONV1X1_CHOICE.items())


def _agree(choice):
    """With ``BH_CONV_TUNE=1`` under an initialised multi-rank default group, every rank takes rank 0's
    timed choice (one int broadcast): ranks that time for themselves pick different kernels when the
    timings are close, and then neither compute identically nor step in lock-step. All ranks reach the
    same ``_pick`` calls in the same order (same model, same shapes), so the broadcasts pair up."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return choice
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if choice == "gemm" else 0], dtype=torch.int32, device=dev)
    dist.broadcast(t, 0)
    return "gemm" if int(t.item()) else "miopen"


def _pick(key, gemm_fn, miopen_fn, mode):
    """``mode`` "gemm" / "miopen" forces a path. "auto" is the own MFMA / strip kernels ("gemm") for
    every shape -- a static, rank-independent rule, so two processes always run the same kernels and
    the same reduction order (round 3's timed picks diverged between two ranks sharing a GPU and broke
    the two-rank equivalence test). ``BH_CONV_TUNE=1`` restores timing both once per shape and keeping
    the faster, with rank 0's result broadcast to all ranks (``_agree``)."""
    if mode != "auto":
        return mode
    choice = _CONV1X1_CHOICE.get(key)
    if choice is None:
        if _config.get().conv_tune:
            # interleaved A, B, A, B and the best of each: the first step runs on a cold GPU (clocks
            # ramping, first-use kernel loads), and a pick made on one noisy sample sticks for the run
            t_gemm, t_miopen = _time_ms(gemm_fn), _time_ms(miopen_fn)
            t_gemm, t_miopen = min(t_gemm, _time_ms(gemm_fn)), min(t_miopen, _time_ms(miopen_fn))
            choice = _agree("gemm" if t_gemm < t_miopen else "miopen")
        else:
            choice = "gemm"
        _CONV1X1_CHOICE[key] = choice
    return choice


def _wgrad(x, gy, weight, r, mode, miopen_fn):
    """Weight gradient of a stride-1 r x r conv: the MFMA kernel of kernels/conv_wgrad.hip or MIOpen,
    per shape ("auto" times both once). Measured at ResNet-50 / batch 256: see
    profiles/conv_wgrad_vs_miopen.jsonl."""
    from ..ops import conv as bhconv

    if _config.get().conv_wgrad == "miopen":  # A/B switch (benchmarks)
        mode = "miopen"
    if mode == "miopen" or not bhconv.wgrad_supported(x, gy, r):
        return miopen_fn()
    n, c, h, w = x.shape
    how = _pick((n, c, h, w, gy.size(1), x.dtype, f"wgrad{r}"), lambda: bhconv.conv_wgrad(x, gy, r), miopen_fn, mode)
    if how != "gemm":
        return miopen_fn()
    return _conv_wgrad(x, gy, r, weight)  # in the parameter's layout


class _GradStash(torch.autograd.Function):
    """Identity in forward. In backward, the gradient arriving through this (second) use of a tensor
    is parked in ``box`` for the block's first 1x1 convolution, whose data-gradient GEMM then adds it
    with beta = 1 (``addmm`` into this buffer) -- the residual-branch gradient sum costs no extra pass
    (otherwise autograd adds the two branch gradients with a separate elementwise kernel: 16 launches,
    1.3 ms per ResNet-50 step at batch 256). If the convolution's backward already ran, the gradient
    is returned normally."""

    @staticmethod
    def forward(ctx, x, box):
        ctx.box = box
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        if box.get("conv_done"):
            return g, None
        box["g"] = g
        return None, None


def _mm64(a2d, b):
    """``a2d @ b.t()`` for a 64-row ``b`` on the streaming MFMA kernel (kernels/gemm_n64.hip: the
    64-channel side of the 56x56 1x1 convolutions, HBM bound), torch.mm (hipBLASLt) otherwise.
    ``BH_GEMM_N64=0`` keeps hipBLASLt (A/B switch)."""
    from ..ops import conv as bhconv

    if b.size(0) == 64 and _config.get().gemm_n64 and bhconv.gemm_n64_supported(a2d, b):
        return bhconv.gemm_n64(a2d, b)
    return torch.mm(a2d, b.t())


class _Conv1x1Fn(torch.autograd.Function):
    """1x1 / stride-1 convolution of a channels_last activation. Forward and data gradient run either
    as ONE hipBLASLt GEMM on the [N*H*W, C] view (no layout change) or as the MIOpen convolution,
    chosen per shape; the weight gradient -- a K = N*H*W split reduction that hipBLASLt handles badly
    (1.0 vs 0.14 ms at 64->256 / 56x56) -- runs on the MFMA wgrad kernel or MIOpen (``_wgrad``)."""

    @staticmethod
    def forward(ctx, x, weight, mode, box=None):
        n, c, h, w = x.shape
        x2d = x.permute(0, 2, 3, 1).reshape(-1, c)
        w2d = weight.view(weight.size(0), c)
        key = (n, c, h, w, weight.size(0), x.dtype, "fwd")
        how = _pick(key, lambda: _mm64(x2d, w2d), lambda: torch.nn.functional.conv2d(x, weight), mode)
        if how == "gemm":
            y = _mm64(x2d, w2d).view(n, h, w, -1).permute(0, 3, 1, 2)
        else:
            y = torch.nn.functional.conv2d(x, weight)
        ctx.save_for_backward(x, weight)
        ctx.mode = mode
        ctx.box = box
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        n, c, h, w = x.shape
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = gw = None
        conv_bwd = torch.ops.aten.convolution_backward
        args = ([1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        box = ctx.box
        acc = box.pop("g", None) if box is not None else None
        if ctx.needs_input_grad[0] and acc is not None and acc.is_contiguous(memory_format=torch.channels_last) \
                and acc.dtype == gy.dtype and acc.shape == x.shape:
            # residual branch gradient already here: dX = acc + dY @ W in one GEMM (beta = 1)
            gy2d = gy.permute(0, 2, 3, 1).reshape(-1, weight.size(0))
            acc2d = acc.permute(0, 2, 3, 1).reshape(-1, c)
            wt = weight.view(weight.size(0), c).t().contiguous() if c == 64 else None
            from ..ops import conv as bhconv

            if wt is not None and _config.get().gemm_n64 and bhconv.gemm_n64_supported(gy2d, wt):
                # 64-channel input (layer1's first block): the streaming kernel adds the stash in its epilogue
                gx = bhconv.gemm_n64(gy2d, wt, acc2d).view(n, h, w, c).permute(0, 3, 1, 2)
            else:
                torch.addmm(acc2d, gy2d, weight.view(weight.size(0), c), out=acc2d)
                gx = acc
            acc = None
        elif ctx.needs_input_grad[0]:
            gy2d = gy.permute(0, 2, 3, 1).reshape(-1, weight.size(0))
            wt = weight.view(weight.size(0), c).t()  # [c, k]: dX = dY @ W = dY . wt^T
            if c == 64:
                wt = wt.contiguous()
            key = (n, c, h, w, weight.size(0), x.dtype, "dgrad")
            how = _pick(key, lambda: _mm64(gy2d, wt),
                        lambda: conv_bwd(gy, x, weight, None, *args, [True, False, False]), ctx.mode)
            if how == "gemm":
                gx = _mm64(gy2d, wt).view(n, h, w, c).permute(0, 3, 1, 2)
            else:
                gx = conv_bwd(gy, x, weight, None, *args, [True, False, False])[0]
        if acc is not None:
            gx = acc if gx is None else gx + acc  # stash arrived but could not be fused
        if box is not None:
            box["conv_done"] = True
        if ctx.needs_input_grad[1]:
            # 1x1: the MFMA wgrad kernel only through the timed per-shape choice (MIOpen wins most shapes)
            gw = _wgrad(x, gy, weight, 1, "auto" if ctx.mode == "auto" else "miopen",
                        lambda: conv_bwd(gy, x, weight, None, *args, [False, True, False])[1])
        return gx, gw, None, None


class Conv1x1(nn.Conv2d):
    """nn.Conv2d(k=1, bias=False) whose stride-1 channels_last GPU path picks hipBLASLt or MIOpen per
    shape and direction (``mode`` "auto" / "gemm" / "miopen"); a regular convolution otherwise."""

    def __init__(self, *args, mode="auto", **kw):
        super().__init__(*args, **kw)
        self.mode = mode

    def fast_path(self, x, w=None):
        w = self.weight if w is None else w
        return (x.is_cuda and self.stride == (1, 1) and self.groups == 1 and x.dim() == 4 and self.mode != "miopen"
                and x.is_contiguous(memory_format=torch.channels_last) and x.dtype == w.dtype)

    def forward(self, x, box=None):
        xk = _kx(x)
        w = _kw(self.weight, xk)
        if w is not None and self.fast_path(xk, w):
            return _Conv1x1Fn.apply(xk, w, self.mode, box)
        return super().forward(x)


_CONV1X1_MODE = "miopen"  # "miopen" (plain nn.Conv2d), "auto" or "gemm" (Conv1x1)
_CONV3X3_MODE = "miopen"  # "miopen" (plain nn.Conv2d), "auto" or "direct" (Conv3x3)


class _Conv3x3Fn(torch.autograd.Function):
    """3x3 / stride-1 / pad-1 convolution of a channels_last activation: forward and data gradient
    on the direct MFMA kernel (kernels/conv.hip; the data gradient is the same kernel on dY with the
    flipped, transposed weights) or on MIOpen, chosen per shape and direction ("auto" times both once);
    the weight gradient likewise on the MFMA wgrad kernel (kernels/conv_wgrad.hip) or MIOpen. Measured at ResNet-50 / batch 256 (benchmarks/
    bench_conv3x3.py): forward 1.45 vs 1.96 ms, data gradient 1.59 vs 1.84 ms per step."""

    @staticmethod
    def forward(ctx, x, weight, mode):
        from ..ops import conv as bhconv

        n, c, h, w = x.shape
        conv = torch.nn.functional.conv2d
        how = _pick((n, c, h, w, weight.size(0), x.dtype, "fwd3"), lambda: bhconv.conv3x3(x, weight),
                    lambda: conv(x, weight, padding=1), "gemm" if mode == "direct" else mode)
        y = bhconv.conv3x3(x, weight) if how == "gemm" else conv(x, weight, padding=1)
        ctx.save_for_backward(x, weight)
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..ops import conv as bhconv

        x, weight = ctx.saved_tensors
        n, c, h, w = x.shape
        gy = gy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = ([1, 1], [1, 1], [1, 1], False, [0, 0], 1)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            how = _pick((n, c, h, w, weight.size(0), x.dtype, "dgrad3"), lambda: bhconv.conv3x3_dgrad(gy, weight),
                        lambda: conv_bwd(gy, x, weight, None, *args, [True, False, False]),
                        "gemm" if ctx.mode == "direct" else ctx.mode)
            if how == "gemm":
                gx = bhconv.conv3x3_dgrad(gy, weight)
            else:
                gx = conv_bwd(gy, x, weight, None, *args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            gw = _wgrad(x, gy, weight, 3, "gemm" if ctx.mode == "direct" else ctx.mode,
                        lambda: conv_bwd(gy, x, weight, None, *args, [False, True, False])[1])
        return gx, gw, None


class _Conv3x3S2Fn(torch.autograd.Function):
    """3x3 / stride-2 / pad-1 convolution of a channels_last activation (the ResNet downsampling
    blocks' middle conv) on the own MFMA kernels in all three directions: forward and data gradient on
    the implicit-GEMM kernel (kernels/conv_igemm.hip; the data gradient as four stride-1 phase
    convolutions), weight gradient on the strided-halo wgrad kernel. No MIOpen: its stride-2 weight
    gradient is split-K with atomics (not run-to-run repeatable, profiles/miopen_s2_determinism.jsonl)."""

    @staticmethod
    def forward(ctx, x, weight):
        from ..ops import conv as bhconv

        y, _ = bhconv.conv3x3_s2(x, weight)
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..ops import conv as bhconv

        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = bhconv.conv3x3_s2_dgrad(gy, weight, (x.size(2), x.size(3)))
        if ctx.needs_input_grad[1]:
            gw = bhconv.conv_wgrad(x, gy, 3, stride=2)
            if gw.stride() != weight.stride():
                gw = gw.contiguous()
        return gx, gw


class Conv3x3(nn.Conv2d):
    """nn.Conv2d(k=3, stride=1 or 2, padding=1, bias=False) whose channels_last fp16 / bf16 GPU path
    runs the own MFMA kernels: stride 1 the direct kernel (or MIOpen per shape, ``mode`` "auto" /
    "direct" / "miopen"), stride 2 the implicit-GEMM kernels (:class:`_Conv3x3S2Fn`)."""

    def __init__(self, *args, mode="auto", **kw):
        super().__init__(*args, **kw)
        self.mode = mode

    def fast_path(self, x, w=None):
        w = self.weight if w is None else w
        if not (self.mode != "miopen" and x.is_cuda and x.dim() == 4 and x.dtype == w.dtype
                and self.stride in ((1, 1), (2, 2)) and self.padding == (1, 1) and self.dilation == (1, 1)
                and self.groups == 1):
            return False
        from ..ops import conv as bhconv

        if self.stride == (2, 2):
            return bhconv.s2_supported(x, w)
        return bhconv.supported(x, w)

    def forward(self, x):
        xk = _kx(x)
        w = _kw(self.weight, xk)
        if w is not None and self.fast_path(xk, w):
            if self.stride == (2, 2):
                return _Conv3x3S2Fn.apply(xk, w)
            return _Conv3x3Fn.apply(xk, w, self.mode)
        return super().forward(x)


class _Conv1x1S2Fn(torch.autograd.Function):
    """1x1 / stride-2 convolution of a channels_last activation (the ResNet downsample branch).
    Every output pixel reads input pixel (2y, 2x), so the layer is a 1x1 convolution of the
    gathered quarter-resolution input ``xg``. The forward gathers ``xg`` once (a strided copy of
    a quarter of the input) and runs the GEMM on it, or it runs MIOpen, whichever is faster per
    shape. ``xg`` is saved instead of the full-resolution input, and the weight gradient is the MFMA
    1x1 wgrad kernel on (xg, dY). The data gradient is one GEMM scattered into a zeroed
    full-resolution tensor, the same work MIOpen's stride-2 backward-data does."""

    @staticmethod
    def forward(ctx, x, weight, mode):
        n, c, h, w = x.shape
        w2d = weight.view(weight.size(0), c)
        conv = torch.nn.functional.conv2d

        def gemm():
            xg = x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
            return xg, torch.mm(xg.permute(0, 2, 3, 1).reshape(-1, c), w2d.t())

        how = _pick((n, c, h, w, weight.size(0), x.dtype, "fwd_s2"), lambda: gemm(), lambda: conv(x, weight, stride=2),
                    mode)
        ho, wo = (h + 1) // 2, (w + 1) // 2
        if how == "gemm":
            xg, y2d = gemm()
            y = y2d.view(n, ho, wo, -1).permute(0, 3, 1, 2)
        else:
            y = conv(x, weight, stride=2)
            xg = x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
        ctx.save_for_backward(xg, weight)
        ctx.in_hw = (h, w)
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, gy):
        xg, weight = ctx.saved_tensors
        n, c, ho, wo = xg.shape
        h, w = ctx.in_hw
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            dxg = torch.mm(gy.permute(0, 2, 3, 1).reshape(-1, weight.size(0)), weight.view(weight.size(0), c))
            gx = torch.zeros((n, c, h, w), dtype=gy.dtype, device=gy.device).contiguous(memory_format=torch.channels_last)
            gx[:, :, ::2, ::2] = dxg.view(n, ho, wo, c).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            conv_bwd = torch.ops.aten.convolution_backward
            args = ([1, 1], [0, 0], [1, 1], False, [0, 0], 1)
            gw = _wgrad(xg, gy, weight, 1, "auto" if ctx.mode == "auto" else "miopen",
                        lambda: conv_bwd(gy, xg, weight, None, *args, [False, True, False])[1])
        return gx, gw, None


class _Conv1x1S2WFn(torch.autograd.Function):
    """1x1 / stride-2 convolution: forward and data gradient on MIOpen, the weight gradient on the
    MFMA wgrad kernel reading the even input pixels in place (``conv_wgrad(..., stride=2)``, no
    gathered copy) or MIOpen, whichever is faster for the shape (timed once)."""

    @staticmethod
    def forward(ctx, x, weight, mode):
        ctx.save_for_backward(x, weight)
        ctx.mode = mode
        return torch.nn.functional.conv2d(x, weight, stride=2)

    @staticmethod
    def backward(ctx, gy):
        from ..ops import conv as bhconv

        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = ([2, 2], [0, 0], [1, 1], False, [0, 0], 1)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = conv_bwd(gy, x, weight, None, *args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            miopen = lambda: conv_bwd(gy, x, weight, None, *args, [False, True, False])[1]  # noqa: E731
            mode = "miopen" if _config.get().conv_wgrad == "miopen" else ctx.mode
            if mode == "miopen" or not bhconv.wgrad_supported(x, gy, 1, 2):
                return gx, miopen(), None
            n, c, h, w = x.shape
            how = _pick((n, c, h, w, weight.size(0), x.dtype, "wgrad1s2"), lambda: bhconv.conv_wgrad_s2(x, gy), miopen,
                        mode)
            gw = bhconv.conv_wgrad_s2(x, gy) if how == "gemm" else miopen()
            if gw.stride() != weight.stride():
                gw = gw.contiguous()
        return gx, gw, None


class _StemConvFn(torch.autograd.Function):
    """ResNet stem 7x7 / stride 2 / pad 3 convolution: forward and weight gradient on the MFMA stem
    kernels (kernels/conv_stem.hip) or MIOpen, whichever is faster for the shape (timed once); the
    input gradient (not needed for the image input) on MIOpen."""

    @staticmethod
    def forward(ctx, x, weight, mode):
        from ..ops import conv as bhconv

        n, c, h, w = x.shape
        conv = torch.nn.functional.conv2d
        how = _pick((n, c, h, w, weight.size(0), x.dtype, "stem"), lambda: bhconv.stem_conv(x, weight),
                    lambda: conv(x, weight, stride=2, padding=3), mode)
        y = bhconv.stem_conv(x, weight) if how == "gemm" else conv(x, weight, stride=2, padding=3)
        ctx.save_for_backward(x, weight)
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..ops import conv as bhconv

        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = ([2, 2], [3, 3], [1, 1], False, [0, 0], 1)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = conv_bwd(gy, x, weight, None, *args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            n, c, h, w = x.shape
            miopen = lambda: conv_bwd(gy, x, weight, None, *args, [False, True, False])[1]  # noqa: E731
            how = _pick((n, c, h, w, weight.size(0), x.dtype, "stem_wgrad"), lambda: bhconv.stem_wgrad(x, gy), miopen,
                        ctx.mode)
            gw = bhconv.stem_wgrad(x, gy) if how == "gemm" else miopen()
            if gw.stride() != weight.stride():
                gw = gw.contiguous()
        return gx, gw, None


class _StemStatsFn(torch.autograd.Function):
    """The stem convolution on the MFMA stem kernel with the stem BatchNorm's statistics partials in its
    epilogue (no statistics pass over the 112x112x64 output); backward as :class:`_StemConvFn`."""

    @staticmethod
    def forward(ctx, x, weight, kshift):
        from .._native import submodule

        y, part = submodule("conv_cuda").stem_forward_stats(x, weight, kshift)
        ctx.save_for_backward(x, weight)
        ctx.mode = "gemm"
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, gy, _gpart):
        gx, gw, _ = _StemConvFn.backward(ctx, gy)
        return gx, gw, None


class _GlobalAvgPoolFn(torch.autograd.Function):
    """Global average pool of a channels_last activation to [N, C]. Backward writes the broadcast
    gradient straight into a channels_last tensor (one pass): nn.AdaptiveAvgPool2d's backward produced
    an NCHW gradient that the BatchNorm backward then copied to channels_last twice."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        if g.is_cuda and g.dtype in (torch.float16, torch.bfloat16) and c % 8 == 0:
            from .._native import submodule

            return submodule("conv_bn").pool_broadcast(g.contiguous(), h, w, 1.0 / (h * w))
        return (g / (h * w)).view(n, c, 1, 1).expand(n, c, h, w).contiguous(memory_format=torch.channels_last)


def _tr(t):
    """``t.t().contiguous()`` of a 2-D tensor; 16-bit GPU tensors through the LDS-tiled transpose kernel
    (gemm.transpose: torch's strided copy took ~9 us per ResNet-50 weight)."""
    if t.is_cuda and t.dtype in (torch.float16, torch.bfloat16) and t.is_contiguous() and t.size(0) % 8 == 0 \
            and t.size(1) % 8 == 0:
        from .._native import submodule

        return submodule("gemm").transpose(t)
    return t.t().contiguous()


class _FcFn(torch.autograd.Function):
    """The classifier ``x W^T + b`` on the MFMA GEMM (kernels/gemm.hip, ``gemm.mm_nt``) in all three
    directions: one fixed kernel per shape, so every rank (and every run) computes it bitwise the
    same -- a library GEMM may pick a split-K / stream-K solution for these skinny shapes, whose
    accumulation order is not fixed. The class dimension is padded to a multiple of 8 with zero
    weight rows (10- or 1000-way heads); the transposed operands are small copies."""

    @staticmethod
    def forward(ctx, x, w, b):
        from .._native import submodule

        gm = submodule("gemm")
        n = w.size(0)
        n8 = (n + 7) // 8 * 8
        wp = w if n8 == n else torch.cat([w, w.new_zeros(n8 - n, w.size(1))])
        bp = None if b is None else (b if n8 == n else torch.cat([b, b.new_zeros(n8 - n)]))
        y = gm.mm_nt(x, wp, bp)
        ctx.save_for_backward(x, wp)
        ctx.n, ctx.has_b = n, b is not None
        return y[:, :n] if n8 != n else y

    @staticmethod
    def backward(ctx, gy):
        from .._native import submodule

        gm = submodule("gemm")
        x, wp = ctx.saved_tensors
        n, n8 = ctx.n, wp.size(0)
        gyp = gy.contiguous() if n8 == n else torch.cat([gy, gy.new_zeros(gy.size(0), n8 - n)], 1)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = gm.mm_nt(gyp, _tr(wp))  # dX = dY . W
        if ctx.needs_input_grad[1]:
            gw = gm.mm_nt(_tr(gyp), _tr(x))[:n]  # dW = dY^T . X
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = gy.float().sum(0).to(gy.dtype)
        return gx, gw, gb


def _fc_args(fc, x):
    """(weight, bias) in x's dtype for :class:`_FcFn` (amp O1 / O4: the 16-bit copies), or None."""
    if not (x.is_cuda and x.dim() == 2 and x.dtype in (torch.float16, torch.bfloat16) and x.size(0) % 8 == 0
            and x.size(1) % 8 == 0 and x.is_contiguous()):
        return None
    w = _kw(fc.weight, x)
    b = _kw(fc.bias, x) if fc.bias is not None else None
    if w is None or (fc.bias is not None and b is None):
        return None
    return w, b


class StemConv(nn.Conv2d):
    """nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False) with the MFMA stem forward (``mode``
    "auto" times it against MIOpen once, "gemm" forces it, "miopen" is plain nn.Conv2d)."""

    def __init__(self, *args, mode="auto", **kw):
        super().__init__(*args, **kw)
        self.mode = mode

    def forward(self, x):
        xk = _kx(x)
        w = _kw(self.weight, xk)
        if self.mode != "miopen" and x.is_cuda and w is not None:
            from ..ops import conv as bhconv

            if bhconv.stem_supported(xk, w):
                return _StemConvFn.apply(xk, w, self.mode)
        return super().forward(x)


class Conv1x1S2(nn.Conv2d):
    """nn.Conv2d(k=1, stride=2, bias=False): MIOpen forward / data gradient with the in-place
    stride-2 MFMA weight gradient (``_Conv1x1S2WFn``), or with ``gather=True`` the gathered-input
    GEMM path (``_Conv1x1S2Fn``)."""

    def __init__(self, *args, mode="auto", gather=False, **kw):
        super().__init__(*args, **kw)
        self.mode = mode
        self.gather = gather

    def forward(self, x):
        xk = _kx(x)
        w = _kw(self.weight, xk)
        if (x.is_cuda and self.mode != "miopen" and x.dim() == 4 and w is not None
                and xk.is_contiguous(memory_format=torch.channels_last) and x.size(2) % 2 == 0 and x.size(3) % 2 == 0):
            fn = _Conv1x1S2Fn if self.gather else _Conv1x1S2WFn
            return fn.apply(xk, w, self.mode)
        return super().forward(x)


def conv1x1(cin, cout, stride=1):
    if _CONV1X1_MODE != "miopen" and stride == 1:
        return Conv1x1(cin, cout, 1, stride=stride, bias=False, mode=_CONV1X1_MODE)
    # the gathered-input path is opt-in (BH_CONV1X1_S2=gather): measured 27.7 vs 26.4 ms per
    # ResNet-50 step on the same box, the strided gather / zero-fill + scatter cost more than
    # MIOpen's stride-2 kernels (profiles/resnet50_conv1x1_s2_ab.txt); BH_CONV1X1_S2=0 is plain MIOpen
    s2 = {"miopen": "0"}.get(_config.get().conv1x1_s2, _config.get().conv1x1_s2)
    if _CONV1X1_MODE != "miopen" and stride == 2 and s2 in ("wgrad", "gather"):
        return Conv1x1S2(cin, cout, 1, stride=2, bias=False, mode=_CONV1X1_MODE, gather=s2 == "gather")
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


# ------------------------------------------------------------------------------------------------
# BatchNorm folded into the convolutions (BH_FOLD_BN=1, default for the fused model): each conv's
# epilogue produces the statistics partials of the BatchNorm that follows it (no statistics pass),
# and the data gradient of each conv whose input came out of a BatchNorm(+ReLU) reduces that
# BatchNorm's backward sums in its epilogue (no backward-reduce pass). See kernels/conv_bn.hip and
# kernels/conv.hip (the 3x3 kernel's EPI variants).


def _kshift(bn):
    """The statistics centre shared by the conv epilogue and syncbn.merge_sums: the running mean."""
    rm = getattr(bn, "running_mean", None)
    return rm if rm is not None and rm.dtype == torch.float32 else None


def _part_from_tensor(y, kshift):
    """Fallback statistics partials ([2, 1, C]) from a statistics pass over y."""
    from ..ops import syncbn

    C = y.size(1)
    return syncbn.stats_local_sums(y, kshift)[:2 * C].view(2, 1, C)


def _link_ok(link, c):
    return link is not None and link.y is not None and link.y.size(1) == c


class _Conv1x1BNFn(torch.autograd.Function):
    """1x1 convolution (stride 1, or stride 2 read in place) of a channels_last activation whose
    epilogue emits the next BatchNorm's statistics partials; backward: data gradient with the
    previous BatchNorm's backward sums (``link_in``) and the parked residual gradient (``box``) in its
    epilogue, weight gradient on the MFMA wgrad kernel (or MIOpen, per shape)."""

    @staticmethod
    def forward(ctx, x, weight, kshift, link_in, box, s2, mlink=None):
        y, part = _c1x1_forward_stats(x, weight, kshift, s2)
        ctx.save_for_backward(x, weight)
        ctx.link_in, ctx.box, ctx.s2 = link_in, box, s2
        ctx.mlink = mlink  # the producing block's ReLU mask (_MaskLink): applied in the data gradient's epilogue
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, gy, _gpart):
        from ..ops import conv as bhconv
        from ..ops import conv_bn

        x, weight = ctx.saved_tensors
        n, c, h, w = x.shape
        k = weight.size(0)
        gy = gy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        st = 2 if ctx.s2 else 1
        args = ([st, st], [0, 0], [1, 1], False, [0, 0], 1)
        box = ctx.box
        acc = box.pop("g", None) if box is not None else None
        if acc is not None and not (acc.is_contiguous(memory_format=torch.channels_last) and acc.dtype == gy.dtype
                                    and acc.shape == x.shape):
            acc = acc.contiguous(memory_format=torch.channels_last).to(gy.dtype)
        gx = gw = None

        def wfn():
            if ctx.s2:
                return (_conv_wgrad(x, gy, 1, weight, stride=2) if bhconv.wgrad_supported(x, gy, 1, 2) else
                        _like(conv_bwd(gy, x, weight, None, *args, [False, True, False])[1], weight))
            # the MFMA wgrad kernel wins every ResNet-50 1x1 shape (profiles/conv_wgrad_vs_miopen.jsonl):
            # no per-shape timing (it would JIT-compile MIOpen's solver on the first step)
            return _wgrad(x, gy, weight, 1, "gemm", lambda: conv_bwd(gy, x, weight, None, *args,
                                                                     [False, True, False])[1])

        if ctx.needs_input_grad[0]:
            if ctx.s2:
                gx = conv_bwd(gy, x, weight, None, *args, [True, False, False])[0]
                if acc is not None:
                    gx = gx + acc
            else:
                gy2d = gy.permute(0, 2, 3, 1).reshape(-1, k)
                w2d = weight.view(k, c)  # dX = dY . W: the strip kernel reads W as the [K, N] operand
                r2d = acc.permute(0, 2, 3, 1).reshape(-1, c) if acc is not None else None
                link = ctx.link_in
                fast = conv_bn.preferred(k, c, gy2d.size(0))
                ml = ctx.mlink
                if ml is not None and conv_bn.supported(gy2d, w2d, resid=r2d is not None, epi="mask", b_trans=True) \
                        and (fast or _MASK_PRODUCER_ANY):
                    # dX = dY . W (+ the parked residual gradient), masked by the previous block's output ReLU,
                    # with its column sums: that block's tail (_ConvBNResFn) skips its mask pass
                    gx2d, part = conv_bn.c1x1(gy2d, w2d, resid=r2d, epi="mask", mbits=ml.bits, b_trans=True)
                    ml.sg, ml.ptr, ml.ver = part[0], gx2d.data_ptr(), gx2d._version
                elif fast and _link_ok(link, c) and conv_bn.supported(gy2d, w2d, resid=r2d is not None, epi="bwd",
                                                                      b_trans=True):
                    y2d = link.y.permute(0, 2, 3, 1).reshape(-1, c)
                    gx2d, part = conv_bn.c1x1(gy2d, w2d, resid=r2d, epi="bwd", by=y2d, bscale=link.scale,
                                              bshift=link.shift, bmean=link.mean, brelu=link.relu, b_trans=True)
                    link.take_part(part)
                elif fast and conv_bn.supported(gy2d, w2d, resid=r2d is not None, b_trans=True):
                    gx2d, _ = conv_bn.c1x1(gy2d, w2d, resid=r2d, b_trans=True)
                elif _own("resid" if r2d is not None else ("bwd" if _link_ok(link, c) else "plain")) and \
                        conv_bn.gemm_bn_supported(gy2d, w2d.t(), resid=r2d is not None):
                    # the tiled MFMA GEMM: dX = dY . W (+ the parked residual gradient), with the previous
                    # BatchNorm's backward sums in its epilogue when that BatchNorm is linked
                    wt = _tr(w2d)
                    if _link_ok(link, c):
                        y2d = link.y.permute(0, 2, 3, 1).reshape(-1, c)
                        gx2d, part = conv_bn.gemm_bn(gy2d, wt, "bwd", by=y2d, bscale=link.scale, bshift=link.shift,
                                                     bmean=link.mean, brelu=link.relu, resid=r2d)
                        link.take_part(part)
                    else:
                        gx2d, _ = conv_bn.gemm_bn(gy2d, wt, "plain", resid=r2d)
                elif r2d is not None:  # beta = 1 into the parked residual gradient (no output copy)
                    gx2d = torch.addmm(r2d, gy2d, w2d, out=r2d)
                else:
                    gx2d = torch.mm(gy2d, w2d)
                gx = gx2d.view(n, h, w, c).permute(0, 3, 1, 2)
            acc = None
        if box is not None:
            box["conv_done"] = True
        if ctx.needs_input_grad[1]:
            gw = wfn()
        return gx, gw, None, None, None, None, None


def _c1x1_forward_stats(x, weight, kshift, s2):
    """Raw 1x1 conv output (channels_last) + its BatchNorm statistics partials: the strip kernel where
    it wins, else hipBLASLt on the [pixels, channels] view (a gathered quarter of x for stride 2) +
    a statistics pass. Never MIOpen (whose first call JIT-compiles its kernels)."""
    from ..ops import conv_bn

    n, c, h, w = x.shape
    k = weight.size(0)
    a2d = x.permute(0, 2, 3, 1).reshape(-1, c)
    w2d = weight.view(k, c)
    ho, wo = (h // 2, w // 2) if s2 else (h, w)
    hw = (h, w) if s2 else None
    if conv_bn.preferred(c, k, n * ho * wo, s2) and conv_bn.supported(a2d, w2d, s2=hw, epi="stats"):
        y2d, part = conv_bn.c1x1(a2d, w2d, s2=hw, epi="stats", kshift=kshift)
        return y2d.view(n, ho, wo, k).permute(0, 3, 1, 2), part
    if s2:
        a2d = conv_bn.s2_gather(x).permute(0, 2, 3, 1).reshape(-1, c)
    if _own("fwd") and conv_bn.gemm_bn_supported(a2d, w2d) and not (c <= 256 and k >= 1024):
        # the MFMA-bound layers (K or N >= 512, or the small 14x14 / 7x7 grids): the tiled MFMA GEMM
        # with the statistics epilogue (kernels/gemm.hip; the ping-pong 256x256 kernel from 160 tiles),
        # no library GEMM and no separate statistics pass (benchmarks/bench_resnet_gemms.py). Not the
        # K <= 256 -> N >= 1024 expansions (stage-3 conv3): four K-steps, the epilogue dominates the
        # one-workgroup-per-CU tile (67 vs 57 us for hipBLASLt + the statistics pass in the step)
        y2d, part = conv_bn.gemm_bn(a2d, w2d, "stats", kshift=kshift)
        return y2d.view(n, ho, wo, k).permute(0, 3, 1, 2), part
    y = torch.mm(a2d, w2d.t()).view(n, ho, wo, k).permute(0, 3, 1, 2)
    return y, _part_from_tensor(y, kshift)


class _Conv1DsFn(torch.autograd.Function):
    """The first 1x1 convolution of a bottleneck and its downsample 1x1 (stride 1 or 2), both reading
    the block input x, as ONE autograd node: each emits the statistics partials of its BatchNorm, and
    the backward produces dX = dY1 . W1 and then ADDS the downsample's data gradient into it in place
    -- at the even pixels only for stride 2 (scatter-accumulate epilogue) -- instead of materialising a
    zero-filled full-resolution gradient and summing the two branches (MIOpen's stride-2 backward-data
    plus an add). Weight gradients on the MFMA wgrad kernels."""

    @staticmethod
    def forward(ctx, x, w1, wd, k1, kd, s2, ds_box=None):
        y1, p1 = _c1x1_forward_stats(x, w1, k1, False)
        yd, pd = _c1x1_forward_stats(x, wd, kd, s2)
        ctx.save_for_backward(x, w1, wd)
        ctx.s2 = s2
        # ds_box: filled by the block's tail (_ConvBNResFn) when it folds the downsample BatchNorm: the
        # downsample conv's weight gradient is then the tail's, and its data gradient is formed here from
        # (g, y_ds, A, B, D) with the BatchNorm-backward prologue
        ctx.ds_box = ds_box
        ctx.mark_non_differentiable(p1, pd)
        ctx.set_materialize_grads(False)
        return y1, p1, yd, pd

    @staticmethod
    def backward(ctx, gy1, _g1, gyd, _gd):
        from ..ops import conv as bhconv
        from ..ops import conv_bn

        x, w1, wd = ctx.saved_tensors
        n, c, h, w = x.shape
        k1, kd = w1.size(0), wd.size(0)
        gy1 = gy1.contiguous(memory_format=torch.channels_last)
        if gyd is not None:  # (None: the tail folded the downsample BatchNorm, see ds_box)
            gyd = gyd.contiguous(memory_format=torch.channels_last)
            gd = gyd.permute(0, 2, 3, 1).reshape(-1, kd)
        g1 = gy1.permute(0, 2, 3, 1).reshape(-1, k1)
        w1_2d, wd_2d = w1.view(k1, c), wd.view(kd, c)
        gx = gw1 = gwd = None
        conv_bwd = torch.ops.aten.convolution_backward
        a1 = ([1, 1], [0, 0], [1, 1], False, [0, 0], 1)

        def w1fn():
            return _wgrad(x, gy1, w1, 1, "gemm", lambda: conv_bwd(gy1, x, w1, None, *a1, [False, True, False])[1])

        def wdfn():
            if ctx.s2:
                a2 = ([2, 2], [0, 0], [1, 1], False, [0, 0], 1)
                return (_conv_wgrad(x, gyd, 1, wd, stride=2) if bhconv.wgrad_supported(x, gyd, 1, 2) else
                        _like(conv_bwd(gyd, x, wd, None, *a2, [False, True, False])[1], wd))
            return _wgrad(x, gyd, wd, 1, "gemm", lambda: conv_bwd(gyd, x, wd, None, *a1, [False, True, False])[1])

        dsb = ctx.ds_box.pop("ds", None) if ctx.ds_box is not None else None
        if ctx.needs_input_grad[0]:
            if conv_bn.preferred(k1, c, g1.size(0)) and conv_bn.supported(g1, w1_2d, b_trans=True):
                gx2d, _ = conv_bn.c1x1(g1, w1_2d, b_trans=True)
            elif _own("plain") and conv_bn.gemm_bn_supported(g1, w1_2d.t()):
                gx2d, _ = conv_bn.gemm_bn(g1, _tr(w1_2d), "plain")
            else:
                gx2d = torch.mm(g1, w1_2d)
            if dsb is not None:
                gx2d = _ds_dgrad_folded(gx2d, dsb, ctx.s2, (n, c, h, w))
            elif ctx.s2:
                # the scatter epilogue wins only where the strip kernel does (K = downsample channels
                # <= 256); else hipBLASLt + a strided add over the quarter of the pixels
                if conv_bn.preferred(kd, c, gd.size(0)) and \
                        conv_bn.supported(gd, wd_2d, b_trans=True, s2=(h, w), s2_scatter=True):
                    conv_bn.c1x1(gd, wd_2d, b_trans=True, s2=(h, w), s2_scatter=True, resid=gx2d)
                else:
                    if _own("plain") and conv_bn.gemm_bn_supported(gd, wd_2d.t()):
                        gdx = conv_bn.gemm_bn(gd, _tr(wd_2d), "plain")[0]
                    else:
                        gdx = torch.mm(gd, wd_2d)
                    conv_bn.s2_scatter_add(gx2d, gdx, n, h, w)
            elif conv_bn.preferred(kd, c, gd.size(0)) and conv_bn.supported(gd, wd_2d, resid=True, b_trans=True):
                gx2d, _ = conv_bn.c1x1(gd, wd_2d, resid=gx2d, b_trans=True)
            elif _own("resid") and conv_bn.gemm_bn_supported(gd, wd_2d.t(), resid=True):
                gx2d, _ = conv_bn.gemm_bn(gd, _tr(wd_2d), "plain", resid=gx2d)
            else:
                torch.addmm(gx2d, gd, wd_2d, out=gx2d)
            gx = gx2d.view(n, h, w, c).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            gw1 = w1fn()
        if ctx.needs_input_grad[2] and dsb is None:
            gwd = wdfn()
        return gx, gw1, gwd, None, None, None, None


def _ds_dgrad_folded(gx2d, dsb, s2, shape):
    """conv1's data gradient gx2d plus the downsample convolution's (gx_ds @ W_ds, gx_ds = A g + B y_ds + D:
    the folded downsample BatchNorm's input gradient, never written): the strip kernel's BatchNorm-backward
    prologue with gx2d as the residual (scatter-accumulated in place at the even pixels for stride 2), else
    gx_ds formed in a pass and a library GEMM. Returns the sum (gx2d itself where accumulated in place)."""
    from ..ops import conv_bn

    from ..ops import syncbn

    n, c, h, w = shape
    g2d, abd, y2d, Wd, bn_args = dsb  # g2d / y2d: [M_ds, kd]; Wd: [kd, c]; bn_args: the BatchNorm's own terms
    kd = Wd.size(0)
    if s2:
        if conv_bn.supported(g2d, Wd, b_trans=True, s2=(h, w), s2_scatter=True, bnb=True):
            return conv_bn.c1x1(g2d, Wd, b_trans=True, bnb=abd, bnb_y=y2d, s2=(h, w), s2_scatter=True, resid=gx2d)[0]
    elif conv_bn.supported(g2d, Wd, resid=True, b_trans=True, bnb=True):
        return conv_bn.c1x1(g2d, Wd, b_trans=True, bnb=abd, bnb_y=y2d, resid=gx2d)[0]
    g4, y4, mean, invstd, weight, sums, count = bn_args
    gxd = syncbn.backward_dgrad(g4, y4, None, mean, invstd, weight, sums, count, None, None, False, False, None)[0]
    gxd = gxd.permute(0, 2, 3, 1).reshape(-1, kd)
    if s2:
        return conv_bn.s2_scatter_add(gx2d, torch.mm(gxd, Wd), n, h, w)
    return torch.addmm(gx2d, gxd, Wd, out=gx2d)


class _Conv3x3BNFn(torch.autograd.Function):
    """3x3 / stride-1 convolution on the direct MFMA kernel with the next BatchNorm's statistics in
    its epilogue; backward: data gradient (flipped-weight kernel) with the previous BatchNorm's
    backward sums in its epilogue, weight gradient on the MFMA wgrad kernel."""

    @staticmethod
    def forward(ctx, x, weight, kshift, link_in):
        from .._native import submodule

        y, part = submodule("conv_cuda").conv3x3_bn_forward(x, weight, None, None, True, kshift)
        ctx.save_for_backward(x, weight)
        ctx.link_in = link_in
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, gy, _gpart):
        from .._native import submodule
        from ..ops import conv as bhconv
        from ..ops import conv_bn

        x, weight = ctx.saved_tensors
        c = x.size(1)
        gy = gy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = ([1, 1], [1, 1], [1, 1], False, [0, 0], 1)
        gx = gw = None
        wfn = lambda: _wgrad(x, gy, weight, 3, "gemm",  # noqa: E731
                             lambda: conv_bwd(gy, x, weight, None, *args, [False, True, False])[1])
        if ctx.needs_input_grad[0]:
            # (a BatchNorm-sums epilogue on the 3x3 data gradient measured slower than the separate
            # reduce pass at 56x56 -- 170 vs 104 + 50 us -- and was removed)
            gx = bhconv.conv3x3_dgrad(gy, weight)
        if ctx.needs_input_grad[1]:
            gw = wfn()
        return gx, gw, None, None


class _BNConvFn(torch.autograd.Function):
    """A training-mode (Sync)BatchNorm + ReLU whose output only feeds the next convolution, folded into
    that convolution: the BatchNorm is never applied as a pass. Forward: the producing convolution's
    statistics partials -> (one all-reduce across ranks) -> mean / invstd / scale / shift + running
    stats, then the convolution reads the raw input y and applies relu(y * scale + shift) to its staged
    tiles (the 3x3 direct kernel's halo prologue, or the 1x1 strip GEMM's A-fragment prologue) and
    emits the NEXT BatchNorm's statistics partials. Backward: the convolution's data gradient dA (for a
    1x1 layer with this BatchNorm's backward sums in its epilogue), its weight gradient from the same
    prologue applied to the LDS tiles of the wgrad kernel, then the BatchNorm backward from (dA, y) with
    the ReLU mask recomputed from y. Same parameters, running statistics and gradients as
    ``bn(y) -> relu -> conv``; one full read + write of the activation less per direction."""

    @staticmethod
    def forward(ctx, y, part, bn_w, bn_b, running_mean, running_var, eps, momentum, process_group, num_batches,
                conv_w, kshift_out, R, stride=1):
        from ..ops import conv_bn
        from ..ops import syncbn
        from ..parallel.optimized_sync_batchnorm import _all_reduce, _world
        from ..parallel import comm_stats
        from .._native import submodule

        world = _world(process_group)
        C = y.size(1)
        count = float(y.numel() // C)
        bumped = world == 1 and momentum >= 0
        if world > 1:
            sums = conv_bn.sum_parts(part, count)
            with comm_stats.timed("syncbn_fwd", sums):
                _all_reduce(sums, process_group)
            mean, invstd, scale, shift, count_t = syncbn.merge_sums(sums, bn_w, bn_b, running_mean, running_var,
                                                                    momentum, eps, num_batches)
        else:  # one launch; with a fixed momentum it also bumps num_batches_tracked
            mean, invstd, scale, shift, count_t = syncbn.merge_parts(part, count, bn_w, bn_b, running_mean,
                                                                     running_var, momentum, eps, num_batches, bumped)
        if num_batches is not None and not bumped:
            num_batches.add_(1)  # (the normalisation pass would have bumped it)
        if R == 3 and stride == 2:  # the downsampling 3x3 on the implicit-GEMM kernel
            out, part_out = submodule("conv_cuda").conv3x3_s2_forward(y, conv_w, scale, shift, True, kshift_out)
        elif R == 3:
            out, part_out = submodule("conv_cuda").conv3x3_bn_forward(y, conv_w, scale, shift, True, kshift_out)
        else:
            n, _, h, w = y.shape
            k = conv_w.size(0)
            o2d, part_out = conv_bn.c1x1(y.permute(0, 2, 3, 1).reshape(-1, C), conv_w.view(k, C), pro_scale=scale,
                                         pro_shift=shift, epi="stats", kshift=kshift_out)
            out = o2d.view(n, h, w, k).permute(0, 3, 1, 2)
        ctx.save_for_backward(y, conv_w, bn_w, mean, invstd, scale, shift, count_t)
        ctx.process_group, ctx.world, ctx.R, ctx.stride = process_group, world, R, stride
        ctx.mark_non_differentiable(part_out)
        ctx.set_materialize_grads(False)
        return out, part_out

    @staticmethod
    def backward(ctx, gy, _gpart):
        from ..ops import conv as bhconv
        from ..ops import conv_bn
        from ..ops import syncbn
        from ..parallel.optimized_sync_batchnorm import _all_reduce_async
        from ..parallel import comm_stats

        y, conv_w, bn_w, mean, invstd, scale, shift, count = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        n, C, h, w = y.shape
        part = None
        wfn = lambda: _conv_wgrad(y, gy, ctx.R, conv_w, scale, shift, stride=ctx.stride)  # noqa: E731
        g_conv = None
        if ctx.R == 3 and ctx.stride == 2:
            dA = bhconv.conv3x3_s2_dgrad(gy, conv_w, (h, w))
        elif ctx.R == 3 and _config.get().conv3x3_bwd_epi and gy.dtype in (torch.float16, torch.bfloat16) \
                and C % 64 == 0 and conv_w.size(0) % 64 == 0 and y.is_contiguous(memory_format=torch.channels_last):
            # the direct kernel's backward epilogue: this BatchNorm's backward sums from the data gradient as
            # it leaves the accumulators (no k_bwd_reduce pass over dA and y)
            from .._native import submodule

            dA, part = submodule("conv_cuda").conv3x3_bn_dgrad(gy, conv_w, y, scale, shift, mean, True)
        elif ctx.R == 3:
            dA = bhconv.conv3x3_dgrad(gy, conv_w)
        else:
            k = conv_w.size(0)
            gy2d = gy.permute(0, 2, 3, 1).reshape(-1, k)
            w2d = conv_w.view(k, C)
            y2d = y.permute(0, 2, 3, 1).reshape(-1, C)
            if conv_bn.preferred(k, C, gy2d.size(0)) and conv_bn.supported(gy2d, w2d, epi="bwd", b_trans=True):
                # the strip GEMM with this BatchNorm's backward sums in its epilogue (where it beats hipBLASLt)
                dA2d, part = conv_bn.c1x1(gy2d, w2d, epi="bwd", by=y2d, bscale=scale, bshift=shift, bmean=mean,
                                          brelu=True, b_trans=True)
            elif _own("bwd") and conv_bn.gemm_bn_supported(gy2d, w2d.t()):
                dA2d, part = conv_bn.gemm_bn(gy2d, _tr(w2d), "bwd", by=y2d, bscale=scale, bshift=shift,
                                             bmean=mean, brelu=True)
            else:
                dA2d = torch.mm(gy2d, w2d)
            dA = dA2d.view(n, h, w, C).permute(0, 3, 1, 2)
        need_w = bn_w is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        if part is None:
            sums, gw, gb = syncbn.backward_reduce(dA, y, None, mean, invstd, scale, shift, True, bn_w, need_w, None)
        else:
            # gb a separate tensor: `sums` is all-reduced in place below, the bias gradient stays this rank's own
            sums, gw, gb = conv_bn.sum_parts_grads(part, invstd, bn_w, need_w)
        # the cross-rank exchange of the BatchNorm's backward sums runs (IPC side stream / async RCCL)
        # while the convolution's weight gradient -- which does not depend on it -- computes
        pending = _all_reduce_async(sums, ctx.process_group) if ctx.world > 1 else None
        if ctx.needs_input_grad[10]:
            g_conv = wfn()
        if pending is not None:
            with comm_stats.timed("syncbn_bwd", sums):
                pending.wait()
        gx, _ = syncbn.backward_dgrad(dA, y, None, mean, invstd, bn_w, sums, count, scale, shift, True, False, None)
        return gx, None, (gw if need_w else None), (gb if need_w else None), None, None, None, None, None, None, \
            g_conv, None, None, None


class _MaskLink(object):
    """Hands a residual block's saved ReLU bit mask to the node that produces the gradient of that block's
    output (the next block's conv1 data gradient): it applies the mask in its epilogue and leaves the column
    sums there (``sg``), and records the tensor it wrote (``ptr``) and that tensor's version counter (``ver``)
    so the block's backward can tell that the gradient it receives is exactly that one: a second consumer of
    the block output (a feature tap, a hook, an auxiliary head) makes autograd's InputBuffer accumulate into
    the same storage in place, which keeps the pointer but bumps the version."""

    __slots__ = ("bits", "ptr", "ver", "sg", "__weakref__")

    def __init__(self, bits):
        self.bits, self.ptr, self.ver, self.sg = bits, None, None, None


class _FoldCfg(object):
    """Non-tensor arguments of :class:`_ConvBNResFn`: the BatchNorm modules (running statistics,
    momentum, eps, process group) and the link of an unfolded bn2."""

    __slots__ = ("bn_in", "bn_out", "link_in", "bn_ds", "ds_box", "ds_s2")

    def __init__(self, bn_in, bn_out, link_in, bn_ds=None, ds_box=None, ds_s2=False):
        self.bn_in, self.bn_out, self.link_in = bn_in, bn_out, link_in
        # downsampling block: the downsample BatchNorm (its input y_ds comes in as `yd`), the box through which
        # the downsample conv's data-gradient inputs go to _Conv1DsFn, and its stride
        self.bn_ds, self.ds_box, self.ds_s2 = bn_ds, ds_box, ds_s2


def _bn_finalize(bn, part, count, world, bump_in_merge):
    """Partials of a conv epilogue -> (mean, invstd, scale, shift, count) of the training BatchNorm ``bn``
    (running statistics updated; one all-reduce across ranks). ``bump_in_merge``: the merge kernel also
    advances num_batches_tracked (fixed momentum, one rank); else the caller's normalisation pass does."""
    from ..ops import conv_bn
    from ..ops import syncbn
    from ..parallel.optimized_sync_batchnorm import _all_reduce
    from ..parallel import comm_stats

    mom = bn.momentum if bn.momentum is not None else -1.0
    if world > 1:
        sums = conv_bn.sum_parts(part, count)
        with comm_stats.timed("syncbn_fwd", sums):
            _all_reduce(sums, bn.process_group)
        return syncbn.merge_sums(sums, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps,
                                 bn.num_batches_tracked)
    return syncbn.merge_parts(part, count, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps,
                              bn.num_batches_tracked, bump_in_merge)


class _ConvBNResFn(torch.autograd.Function):
    """The tail of a bottleneck as ONE node: [bn2 + ReLU folded into the prologue] -> conv3 (1x1) -> bn3 ->
    + z -> ReLU, whose backward never touches conv3's output y or bn3's input gradient (ops/bn_fold.py):

    forward: conv3 (strip / tiled GEMM with bn3's statistics in the epilogue) -> merge -> one pass
      out = relu(bn3(y) + z) that also stores the 1-bit ReLU mask. y is NOT saved.
    backward, from g_out: g = mask * g_out with its column sums (one pass; g is also z's gradient) ->
      P = g^T a (the weight-gradient kernel, fp32) and Gm = a^T a (Gram kernel over the 4x narrower a) ->
      bn3's sums, dW3, dgamma3, dbeta3 from small matrices -> da = g @ Wa (GEMM) + a @ H + c (strip kernel,
      with bn2's backward sums in its epilogue) -> bn2's data gradient (folded case).
    Replaces bn3's backward-reduce and data-gradient passes over the [M, N] tensors (two reads of g_out and y,
    writes of gx and dz) and the reads of gx by conv3's data and weight gradients.

    ``src``: bn2's raw input y2 (``cfg.bn_in`` given: bn2 + ReLU in conv3's prologue) or the materialised a2
    (``cfg.link_in``: the unfolded bn2's link, its backward sums come from the data-gradient epilogue)."""

    @staticmethod
    def forward(ctx, src, p_src, w3, bn_in_w, bn_in_b, bn_w, bn_b, z, cfg, yd=None, pd=None, xd=None, wd=None,
                bnd_w=None, bnd_b=None):
        from ..ops import conv_bn
        from ..ops import syncbn
        from ..parallel.optimized_sync_batchnorm import _world

        bn_in, bn = cfg.bn_in, cfg.bn_out
        world = _world(bn.process_group)
        n, K, h, w = src.shape
        N = w3.size(0)
        M = n * h * w
        src2d = src.permute(0, 2, 3, 1).reshape(-1, K)
        pro = None
        if bn_in is not None:
            nb_in = bn_in.num_batches_tracked
            bumped = world == 1 and bn_in.momentum is not None
            mean_i, invstd_i, scale_i, shift_i, count_i = _bn_finalize(bn_in, p_src, float(M), world, bumped)
            if nb_in is not None and not bumped:
                nb_in.add_(1)
            pro = (scale_i, shift_i)
            y2d, part = conv_bn.c1x1(src2d, w3.view(N, K), pro_scale=scale_i, pro_shift=shift_i, epi="stats",
                                     kshift=_kshift(bn))
            y = y2d.view(n, h, w, N).permute(0, 3, 1, 2)
        else:
            mean_i = invstd_i = scale_i = shift_i = count_i = None
            y, part = _c1x1_forward_stats(src, w3, _kshift(bn), False)
        mean, invstd, scale, shift, count = _bn_finalize(bn, part, float(M), world, False)
        ds = cfg.bn_ds
        if ds is not None:
            # downsampling block: the downsample BatchNorm is normalised inside the residual pass
            # (relu(bn3(y) + bn_ds(y_ds)): no normalised identity tensor) and its backward folded too
            nb_d = ds.num_batches_tracked
            bumped_d = world == 1 and ds.momentum is not None
            mean_d, invstd_d, scale_d, shift_d, count_d = _bn_finalize(ds, pd, float(M), world, bumped_d)
            if nb_d is not None and not bumped_d:
                nb_d.add_(1)
            out, bits = syncbn.forward_mask(y, yd, scale, shift, bn.num_batches_tracked, scale_d, shift_d)
        else:
            mean_d = invstd_d = count_d = None
            out, bits = syncbn.forward_mask(y, z, scale, shift, bn.num_batches_tracked)
        ctx.save_for_backward(src, w3, y, bn_w, mean, invstd, count, bits, bn_in_w, mean_i, invstd_i, scale_i,
                              shift_i, count_i, yd, xd, wd, bnd_w, mean_d, invstd_d, count_d)
        ctx.cfg, ctx.world, ctx.pro = cfg, world, pro is not None
        ctx.mlink = _MaskLink(bits) if _MASK_PRODUCER else None
        if ctx.mlink is not None:
            out._bh_mask = ctx.mlink  # read by the next block's conv1 (its data gradient masks for us)
        ctx.mark_non_differentiable(bits)
        return out

    @staticmethod
    def backward(ctx, g_out):
        from ..ops import bn_fold
        from ..ops import conv_bn
        from ..ops import syncbn
        from ..parallel.optimized_sync_batchnorm import _all_reduce_async
        from ..parallel import comm_stats

        src, w3, y, bn_w, mean, invstd, count, bits, bn_in_w, mean_i, invstd_i, scale_i, shift_i, count_i, \
            yd, xd, wd, bnd_w, mean_d, invstd_d, count_d = ctx.saved_tensors
        cfg = ctx.cfg
        n, K, h, w = src.shape
        N = w3.size(0)
        g_out = g_out.contiguous(memory_format=torch.channels_last)
        ml = ctx.mlink
        if ml is not None and ml.ptr is not None and ml.ptr == g_out.data_ptr() and ml.sg is not None \
                and ml.ver == g_out._version:
            # the producer already applied the mask and summed the columns (and nothing was added since)
            g2d, sg_ws = g_out.permute(0, 2, 3, 1).reshape(-1, N), ml.sg
        else:  # (masking is idempotent: a gradient summed from a masked and an unmasked part is handled too)
            g2d, sg_ws = bn_fold.mask_colsum_partials(g_out.permute(0, 2, 3, 1).reshape(-1, N), bits)
        if ml is not None:
            ml.ptr = ml.sg = ml.ver = None
        g = g2d.view(n, h, w, N).permute(0, 3, 1, 2)  # bn3's masked output gradient = z's gradient
        W = w3.view(N, K)
        ps, ph = (scale_i, shift_i) if ctx.pro else (None, None)
        src2d = src.permute(0, 2, 3, 1).reshape(-1, K)
        # conv3's weight gradient and bn3's sums from P = g^T a and the Gram matrix of a (ops/bn_fold.py)
        p_ws = bn_fold.wgrad_partials(src, g, ps, ph)
        g_ws, sa_ws = bn_fold.gram_partials(src2d, ps, ph)
        P, Gm, Sa, sums, bn_grads = bn_fold.fold_reduce(W, p_ws, g_ws, sa_ws, sg_ws, mean, invstd)
        need_bn = bn_w is not None and (ctx.needs_input_grad[5] or ctx.needs_input_grad[6])
        gw = bn_grads[:N].to(bn_w.dtype) if need_bn else None  # this rank's own (bn_grads is not all-reduced)
        gb = bn_grads[N:].to(bn_w.dtype) if need_bn else None
        if ctx.world > 1:
            with comm_stats.timed("syncbn_bwd", sums):
                _all_reduce_async(sums, cfg.bn_out.process_group).wait()
        dW, abd = bn_fold.fold_finish(W, sums, count, mean, invstd, bn_w, P, Gm, Sa)
        gw3 = dW.view(N, K, 1, 1)
        if gw3.stride() != w3.stride():
            gw3 = gw3.contiguous(memory_format=torch.channels_last)
        gwd = gw_d = gb_d = None
        if cfg.bn_ds is not None:
            # the downsample BatchNorm after the 1x1 (stride 1 or 2) downsample conv of the block input x: the
            # same algebra on (g, x) -- dW_ds and its sums from P_ds = g^T x_s and the Gram matrix of x_s
            # (the even pixels at stride 2); its data gradient is formed in _Conv1DsFn from (g, y_ds, A, B, D)
            Cin = xd.size(1)
            Wd = wd.view(N, Cin)
            st = 2 if cfg.ds_s2 else 1
            p_ws_d = bn_fold.wgrad_partials(xd, g, None, None, st)
            g_ws_d, sa_ws_d = bn_fold.gram_partials(xd.permute(0, 2, 3, 1).reshape(-1, Cin), None, None,
                                                    (xd.size(2), xd.size(3)) if cfg.ds_s2 else None)
            P_d, Gm_d, Sa_d, sums_d, bn_grads_d = bn_fold.fold_reduce(Wd, p_ws_d, g_ws_d, sa_ws_d, sg_ws, mean_d,
                                                                     invstd_d)
            need_d = bnd_w is not None and (ctx.needs_input_grad[13] or ctx.needs_input_grad[14])
            gw_d = bn_grads_d[:N].to(bnd_w.dtype) if need_d else None
            gb_d = bn_grads_d[N:].to(bnd_w.dtype) if need_d else None
            if ctx.world > 1:
                with comm_stats.timed("syncbn_bwd", sums_d):
                    _all_reduce_async(sums_d, cfg.bn_ds.process_group).wait()
            dWd, abd_d = bn_fold.fold_finish(Wd, sums_d, count_d, mean_d, invstd_d, bnd_w, P_d, Gm_d, Sa_d)
            gwd = dWd.view(N, Cin, 1, 1)
            if gwd.stride() != wd.stride():
                gwd = gwd.contiguous(memory_format=torch.channels_last)
            cfg.ds_box["ds"] = (g2d, abd_d, yd.permute(0, 2, 3, 1).reshape(-1, N), Wd,
                                (g, yd, mean_d, invstd_d, bnd_w, sums_d, count_d))
        # conv3's data gradient gx3 @ W3, gx3 = A g + B y + D: formed per fragment inside the strip GEMM where
        # it runs, else one elementwise pass; the previous BatchNorm's backward sums in the epilogue
        y2d = y.permute(0, 2, 3, 1).reshape(-1, N)
        M = g2d.size(0)
        if ctx.pro:
            lk = (src2d, scale_i, shift_i, mean_i, True)
        elif _link_ok(cfg.link_in, K):
            l = cfg.link_in
            lk = (l.y.permute(0, 2, 3, 1).reshape(-1, K), l.scale, l.shift, l.mean, l.relu)
        else:
            lk = None
        s_i = part_i = None
        epi = "bwd" if lk is not None else "plain"
        kw = dict(epi=epi, by=lk[0], bscale=lk[1], bshift=lk[2], bmean=lk[3], brelu=lk[4]) if lk else {}
        nseg = _bnb_segments(g2d, W, epi)
        if nseg == 1:
            da2d, part = conv_bn.c1x1(g2d, W, b_trans=True, bnb=abd, bnb_y=y2d, **kw)
            if lk is not None:
                part_i = part
        elif nseg > 1:
            # split-K: the strip kernel keeps its B slice in LDS, so a wide gradient runs as column segments
            # accumulated through the residual input; the BatchNorm-backward sums come with the last one.
            # The segments' (A, B, D) constants regrouped by one copy: [nseg][3][Ks]
            Ks = N // nseg
            abd_seg = abd.view(3, nseg, Ks).permute(1, 0, 2).contiguous()
            da2d = None
            for sgi in range(nseg):
                cols = slice(sgi * Ks, (sgi + 1) * Ks)
                last = sgi == nseg - 1
                da2d, part = conv_bn.c1x1(g2d[:, cols], W[cols], b_trans=True, bnb=abd_seg[sgi].reshape(-1),
                                          bnb_y=y2d[:, cols], lda=N, resid=da2d, **(kw if last else {}))
            if lk is not None:
                part_i = part
        else:
            gx3, _ = syncbn.backward_dgrad(g, y, None, mean, invstd, bn_w, sums, count, None, None, False, False, None)
            gx3 = gx3.permute(0, 2, 3, 1).reshape(-1, N)
            da2d, s_i = _dgrad_bn_sums(gx3, W, lk)
        da = da2d.view(n, h, w, K).permute(0, 3, 1, 2)
        gw_i = gb_i = None
        if ctx.pro:
            need_i = bn_in_w is not None and (ctx.needs_input_grad[3] or ctx.needs_input_grad[4])
            if part_i is not None:  # sums and fp32 parameter gradients from one launch
                s_i, gw_i, gb_i = conv_bn.sum_parts_grads(part_i, invstd_i, bn_in_w, need_i)
            elif s_i is None:
                s_i, gw_i, gb_i = syncbn.backward_reduce(da, src, None, mean_i, invstd_i, scale_i, shift_i, True,
                                                         bn_in_w, need_i, None)
            elif need_i:
                gw_i = (s_i[K:] * invstd_i).to(bn_in_w.dtype)
                gb_i = s_i[:K].to(bn_in_w.dtype, copy=True)  # (s_i is all-reduced in place below)
            if ctx.world > 1:
                with comm_stats.timed("syncbn_bwd", s_i):
                    _all_reduce_async(s_i, cfg.bn_in.process_group).wait()
            gx, _ = syncbn.backward_dgrad(da, src, None, mean_i, invstd_i, bn_in_w, s_i, count_i, scale_i, shift_i,
                                          True, False, None)
            if not need_i:
                gw_i = gb_i = None
        else:
            if part_i is not None:
                cfg.link_in.take_part(part_i)
            elif s_i is not None:
                cfg.link_in.sums = s_i
            gx = da
        gz = g if cfg.bn_ds is None else None
        return gx, None, gw3, gw_i, gb_i, gw, gb, gz, None, None, None, None, gwd, gw_d, gb_d


def _bnb_segments(g2d, W, epi):
    """Column segments for conv3's data gradient with the BatchNorm-backward prologue on the strip kernel:
    1 where the whole [N, K] weight fits one strip-kernel call, 2 / 4 for the wider 28x28 layers (each segment
    <= 256 channels), 0 where the strip kernel does not take the shape (then gx is formed in its own pass)."""
    from ..ops import conv_bn

    N, K = W.shape
    M = g2d.size(0)
    if conv_bn.preferred(N, K, M) and conv_bn.supported(g2d, W, epi=epi, b_trans=True, bnb=True):
        return 1
    if M < 100000 or N % 256 or N // 256 > 4:
        return 0
    probe = g2d.new_empty((M, 256))
    ok = (conv_bn.supported(probe, W[:256], epi="plain", b_trans=True, bnb=True) and
          conv_bn.supported(probe, W[:256], epi=epi, resid=True, b_trans=True, bnb=True))
    return N // 256 if ok else 0


def _dgrad_bn_sums(gy2d, w2d, lk):
    """``gy2d @ w2d`` (``w2d [N, K]``: the data gradient of a 1x1 convolution) with the backward sums of the
    BatchNorm ``lk = (y2d, scale, shift, mean, relu)`` that produced its input in the epilogue where an own
    kernel runs (strip GEMM or tiled MFMA GEMM), else hipBLASLt: ``(dA2d, sums or None)``."""
    from ..ops import conv_bn

    N, K = w2d.shape
    M = gy2d.size(0)
    if conv_bn.preferred(N, K, M) and conv_bn.supported(gy2d, w2d, epi="bwd" if lk else "plain", b_trans=True):
        if lk is not None:
            da, part = conv_bn.c1x1(gy2d, w2d, epi="bwd", by=lk[0], bscale=lk[1], bshift=lk[2], bmean=lk[3],
                                    brelu=lk[4], b_trans=True)
            return da, conv_bn.sum_parts(part)
        return conv_bn.c1x1(gy2d, w2d, b_trans=True)[0], None
    if _own("bwd" if lk else "plain") and conv_bn.gemm_bn_supported(gy2d, w2d.t()):
        wt = _tr(w2d)
        if lk is not None:
            da, part = conv_bn.gemm_bn(gy2d, wt, "bwd", by=lk[0], bscale=lk[1], bshift=lk[2], bmean=lk[3], brelu=lk[4])
            return da, conv_bn.sum_parts(part)
        return conv_bn.gemm_bn(gy2d, wt, "plain")[0], None
    return torch.mm(gy2d, w2d), None


def _conv_bn_res_ok(src, w3, z, pro):
    """Whether :class:`_ConvBNResFn` covers the shapes (else the per-layer path runs). ``BH_BN_RES_FOLD``:
    "pro" (default) only where bn2 is folded into conv3's prologue (the HBM-bound 56x56 / 28x28 stages),
    "all" also the wider stages, "0" never."""
    from ..ops import conv as bhconv
    from ..ops import syncbn

    if _BN_RES_FOLD == "0" or (_BN_RES_FOLD == "pro" and not pro):
        return False
    if not (src.is_cuda and z is not None and z.dtype == src.dtype and
            z.is_contiguous(memory_format=torch.channels_last) and src.is_contiguous(memory_format=torch.channels_last)):
        return False
    n, K, h, w = src.shape
    N = w3.size(0)
    if tuple(z.shape) != (n, N, h, w) or K % 64 or N % 64 or w3.dtype != src.dtype:
        return False
    # z stands in for conv3's output (same shape, dtype and layout) in the shape checks
    return syncbn.mask_ok(z, z) and bhconv.wgrad_supported(src, z, 1)


def _bn_conv(bn, y, part, conv_w, kshift_out, R, stride=1):
    exp_avg = bn.momentum if bn.momentum is not None else -1.0
    return _BNConvFn.apply(y, part, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, exp_avg,
                           bn.process_group, bn.num_batches_tracked, conv_w, kshift_out, R, stride)


# Switches of the fused model, from the typed configuration (beforeholiday_amd/config.py; the env names in
# brackets). Kept as module globals (refreshed by config.set) so the hot path reads a plain global.
#  _FOLD_BN [BH_FOLD_BN]: BatchNorm statistics / apply folded into the convolutions.
#  _FOLD_APPLY [BH_FOLD_APPLY]: BatchNorm + ReLU applied inside the consuming convolution instead of a
#    normalisation pass: "all" folds bn1 into the 3x3 conv and bn2 into conv3's 1x1 strip GEMM; "bn2" /
#    "bn1" only one of them; "none" keeps every pass. Same box: all 10443 / 10423, bn2 10430 / 10420, none
#    10380 / 10386 img/s (profiles/resnet50_fold_apply_ab.txt).
#  _STEM_STATS [BH_STEM_STATS]: the stem convolution's epilogue reduces the stem BatchNorm's statistics.
#  _OWN_GEMM_KINDS [BH_OWN_GEMM]: the 1x1 layers the strip kernel does not take run on the own tiled MFMA
#    GEMM (kernels/gemm.hip) with the BatchNorm epilogues: "fwd" (forward + statistics epilogue), "bwd"
#    (data gradient + the previous BatchNorm's backward sums), "plain" (data gradient), "resid" (data
#    gradient + the parked residual gradient).
#  _BN_RES_FOLD [BH_BN_RES_FOLD]: bottleneck tail (conv3 -> bn3 -> + z -> ReLU) as one node whose backward
#    folds bn3 into conv3 by linear algebra (_ConvBNResFn): "pro" where bn2 is folded into conv3's
#    prologue, "all" everywhere, "0" never.
#  _MASK_PRODUCER / _MASK_PRODUCER_ANY [BH_MASK_PRODUCER]: the next block's conv1 data gradient applies the
#    tail's ReLU mask in its epilogue, also where hipBLASLt's residual GEMM ran before ("any"); "fast":
#    only where the strip kernel is preferred anyway; "off": the tail's own mask pass. Same box: off 11102,
#    fast 11195, any 11286 img/s.
#  _DS_FOLD [BH_DS_FOLD]: the downsample BatchNorm folded into the tail node too (True: stride-1 blocks,
#    "all": also stride 2, False: its own passes).
_FOLD_BN = True
_FOLD_APPLY = "all"
_STEM_STATS = True
_OWN_GEMM_KINDS = {"fwd", "plain"}
_OWN_GEMM = True
_BN_RES_FOLD = "pro"
_MASK_PRODUCER = True
_MASK_PRODUCER_ANY = True
_DS_FOLD = True


def _apply_config(c):
    global _FOLD_BN, _FOLD_APPLY, _STEM_STATS, _OWN_GEMM_KINDS, _OWN_GEMM, _BN_RES_FOLD, _MASK_PRODUCER
    global _MASK_PRODUCER_ANY, _DS_FOLD
    _FOLD_BN, _FOLD_APPLY, _STEM_STATS = c.fold_bn, c.fold_apply, c.stem_stats
    _OWN_GEMM_KINDS = {k for k in c.own_gemm.split(",") if k}
    _OWN_GEMM = bool(_OWN_GEMM_KINDS)
    _BN_RES_FOLD = {"off": "0"}.get(c.bn_res_fold, c.bn_res_fold)
    _MASK_PRODUCER, _MASK_PRODUCER_ANY = c.mask_producer != "off", c.mask_producer == "any"
    _DS_FOLD = {"off": False, "stride1": True, "all": "all"}[c.ds_fold]


def _own(kind):
    return kind in _OWN_GEMM_KINDS


_config.on_change(_apply_config)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample: Optional[nn.Module] = None,
                 norm_layer=nn.BatchNorm2d, fused=False):
        super().__init__()
        self.fused = fused
        relu_kw = {"fuse_relu": True} if fused else {}
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = norm_layer(planes, **relu_kw)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = norm_layer(planes, **relu_kw)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion, **relu_kw)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def _fold_ok(self, x):
        from ..parallel import SyncBatchNorm

        bns = [self.bn1, self.bn2, self.bn3] + ([self.downsample[1]] if self.downsample is not None else [])
        return (_FOLD_BN and self.training and x.is_cuda and x.dim() == 4 and x.dtype in (torch.float16, torch.bfloat16)
                and x.is_contiguous(memory_format=torch.channels_last) and _kw(self.conv1.weight, x) is not None
                and all(isinstance(b, SyncBatchNorm) and b.track_running_stats and b.channel_last
                        and b.running_mean is not None and b.running_mean.dtype == torch.float32 for b in bns)
                and (self.downsample is None or len(self.downsample) == 2))

    def _ds_fold_ok(self, x, yd, wd):
        """The downsample BatchNorm folds into the tail node (_ConvBNResFn): the two-BatchNorm residual pass
        keeps 4 C floats in LDS, the downsample conv's fp32 weight-gradient partials and Gram cover x."""
        from ..ops import conv as bhconv

        C, Cin = yd.size(1), x.size(1)
        st = self.stride
        # stride 1 only (by default): at stride 2 the Gram of the gathered input costs about what the removed
        # passes save (BH_DS_FOLD=all also folds those)
        if st == 2 and _DS_FOLD != "all":
            return False
        return (C <= 4096 and Cin % 64 == 0 and wd.dtype == x.dtype and bhconv.wgrad_supported(x, yd, 1, st) and
                (st == 1 or (x.size(2) % 2 == 0 and x.size(3) % 2 == 0)))

    def _fold_bn2(self, y2):
        """bn2 folds into conv3 where conv3 runs on the 1x1 strip GEMM (the HBM-bound 56x56 / 28x28
        layers): its prologue variant measured 0.083 vs 0.19 ms for BN pass + GEMM + statistics pass at
        K 128 -> N 512 (profiles/conv_bn_vs_unfused.jsonl, mode "pro"); the wider layers keep the pass
        and the library GEMM."""
        from ..ops import conv_bn

        n, c, h, w = y2.shape
        k = self.conv3.weight.size(0)
        if c > 128 or n * h * w < 100000:
            return False
        a2d = y2.permute(0, 2, 3, 1).reshape(-1, c)
        w3 = self.conv3.weight if self.conv3.weight.dtype == y2.dtype else self.conv3.weight.detach().to(y2.dtype)
        return conv_bn.supported(a2d, w3.view(k, c), pro=True, epi="stats")

    def _forward_folded(self, x):
        from ..ops import conv as bhconv
        from ..parallel.optimized_sync_batchnorm import BNLink

        ds = self.downsample
        # the convolutions' weights in x's dtype (amp O1 / O4: the per-iteration 16-bit copies)
        w1, w2, w3 = (_kw(c.weight, x) for c in (self.conv1, self.conv2, self.conv3))
        wd = _kw(ds[0].weight, x) if ds is not None else None
        ds_box = None
        if ds is not None:  # conv1 and the downsample conv as one node (no residual stash needed)
            ds_box = {}
            y1, p1, yd, pd = _Conv1DsFn.apply(x, w1, wd, _kshift(self.bn1), _kshift(ds[1]),
                                              self.stride == 2, ds_box)
            box = None
        else:
            box = {} if (torch.is_grad_enabled() and x.requires_grad) else None
            y1, p1 = _Conv1x1BNFn.apply(x, w1, _kshift(self.bn1), None, box, False, getattr(x, "_bh_mask", None))
        l2 = None
        y3 = None
        y2 = None
        if _FOLD_APPLY in ("all", "bn1") and self.stride == 1 and bhconv.supported(y1, w2):
            # bn1 + ReLU inside conv2's halo prologue (and its weight gradient's LDS prologue)
            y2, p2 = _bn_conv(self.bn1, y1, p1, w2, _kshift(self.bn2), 3)
        elif _FOLD_APPLY in ("all", "bn1") and self.stride == 2 and y1.size(1) <= 512 and \
                bhconv.s2_supported(y1, w2):
            # the downsampling 3x3: bn1 + ReLU in the implicit-GEMM kernel's A-fragment prologue (and the
            # strided wgrad kernel's LDS prologue), bn2's statistics in its epilogue. The prologue variant
            # of the implicit GEMM takes at most 512 input channels (kMaxProC, kernels/conv_igemm.hip);
            # s2_supported() checks the shape without a prologue
            y2, p2 = _bn_conv(self.bn1, y1, p1, w2, _kshift(self.bn2), 3, stride=2)
        else:
            l1 = BNLink()
            a1 = self.bn1.forward_from_stats(y1, p1, link=l1)
            if self.stride == 1 and bhconv.supported(a1, w2):
                y2, p2 = _Conv3x3BNFn.apply(a1, w2, _kshift(self.bn2), l1)
            else:  # stride-2 3x3 (MIOpen): its BatchNorm computes its own statistics
                a2 = self.bn2(self.conv2(a1))
        fold2 = y2 is not None and _FOLD_APPLY in ("all", "bn2") and self._fold_bn2(y2)
        if y2 is not None and not fold2:
            l2 = BNLink()
            a2 = self.bn2.forward_from_stats(y2, p2, link=l2)
        src = y2 if fold2 else a2
        # the tail as one node (conv3 -> bn3 -> + z -> ReLU, bn3's backward folded into conv3's): z is the
        # block input or the downsample BatchNorm's output, both shaped like conv3's output
        if _conv_bn_res_ok(src, w3, yd if ds is not None else x, fold2):
            if ds is not None and _DS_FOLD and self._ds_fold_ok(x, yd, wd):
                cfg = _FoldCfg(self.bn2 if fold2 else None, self.bn3, None if fold2 else l2, ds[1], ds_box,
                               self.stride == 2)
                return _ConvBNResFn.apply(src, p2 if fold2 else None, w3, self.bn2.weight if fold2 else None,
                                          self.bn2.bias if fold2 else None, self.bn3.weight, self.bn3.bias, None,
                                          cfg, yd, pd, x, wd, ds[1].weight, ds[1].bias)
            if ds is not None:
                identity = ds[1].forward_from_stats(yd, pd)
            else:
                identity = _GradStash.apply(x, box) if box is not None else x
            if _conv_bn_res_ok(src, w3, identity, fold2):
                cfg = _FoldCfg(self.bn2 if fold2 else None, self.bn3, None if fold2 else l2)
                return _ConvBNResFn.apply(src, p2 if fold2 else None, w3, self.bn2.weight if fold2 else None,
                                          self.bn2.bias if fold2 else None, self.bn3.weight, self.bn3.bias, identity,
                                          cfg)
            if fold2:
                y3, p3 = _bn_conv(self.bn2, y2, p2, w3, _kshift(self.bn3), 1)
            else:
                y3, p3 = _Conv1x1BNFn.apply(a2, w3, _kshift(self.bn3), l2, None, False)
            return self.bn3.forward_from_stats(y3, p3, z=identity)
        if fold2:
            # bn2 + ReLU inside conv3's strip-GEMM prologue (statistics of bn3 in its epilogue)
            y3, p3 = _bn_conv(self.bn2, y2, p2, w3, _kshift(self.bn3), 1)
        if y3 is None:
            y3, p3 = _Conv1x1BNFn.apply(a2, w3, _kshift(self.bn3), l2, None, False)
        if ds is not None:
            identity = ds[1].forward_from_stats(yd, pd)
        else:
            identity = _GradStash.apply(x, box) if box is not None else x
        return self.bn3.forward_from_stats(y3, p3, z=identity)

    def forward(self, x):
        identity = x
        if self.fused and self._fold_ok(x):
            return self._forward_folded(x)
        if self.fused:
            # BN+ReLU and BN+residual-add+ReLU run as single fused passes (SyncBatchNorm fuse_relu)
            box = None
            if isinstance(self.conv1, Conv1x1) and torch.is_grad_enabled() and x.requires_grad and \
                    self.conv1.fast_path(x):
                box = {}  # the residual branch gradient is summed inside conv1's data-gradient GEMM
            out = self.bn1(self.conv1(x, box) if box is not None else self.conv1(x))
            out = self.bn2(self.conv2(out))
            xs = _GradStash.apply(x, box) if box is not None else x
            if self.downsample is not None:
                identity = self.downsample(xs)
            else:
                identity = xs
            return self.bn3(self.conv3(out), z=identity)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = out + identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block: Type[Bottleneck], layers: List[int], num_classes=1000,
                 zero_init_residual=False, norm_layer=nn.BatchNorm2d, fused=False, stem_pool_fused=False):
        super().__init__()
        self._norm_layer = norm_layer
        self.fused = fused
        # stem_pool_fused: bn1 also applies the 3x3/2 max pool (one pass, the normalised stem
        # activation is never materialised); same parameters / state_dict as the unfused stem
        self.stem_pool_fused = fused and stem_pool_fused
        self.inplanes = 64
        if _CONV3X3_MODE != "miopen":  # the fused model: MFMA stem forward and weight gradient
            # (0.15 / 0.27 ms vs MIOpen's 0.48 / 0.39, profiles/resnet50_stem_mfma_vs_miopen.jsonl)
            self.conv1 = StemConv(3, 64, kernel_size=7, stride=2, padding=3, bias=False, mode="gemm")
        else:
            self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        if self.stem_pool_fused:
            self.bn1 = norm_layer(64, fuse_relu=True, fuse_maxpool=(3, 2, 1))
        else:
            self.bn1 = norm_layer(64, fuse_relu=True) if fused else norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.modules.batchnorm._BatchNorm):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, norm_layer, fused=self.fused)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, norm_layer=norm_layer, fused=self.fused))
        return nn.Sequential(*layers)

    def _stem_stats_ok(self, x):
        from ..ops import conv as bhconv
        from ..parallel import SyncBatchNorm

        bn = self.bn1
        return (_FOLD_BN and _STEM_STATS and self.training and isinstance(self.conv1, StemConv) and self.conv1.mode == "gemm"
                and isinstance(bn, SyncBatchNorm) and bn.track_running_stats and bn.running_mean is not None
                and bn.running_mean.dtype == torch.float32 and _kw(self.conv1.weight, x) is not None
                and bhconv.stem_supported(x, _kw(self.conv1.weight, x)))

    def forward(self, x):
        if self.fused:
            x = _kx(x)  # amp O1 / O4: the whole network runs the 16-bit kernels (fp32 parameters)
        if self.stem_pool_fused and self._stem_stats_ok(x):
            # stem conv with the BatchNorm statistics in its epilogue, then BN + ReLU + max pool in one pass
            y, part = _StemStatsFn.apply(x, _kw(self.conv1.weight, x), _kshift(self.bn1))
            x = self.bn1.forward_from_stats(y, part) if self.bn1._pool_ok(y, None) else self.bn1(y)
        elif self.stem_pool_fused:
            x = self.bn1(self.conv1(x))
        else:
            x = self.bn1(self.conv1(x)) if self.fused else self.relu(self.bn1(self.conv1(x)))
            x = self.maxpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.fused and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.size(1) > 1:
            x = _GlobalAvgPoolFn.apply(x)
        else:
            x = torch.flatten(self.avgpool(x), 1)
        fc = _fc_args(self.fc, x) if self.fused else None
        if fc is not None:  # the classifier on the MFMA GEMM too (fixed kernels, rank-identical)
            return _FcFn.apply(x, *fc)
        return self.fc(x)


def resnet50(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet50_fused(process_group=None, channel_last=True, conv1x1_mode="auto", stem_pool_fused=True,
                   gemm_1x1=None, conv3x3_mode="auto", layers=(3, 4, 6, 3), **kw) -> ResNet:
    """ResNet-50 whose BatchNorms are fused SyncBatchNorms (BN+ReLU and BN+add+ReLU in one pass),
    synchronised over ``process_group`` -- the 'amp O2 + SyncBatchNorm' benchmark model.
    ``conv1x1_mode``: stride-1 1x1 convolutions as hipBLASLt GEMMs on the channels_last view
    ("gemm"), MIOpen ("miopen"), or the faster of the two per shape and direction ("auto").
    ``conv3x3_mode``: stride-1 3x3 convolutions on the direct MFMA kernel ("direct"), MIOpen, or "auto"."""
    global _CONV1X1_MODE, _CONV3X3_MODE
    if gemm_1x1 is not None:  # older keyword
        conv1x1_mode = "gemm" if gemm_1x1 else "miopen"
    from ..parallel import SyncBatchNorm

    def norm(c, fuse_relu=False, fuse_maxpool=None):
        return SyncBatchNorm(c, process_group=process_group, channel_last=channel_last, fuse_relu=fuse_relu,
                             fuse_maxpool=fuse_maxpool)

    old, _CONV1X1_MODE = _CONV1X1_MODE, conv1x1_mode
    old3, _CONV3X3_MODE = _CONV3X3_MODE, conv3x3_mode
    try:
        return ResNet(Bottleneck, list(layers), norm_layer=norm, fused=True, stem_pool_fused=stem_pool_fused, **kw)
    finally:
        _CONV1X1_MODE = old
        _CONV3X3_MODE = old3


def resnet18_like(**kw) -> ResNet:
    """Small bottleneck ResNet used by fast tests (same block structure, fewer blocks)."""
    return ResNet(Bottleneck, [1, 1, 1, 1], **kw)
