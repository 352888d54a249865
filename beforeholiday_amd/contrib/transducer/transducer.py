"""RNN-T joint and loss (reference: apex/contrib/transducer/transducer.py:5-200).

``TransducerLoss``: log-softmax + lattice forward/backward; on GPU the alpha/beta recursions and
the (optionally softmax-fused) gradient are HIP kernels (``transducer_loss_cuda``,
kernels/transducer.hip); on CPU a torch reference with identical semantics.
``TransducerJoint``: h[b,t,u] = f[b,t] + g[b,u] (+ ReLU, dropout), padded or packed output; the
broadcast-add / mask ops are single torch elementwise passes and the backward reductions
(sum over u for f, over t for g) are torch reductions.
"""
import torch

from ..._native import submodule


# ------------------------------------------------------------------------------------------ loss
def _node_rows(f_len, y_len, batch_offset, packed, T, U1, B):
    """[(b, t, u) -> row] index helper for the CPU path."""
    def row(b, t, u):
        if packed:
            start = 0 if b == 0 else int(batch_offset[b - 1])
            return start + t * (int(y_len[b]) + 1) + u
        return (b * T + t) * U1 + u
    return row


def _loss_fwd_ref(x, label, f_len, y_len, batch_offset, max_f_len, blank, packed):
    V = x.size(-1)
    B = f_len.numel()
    T = max_f_len if packed else x.size(1)
    U1 = (label.size(1) + 1) if packed else x.size(2)
    xf = x.reshape(-1, V).float()
    row = _node_rows(f_len, y_len, batch_offset, packed, T, U1, B)
    alpha = torch.full((B, T, U1), float("-inf"))
    beta = torch.full((B, T, U1), float("-inf"))
    loss = torch.zeros(B)
    for b in range(B):
        Tb, Ub = int(f_len[b]), int(y_len[b])
        for t in range(Tb):
            for u in range(Ub + 1):
                if t == 0 and u == 0:
                    alpha[b, t, u] = 0.0
                    continue
                a = alpha[b, t - 1, u] + xf[row(b, t - 1, u), blank] if t > 0 else torch.tensor(float("-inf"))
                c = (alpha[b, t, u - 1] + xf[row(b, t, u - 1), label[b, u - 1]]) if u > 0 else torch.tensor(
                    float("-inf"))
                alpha[b, t, u] = torch.logaddexp(a, c)
        for t in range(Tb - 1, -1, -1):
            for u in range(Ub, -1, -1):
                xb = xf[row(b, t, u), blank]
                if t == Tb - 1 and u == Ub:
                    beta[b, t, u] = xb
                    continue
                a = beta[b, t + 1, u] + xb if t < Tb - 1 else torch.tensor(float("-inf"))
                c = beta[b, t, u + 1] + xf[row(b, t, u), label[b, u]] if u < Ub else torch.tensor(float("-inf"))
                beta[b, t, u] = torch.logaddexp(a, c)
        loss[b] = -beta[b, 0, 0]
    return alpha, beta, loss


def _loss_bwd_ref(x, loss_grad, alpha, beta, f_len, y_len, label, batch_offset, max_f_len, blank, fuse, packed):
    V = x.size(-1)
    B = f_len.numel()
    T, U1 = alpha.size(1), alpha.size(2)
    xf = x.reshape(-1, V).float()
    dx = torch.zeros_like(xf)
    row = _node_rows(f_len, y_len, batch_offset, packed, T, U1, B)
    for b in range(B):
        Tb, Ub = int(f_len[b]), int(y_len[b])
        ll = beta[b, 0, 0]
        for t in range(Tb):
            for u in range(Ub + 1):
                r = row(b, t, u)
                a = alpha[b, t, u]
                d = torch.zeros(V)
                if t == Tb - 1 and u == Ub:
                    d[blank] += torch.exp(a + xf[r, blank] - ll)
                elif t < Tb - 1:
                    d[blank] += torch.exp(a + beta[b, t + 1, u] + xf[r, blank] - ll)
                if u < Ub:
                    d[label[b, u]] += torch.exp(a + beta[b, t, u + 1] + xf[r, label[b, u]] - ll)
                if fuse:
                    d -= torch.exp(xf[r]) * torch.exp(a + beta[b, t, u] - ll)
                dx[r] = -float(loss_grad[b]) * d
    return dx.view(x.shape).to(x.dtype)


class TransducerLossFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, label, f_len, y_len, batch_offset, max_f_len, blank_idx, fuse_softmax_backward, debug_list,
                opt, packed_input):
        if not fuse_softmax_backward:
            with torch.enable_grad():
                x = torch.nn.functional.log_softmax(x, dim=-1)
        else:
            x = torch.nn.functional.log_softmax(x, dim=-1)
        if x.is_cuda:
            alpha, beta, loss = submodule("transducer_loss_cuda").forward(
                x.detach(), label, f_len, y_len, batch_offset, max_f_len, blank_idx, opt, packed_input)
        else:
            alpha, beta, loss = _loss_fwd_ref(x.detach(), label, f_len, y_len, batch_offset, max_f_len, blank_idx,
                                              packed_input)
        if debug_list == []:
            debug_list += [alpha, beta]
        ctx.save_for_backward(x, alpha, beta, f_len, y_len, label, batch_offset)
        ctx.blank_idx = blank_idx
        ctx.fuse_softmax_backward = fuse_softmax_backward
        ctx.opt = opt
        ctx.packed_input = packed_input
        ctx.max_f_len = max_f_len
        return loss.to(x.dtype)

    @staticmethod
    def backward(ctx, loss_grad):
        x, alpha, beta, f_len, y_len, label, batch_offset = ctx.saved_tensors
        if x.is_cuda:
            x_grad = submodule("transducer_loss_cuda").backward(
                x.detach(), loss_grad, alpha, beta, f_len, y_len, label, batch_offset, ctx.max_f_len, ctx.blank_idx,
                ctx.opt, ctx.fuse_softmax_backward, ctx.packed_input)
        else:
            x_grad = _loss_bwd_ref(x.detach(), loss_grad, alpha, beta, f_len, y_len, label, batch_offset,
                                   ctx.max_f_len, ctx.blank_idx, ctx.fuse_softmax_backward, ctx.packed_input)
        if not ctx.fuse_softmax_backward:
            x_grad = _lsm_bwd(x, x_grad)
        return x_grad, None, None, None, None, None, None, None, None, None, None


def _lsm_bwd(logp, g):
    """log-softmax backward: g - softmax * sum(g)."""
    return g - torch.exp(logp.detach()) * g.sum(-1, keepdim=True)


class TransducerLoss(torch.nn.Module):
    def __init__(self, fuse_softmax_backward=True, opt=1, packed_input=False):
        super().__init__()
        self.fuse_softmax_backward = fuse_softmax_backward
        self.opt = opt
        self.packed_input = packed_input
        self.dummy_batch_offset = torch.empty(0)

    def forward(self, x, label, f_len, y_len, blank_idx, batch_offset=None, max_f_len=None, debug_list=None):
        if self.packed_input:
            if batch_offset is None or max_f_len is None:
                raise Exception("Please specify batch_offset and max_f_len when packing is enabled")
            bo, mf = batch_offset, max_f_len
        else:
            bo, mf = self.dummy_batch_offset.to(x.device), x.size(1)
        return TransducerLossFunc.apply(x, label, f_len, y_len, bo, mf, blank_idx, self.fuse_softmax_backward,
                                        debug_list, self.opt, self.packed_input)


# ------------------------------------------------------------------------------------------ joint
def _joint_native_ok(f, g):
    return f.is_cuda and g.is_cuda and f.dtype == g.dtype and f.dtype in (torch.float16, torch.bfloat16, torch.float32) \
        and f.size(-1) % 8 == 0


class _TransducerJointNative(torch.autograd.Function):
    """HIP joint (kernels/transducer.hip): f + g broadcast-add, packing, ReLU and counter-hash dropout
    in one pass; the backward regenerates the dropout bits and reads the ReLU mask off the output, so
    neither pass materialises [B, T, U, H] temporaries or a mask tensor."""

    @staticmethod
    def forward(ctx, f, g, f_len, g_len, pack_output, relu, dropout, batch_offset, packed_batch, dropout_prob,
                mask_probe):
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())  # host generator: no device sync
        out, mask = submodule("transducer_joint_cuda").forward(
            f, g, f_len, g_len, batch_offset, int(packed_batch), bool(pack_output), bool(relu), bool(dropout),
            float(dropout_prob), seed, mask_probe is not None)
        if mask_probe is not None:
            mask_probe.append(mask)
        ctx.save_for_backward(out if relu else None, f_len, g_len, batch_offset if pack_output else None)
        ctx.meta = (f.size(1), g.size(1), bool(pack_output), bool(relu), bool(dropout), float(dropout_prob), seed)
        return out

    @staticmethod
    def backward(ctx, grad):
        out, f_len, g_len, bo = ctx.saved_tensors
        T, U, pack, relu, dropout, prob, seed = ctx.meta
        df, dg = submodule("transducer_joint_cuda").backward(
            grad, out if out is not None else torch.empty(0, device=grad.device), f_len, g_len, bo if bo is not None else torch.empty(0, device=grad.device), T, U, pack, relu,
            dropout, prob, seed)
        return df, dg, None, None, None, None, None, None, None, None, None


class TransducerJointFunc(torch.autograd.Function):
    """PyTorch reference joint (CPU tensors, or shapes the HIP kernel does not take)."""

    @staticmethod
    def forward(ctx, f, g, f_len, g_len, pack_output, relu, dropout, batch_offset, packed_batch, opt, fwd_tile_size,
                dropout_prob, mask_probe):
        B, T, H = f.shape
        U = g.size(1)
        h = f.unsqueeze(2) + g.unsqueeze(1)  # one broadcast-add pass
        mask = None
        scale = 1.0
        if relu or dropout:
            mask = h > 0 if relu else torch.ones_like(h, dtype=torch.bool)
            if dropout:
                mask &= torch.rand_like(h, dtype=torch.float32) >= dropout_prob
                scale = 1.0 / (1.0 - dropout_prob) if dropout_prob != 1 else 1.0
            h = h * mask.to(h.dtype) * scale
        valid = (torch.arange(T, device=f.device).view(1, T, 1) < f_len.view(B, 1, 1)) & \
                (torch.arange(U, device=f.device).view(1, 1, U) < g_len.view(B, 1, 1))
        if pack_output:
            out = h[valid]
            if mask is not None:
                mask = mask[valid]
        else:
            out = h.masked_fill(~valid.unsqueeze(-1), 0.0)
        if mask is not None and mask_probe is not None:
            mask_probe.append(mask)
        ctx.save_for_backward(mask if mask is not None else torch.empty(0), valid)
        ctx.meta = (pack_output, mask is not None, scale, B, T, U, H)
        return out

    @staticmethod
    def backward(ctx, grad):
        mask, valid = ctx.saved_tensors
        pack, masked, scale, B, T, U, H = ctx.meta
        if pack:
            gfull = grad.new_zeros(B, T, U, H)
            gfull[valid] = grad * (mask.to(grad.dtype) * scale if masked else 1.0)
        else:
            gfull = grad.masked_fill(~valid.unsqueeze(-1), 0.0)
            if masked:
                gfull = gfull * mask.to(grad.dtype) * scale
        return (gfull.sum(2), gfull.sum(1), None, None, None, None, None, None, None, None, None, None, None)


class TransducerJoint(torch.nn.Module):
    def __init__(self, pack_output=False, relu=False, dropout=False, opt=1, fwd_tile_size=4, dropout_prob=0,
                 probe_mask=False):
        super().__init__()
        self.pack_output = pack_output
        self.relu = relu
        self.dropout = dropout
        self.dropout_prob = dropout_prob
        self.opt = opt
        self.fwd_tile_size = fwd_tile_size
        self.dummy_batch_offset = torch.empty(0)
        masked = relu or dropout
        self.mask_probe = [] if masked and probe_mask else None
        if masked and opt != 1:
            raise NotImplementedError("ReLU and dropout fusion is only supported with opt=1")

    def forward(self, f, g, f_len, g_len, batch_offset=None, packed_batch=0):
        bo = batch_offset if self.pack_output else self.dummy_batch_offset
        if self.pack_output and (batch_offset is None or packed_batch == 0):
            raise Exception("Please specify batch_offset and packed_batch when packing is enabled")
        dropout = self.dropout and self.training
        if _joint_native_ok(f, g):
            return _TransducerJointNative.apply(f, g, f_len, g_len, self.pack_output, self.relu, dropout,
                                                bo.to(f.device), packed_batch, self.dropout_prob, self.mask_probe)
        return TransducerJointFunc.apply(f, g, f_len, g_len, self.pack_output, self.relu, dropout, bo, packed_batch,
                                         self.opt, self.fwd_tile_size, self.dropout_prob, self.mask_probe)
