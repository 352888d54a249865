"""``fused_dense_cuda`` / ``mlp_cuda`` / ``fused_weight_gradient_mlp_cuda`` ops.

GPU tensors run ``beforeholiday_amd._C`` -- the SAME native entry points that ``import fused_dense_cuda``
/ ``mlp_cuda`` reach after ``install_apex_aliases()`` (bindings/dense.cpp): forward GEMMs with the bias /
GELU epilogue on the MFMA kernel (kernels/gemm.hip) where its static rule picks it, data gradients with
the dActivation + bias-gradient epilogue on the MFMA kernel (hipBLASLt for a plain dY . W), weight
gradients on the transposed-operand MFMA GEMM (kernels/gemm_tn.hip) or the 1x1 weight-gradient kernel
(static shape rules, ``weight_grad``), activation / bias-gradient passes in kernels/dense.hip. CPU
tensors run the PyTorch reference below with the same semantics (exact-erf GELU; ReLU / sigmoid
derivatives taken from the activation output).
"""
from typing import List, Optional

import torch
import torch.nn.functional as F

from .. import config as _config
from .._native import submodule

ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_GELU, ACT_GELU_TANH = 0, 1, 2, 3, 4


def _fd():
    return submodule("fused_dense_cuda")


def _act_ref(x, act):
    if act == ACT_RELU:
        return torch.relu(x)
    if act == ACT_SIGMOID:
        return torch.sigmoid(x)
    if act == ACT_GELU:
        return F.gelu(x)
    if act == ACT_GELU_TANH:
        return F.gelu(x, approximate="tanh")
    return x


def _act_grad_ref(dy, aux, act):
    a = aux.float()
    if act == ACT_RELU:
        d = (a > 0).float()
    elif act == ACT_SIGMOID:
        d = a * (1 - a)
    elif act == ACT_GELU:
        d = 0.5 * (1 + torch.erf(a * 0.7071067811865476)) + a * 0.3989422804014327 * torch.exp(-0.5 * a * a)
    elif act == ACT_GELU_TANH:
        k = 0.7978845608028654
        t = torch.tanh(k * (a + 0.044715 * a ** 3))
        d = 0.5 * (1 + t) + 0.5 * a * (1 - t * t) * k * (1 + 3 * 0.044715 * a * a)
    else:
        return dy
    return (dy.float() * d).to(dy.dtype)


def bias_act_forward(x: torch.Tensor, bias: Optional[torch.Tensor], act: int) -> torch.Tensor:
    """act(x + bias) in one pass."""
    if x.is_cuda:
        return _fd().act_forward(x, bias, act)
    return _act_ref(x + bias if bias is not None else x, act)


def act_backward(dy: torch.Tensor, aux: torch.Tensor, act: int, want_bgrad: bool):
    """(dy * act'(aux), sum over rows of it) in one pass."""
    if dy.is_cuda:
        dx, db = _fd().act_backward(dy, aux, act, want_bgrad)
        return dx, (db if want_bgrad else None)
    dx = _act_grad_ref(dy, aux, act)
    return dx, (dx.reshape(-1, dx.size(-1)).float().sum(0).to(dx.dtype) if want_bgrad else None)


def bias_grad(dy: torch.Tensor) -> torch.Tensor:
    """Bias gradient: sum of ``dy`` over every leading dim (fp32 accumulation, ``dy``'s dtype).
    GPU: one split-row partial-sum pass + a column-sum finalize (kernels/dense.hip)."""
    if dy.is_cuda and dy.dtype in (torch.float16, torch.bfloat16, torch.float32) and dy.size(-1) > 0:
        return _fd().bias_grad(dy)
    return dy.reshape(-1, dy.size(-1)).float().sum(0).to(dy.dtype)


def _gemm_ok(*ts):
    return all(t.is_cuda and t.dtype in (torch.float16, torch.bfloat16) for t in ts) and len({t.dtype for t in ts}) == 1


def linear_bias_forward(input, weight, bias):
    """y = x . W^T + b. 16-bit GPU tensors: the MFMA GEMM with the bias in its epilogue where the static
    dispatch rule of kernels/gemm.hip picks it (K <= 1024, ``gemm.linear_act``), hipBLASLt's addmm
    otherwise -- the same rule for every rank."""
    if input.is_cuda:
        if _gemm_ok(input, weight) and (bias is None or bias.dtype == input.dtype):
            x = input.reshape(-1, input.size(-1)).contiguous()
            y = submodule("gemm").linear_act(x, weight.contiguous(), bias, ACT_NONE, False)[0]
            return y.view(*input.shape[:-1], weight.size(0))
        return _fd().linear_bias_forward(input, weight, bias)
    return F.linear(input, weight, bias)


def linear_bias_backward(input, weight, d_output):
    """(d_input, d_weight, d_bias). GPU: one native call (bindings/dense.cpp): the weight gradient by
    the static MFMA rule (``weight_grad``), the input gradient through ``data_grad`` (hipBLASLt for a
    plain data gradient, where the library measured 1.0-1.18x faster:
    profiles/dgrad_transformer_nt_vs_hipblaslt.jsonl), the bias gradient as one column-sum pass."""
    if input.is_cuda:
        return tuple(_fd().linear_bias_backward(input, weight, d_output))
    dy = d_output.reshape(-1, d_output.size(-1))
    x = input.reshape(-1, input.size(-1))
    return (dy.mm(weight).view(input.shape), dy.t().mm(x), dy.sum(0))


def linear_gelu_linear_forward(input, weight1, bias1, weight2, bias2):
    """Returns (gelu_in, gelu_out, output): both GEMMs through ``gemm.linear_act`` (bias + GELU + the
    pre-activation in the first one's epilogue, bias in the second's) on 16-bit GPU tensors."""
    if input.is_cuda:
        if _gemm_ok(input, weight1, weight2) and bias1 is not None and bias2 is not None:
            gm = submodule("gemm")
            x = input.reshape(-1, input.size(-1)).contiguous()
            gelu_out, gelu_in = gm.linear_act(x, weight1.contiguous(), bias1.contiguous(), ACT_GELU, True)
            out = gm.linear_act(gelu_out, weight2.contiguous(), bias2.contiguous(), ACT_NONE, False)[0]
            return gelu_in, gelu_out, out
        return _fd().linear_gelu_linear_forward(input, weight1, bias1, weight2, bias2)
    x = input.reshape(-1, input.size(-1))
    gelu_in = F.linear(x, weight1, bias1)
    h = F.gelu(gelu_in)
    return gelu_in, h, F.linear(h, weight2, bias2)


def linear_gelu_linear_backward(input, gelu_in, output1, weight1, weight2, d_output2):
    """Returns (d_input, d_weight1, d_bias1, d_weight2, d_bias2) -- with the dGELU applied. GPU: one
    native call: d(gelu_in) and d_bias1 from one MFMA GEMM with the dGELU + bias-gradient epilogue, the
    weight gradients by the static MFMA rule (bindings/dense.cpp)."""
    if input.is_cuda:
        return tuple(_fd().linear_gelu_linear_backward(input, gelu_in, output1, weight1, weight2, d_output2))
    x = input.reshape(-1, input.size(-1))
    dy = d_output2.reshape(-1, d_output2.size(-1))
    d_w2 = dy.t().mm(output1)
    d_b2 = dy.sum(0)
    d_h = _act_grad_ref(dy.mm(weight2), gelu_in, ACT_GELU)
    return d_h.mm(weight1).view(input.shape), d_h.t().mm(x), d_h.sum(0), d_w2, d_b2


def mlp_forward(use_bias: int, activation: int, inputs: List[torch.Tensor]) -> List[torch.Tensor]:
    """Layer outputs (last = result). activation: 0 none, 1 relu, 2 sigmoid, after every layer."""
    if inputs[0].is_cuda:
        return submodule("mlp_cuda").forward(use_bias, activation, list(inputs))
    n = (len(inputs) - 1) // 2 if use_bias else len(inputs) - 1
    act = {0: ACT_NONE, 1: ACT_RELU, 2: ACT_SIGMOID}[activation]
    h, outs = inputs[0], []
    for i in range(n):
        h = _act_ref(F.linear(h, inputs[1 + i], inputs[1 + n + i] if use_bias else None), act)
        outs.append(h)
    return outs


def mlp_backward(use_bias: int, activation: int, grad_o, outputs, inputs) -> List[torch.Tensor]:
    """Gradients for ``inputs``. On the GPU one native call (bindings/dense.cpp mlp_backward): the
    dActivation + bias gradient inside the data-gradient GEMM's epilogue, the weight gradients by the
    static MFMA rule (``weight_grad``)."""
    if inputs[0].is_cuda:
        return submodule("mlp_cuda").backward(use_bias, activation, grad_o, list(outputs), list(inputs))
    n = (len(inputs) - 1) // 2 if use_bias else len(inputs) - 1
    act = {0: ACT_NONE, 1: ACT_RELU, 2: ACT_SIGMOID}[activation]
    grads = [None] * len(inputs)
    g = grad_o
    for i in range(n - 1, -1, -1):
        dpre = _act_grad_ref(g, outputs[i], act)
        x = inputs[0] if i == 0 else outputs[i - 1]
        grads[1 + i] = dpre.t().mm(x)
        if use_bias:
            grads[1 + n + i] = dpre.sum(0)
        g = dpre.mm(inputs[1 + i])
    grads[0] = g
    return grads


def weight_grad(d_output: torch.Tensor, input: torch.Tensor) -> torch.Tensor:
    """``d_output^T @ input`` for 2-D ``[tokens, out]`` / ``[tokens, in]`` tensors: the dense layers'
    weight gradient ``[out, in]`` in ``d_output``'s dtype. GPU: bindings/dense.cpp ``weight_grad`` (the
    transposed-operand MFMA GEMM from 1.5M-element weights, the 1x1 weight-gradient kernel up to ~2.4M
    elements, both from 4096 tokens, else the library GEMM; static shape rules, the same on every rank
    and for the reference-named extensions)."""
    if d_output.is_cuda:
        return _fd().weight_grad(d_output, input)
    return d_output.t().matmul(input)


def wgrad_gemm_accum_fp32(input, d_output, main_grad):
    """main_grad (fp32) += d_output^T @ input, accumulated in fp32 in place."""
    if input.is_cuda:
        return submodule("fused_weight_gradient_mlp_cuda").wgrad_gemm_accum_fp32(input, d_output, main_grad)
    main_grad.add_(d_output.reshape(-1, d_output.size(-1)).float().t().mm(input.reshape(-1, input.size(-1)).float()))


def wgrad_gemm_accum_fp16(input, d_output, main_grad):
    """main_grad (same 16-bit dtype as input) += d_output^T @ input."""
    if input.is_cuda:
        return submodule("fused_weight_gradient_mlp_cuda").wgrad_gemm_accum_fp16(input, d_output, main_grad)
    main_grad.add_(d_output.reshape(-1, d_output.size(-1)).t().mm(input.reshape(-1, input.size(-1))))


class _BiasDropoutAddFn(torch.autograd.Function):
    """out = residual + dropout(x + bias) as ONE HIP pass that also stores 1 keep bit per element;
    backward is one pass that applies the bits and reduces the bias gradient from the same data
    (replaces Megatron's three elementwise kernels + a separate bias-grad reduction;
    reference: apex/transformer/testing/standalone_transformer_lm.py:188-207 bias_dropout_add)."""

    @staticmethod
    def forward(ctx, x, bias, residual, p, model_parallel=False, resid_link=None):
        # host-side seed stream (no device sync): "replicated" is identical on every TP rank,
        # "model-parallel" differs per TP rank (sequence-parallel shards); see random.dropout_seed
        from ..transformer.tensor_parallel.random import dropout_seed
        from ..utils import graph_rng

        sd = None
        if graph_rng.active():  # replayable: a per-call salt + the device step seed (utils/graph_rng.py)
            stream = 0
            if model_parallel:
                from ..transformer import parallel_state

                stream = 1 + parallel_state.get_tensor_model_parallel_rank()
            seed, sd = graph_rng.next_salt(stream) & 0xFFFFFFFF, graph_rng.step_seed()
        else:
            seed = dropout_seed(model_parallel)
        out, keep = _fd().bias_dropout_add(x, bias, residual, p, seed, sd)
        ctx.save_for_backward(keep)
        ctx.p = p
        ctx.has_bias = bias is not None
        # normalization.ResidualGradLink: the LayerNorm that also reads `residual` adds its gradient in-kernel
        ctx.resid_link = resid_link if residual.requires_grad else None
        if ctx.resid_link is not None:
            ctx.resid_link.armed, ctx.resid_link.g = True, None
        return out.view_as(x)

    @staticmethod
    def backward(ctx, dout):
        (keep,) = ctx.saved_tensors
        want_b = ctx.has_bias and ctx.needs_input_grad[1]
        dx, db = _fd().dropout_backward(dout, keep, ctx.p, want_b)
        dres = dout
        if ctx.resid_link is not None:
            ctx.resid_link.g, dres = dout, None
        return dx.view_as(dout), (db if want_b else None), dres, None, None, None


def _bda_native_ok(x, bias, residual) -> bool:
    return (x.is_cuda and residual.is_cuda and x.dtype == residual.dtype and x.shape == residual.shape and
            x.dtype in (torch.float16, torch.bfloat16, torch.float32) and x.size(-1) % 8 == 0 and
            x.is_contiguous() and residual.is_contiguous() and x.data_ptr() % 16 == 0 and
            residual.data_ptr() % 16 == 0 and
            (bias is None or (bias.dtype == x.dtype and bias.numel() == x.size(-1))))


def bias_dropout_add(x: torch.Tensor, bias: Optional[torch.Tensor], residual: torch.Tensor, prob: float,
                     training: bool, model_parallel: bool = False, resid_link=None) -> torch.Tensor:
    """``residual + dropout(x + bias, prob, training)``; fused HIP kernels on GPU, PyTorch otherwise.

    ``model_parallel=True`` (sequence parallelism: every TP rank holds a different shard) draws the
    mask from the per-TP-rank stream -- the fused kernel's model-parallel seed stream, or the
    tracker's "model-parallel-rng" state for the PyTorch fallback; otherwise TP replicas draw
    identical masks from the replicated stream.

    ``resid_link`` (normalization.ResidualGradLink, native path only): ``residual``'s gradient is parked
    there for the LayerNorm that also reads ``residual`` (its backward adds it in-kernel) instead of being
    returned to autograd."""
    p = float(prob) if training else 0.0
    if _bda_native_ok(x, bias, residual):
        return _BiasDropoutAddFn.apply(x, bias, residual, p, bool(model_parallel), resid_link)
    if model_parallel and training and prob > 0:
        from ..transformer.tensor_parallel.random import get_cuda_rng_tracker

        with get_cuda_rng_tracker().fork():
            out = F.dropout(x + bias if bias is not None else x, p=prob, training=training)
    else:
        out = F.dropout(x + bias if bias is not None else x, p=prob, training=training)
    return residual + out




class _EmbeddingFn(torch.autograd.Function):
    """F.embedding with the weight gradient from kernels/dense.hip (embedding_backward): stable sort of
    the ids, ordered per-id sums in fp32, no host synchronisation (torch's CUDA embedding backward
    reads its segment count back every call, which stalls the launch queue once per step)."""

    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.meta = (weight.size(0), -1 if padding_idx is None else int(padding_idx))
        return F.embedding(ids, weight, padding_idx)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        v, pad = ctx.meta
        return None, _fd().embedding_backward(dy, ids, v, pad), None


def embedding(ids: torch.Tensor, weight: torch.Tensor, padding_idx: Optional[int] = None) -> torch.Tensor:
    """``F.embedding(ids, weight, padding_idx)``; on the GPU (fp32 / fp16 / bf16 weights that need a
    gradient) the backward runs the deterministic sync-free kernel above."""
    if (weight.is_cuda and weight.requires_grad and torch.is_grad_enabled()
            and weight.dtype in (torch.float32, torch.float16, torch.bfloat16) and _config.get().embed_native):
        if padding_idx is not None and padding_idx < 0:
            padding_idx += weight.size(0)
        return _EmbeddingFn.apply(ids, weight, padding_idx)
    return F.embedding(ids, weight, padding_idx)
