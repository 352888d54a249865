// `fused_dense_cuda`, `mlp_cuda`, `fused_weight_gradient_mlp_cuda` front-ends
// (reference APIs: csrc/fused_dense_base.cpp:15-20, csrc/mlp.cpp:46-164,
// csrc/megatron/fused_weight_gradient_dense.cpp).
//
// GEMMs go to hipBLASLt through ATen (at::addmm folds the bias into the GEMM epilogue; the fp32
// weight-gradient accumulation uses addmm's out_dtype form so bf16/fp16 products accumulate in
// place into the fp32 main_grad, C == D). Activation, dActivation and bias-gradient reductions are
// the HIP kernels in kernels/dense.hip.
#include "common.h"

#include "bh/dense_api.h"

namespace bhb {
namespace {

bool al16(const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

at::Tensor as2d(const at::Tensor& t) { return t.dim() == 2 ? t : t.reshape({-1, t.size(-1)}); }

// y = act(x (+ bias)) in place on x
void act_inplace(at::Tensor& x, const at::Tensor& bias, int act) {
  if (act == bh::kActNone && !bias.defined()) return;
  const int64_t N = x.size(-1), M = x.numel() / std::max<int64_t>(N, 1);
  const bool vec = (N % 8 == 0) && al16(x) && (!bias.defined() || al16(bias));
  bh::dense_act_forward(dtype_code(x.scalar_type()), x.data_ptr(), bias.defined() ? bias.data_ptr() : nullptr,
                        x.data_ptr(), M, (int)N, act, vec, stream_for(x));
}

// dx = dy * act'(aux) (into dx_out, may be dy itself), returns bias grad if want_bgrad
at::Tensor act_backward(const at::Tensor& dy, const at::Tensor& aux, at::Tensor dx_out, int act, bool want_bgrad) {
  const int64_t N = dy.size(-1), M = dy.numel() / std::max<int64_t>(N, 1);
  at::Tensor bgrad;
  if (want_bgrad) bgrad = at::empty({N}, dy.options());
  if (act == bh::kActNone && !want_bgrad) return bgrad;
  const int splits = bh::dense_bgrad_splits(M, (int)N);
  auto part = at::empty({(int64_t)splits * N}, dy.options().dtype(at::kFloat));
  const bool vec = (N % 8 == 0) && al16(dy) && (!aux.defined() || al16(aux)) && (!dx_out.defined() || al16(dx_out));
  bh::dense_act_backward(dtype_code(dy.scalar_type()), dy.data_ptr(), aux.defined() ? aux.data_ptr() : nullptr,
                         (act != bh::kActNone && dx_out.defined()) ? dx_out.data_ptr() : nullptr,
                         want_bgrad ? bgrad.data_ptr() : nullptr, part.data_ptr<float>(), splits, M, (int)N, act, vec,
                         stream_for(dy));
  return bgrad;
}

at::Tensor bias_grad(const at::Tensor& dy) { return act_backward(dy, at::Tensor(), at::Tensor(), bh::kActNone, true); }

// ------------------------------------------------------------------------------------------------
// fused_dense_cuda
// ------------------------------------------------------------------------------------------------
at::Tensor linear_bias_forward(at::Tensor input, at::Tensor weight, at::Tensor bias) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto y = bias.defined() ? at::addmm(bias, x, weight.t()) : at::mm(x, weight.t());
  auto shape = input.sizes().vec();
  shape.back() = weight.size(0);
  return y.view(shape);
}

std::vector<at::Tensor> linear_bias_backward(at::Tensor input, at::Tensor weight, at::Tensor d_output) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output.contiguous());
  auto d_input = at::mm(dy, weight).view(input.sizes());
  auto d_weight = at::mm(dy.t(), x);
  return {d_input, d_weight, bias_grad(dy)};
}

std::vector<at::Tensor> linear_gelu_linear_forward(at::Tensor input, at::Tensor weight1, at::Tensor bias1,
                                                   at::Tensor weight2, at::Tensor bias2) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto gelu_in = at::addmm(bias1, x, weight1.t());
  auto out1 = at::empty_like(gelu_in);
  const int64_t N = gelu_in.size(1), M = gelu_in.size(0);
  bh::dense_act_forward(dtype_code(gelu_in.scalar_type()), gelu_in.data_ptr(), nullptr, out1.data_ptr(), M, (int)N,
                        bh::kActGelu, (N % 8 == 0) && al16(gelu_in) && al16(out1), stream_for(x));
  auto out2 = at::addmm(bias2, out1, weight2.t());
  return {gelu_in, out1, out2};
}

// returns {d_input, d_weight1, d_bias1, d_weight2, d_bias2}
std::vector<at::Tensor> linear_gelu_linear_backward(at::Tensor input, at::Tensor gelu_in, at::Tensor output1,
                                                    at::Tensor weight1, at::Tensor weight2, at::Tensor d_output2) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output2.contiguous());
  auto h = as2d(output1.contiguous());
  auto d_weight2 = at::mm(dy.t(), h);
  auto d_bias2 = bias_grad(dy);
  auto d_h = at::mm(dy, weight2);
  auto d_bias1 = act_backward(d_h, as2d(gelu_in.contiguous()), d_h, bh::kActGelu, true);  // d_h := dGELU in place
  auto d_weight1 = at::mm(d_h.t(), x);
  auto d_input = at::mm(d_h, weight1).view(input.sizes());
  return {d_input, d_weight1, d_bias1, d_weight2, d_bias2};
}

// ------------------------------------------------------------------------------------------------
// mlp_cuda: inputs = (x, W_0..W_{n-1}[, b_0..b_{n-1}]); activation 0 none, 1 relu, 2 sigmoid after
// every layer. forward returns the n layer outputs (last = result); backward returns grads for inputs.
// ------------------------------------------------------------------------------------------------
int mlp_act(int activation) {
  switch (activation) {
    case 0: return bh::kActNone;
    case 1: return bh::kActRelu;
    case 2: return bh::kActSigmoid;
    default: TORCH_CHECK(false, "mlp: activation must be 0 (none), 1 (relu) or 2 (sigmoid)");
  }
  return 0;
}

std::vector<at::Tensor> mlp_forward(int use_bias, int activation, std::vector<at::Tensor> inputs) {
  TORCH_CHECK(!inputs.empty(), "mlp: no inputs");
  check_cuda(inputs[0], "input");
  const int64_t n = use_bias ? (int64_t)(inputs.size() - 1) / 2 : (int64_t)inputs.size() - 1;
  const int act = mlp_act(activation);
  std::vector<at::Tensor> outs;
  at::Tensor h = inputs[0].contiguous();
  for (int64_t i = 0; i < n; ++i) {
    const at::Tensor& w = inputs[1 + i];
    at::Tensor y;
    if (use_bias) y = at::addmm(inputs[1 + n + i], h, w.t());
    else y = at::mm(h, w.t());
    act_inplace(y, at::Tensor(), act);
    outs.push_back(y);
    h = y;
  }
  return outs;
}

std::vector<at::Tensor> mlp_backward(int use_bias, int activation, at::Tensor grad_o, std::vector<at::Tensor> outputs,
                                     std::vector<at::Tensor> inputs) {
  const int64_t n = use_bias ? (int64_t)(inputs.size() - 1) / 2 : (int64_t)inputs.size() - 1;
  const int act = mlp_act(activation);
  std::vector<at::Tensor> grads(inputs.size());
  at::Tensor g = grad_o.contiguous();
  for (int64_t i = n - 1; i >= 0; --i) {
    // g := dL/d(pre-activation of layer i), bias grad fused into the same pass
    at::Tensor dpre = (act == bh::kActNone) ? g : at::empty_like(g);
    at::Tensor db = act_backward(g, outputs[i], dpre, act, use_bias != 0);
    if (act == bh::kActNone) dpre = g;
    const at::Tensor& x = (i == 0) ? inputs[0] : outputs[i - 1];
    grads[1 + i] = at::mm(dpre.t(), x.contiguous());
    if (use_bias) grads[1 + n + i] = db;
    if (i > 0 || inputs[0].requires_grad()) g = at::mm(dpre, inputs[1 + i]);
  }
  grads[0] = inputs[0].requires_grad() ? g : at::zeros_like(inputs[0]);
  return grads;
}

// ------------------------------------------------------------------------------------------------
// fused_weight_gradient_mlp_cuda: main_grad[N,K] += d_output[M,N]^T @ input[M,K]
// ------------------------------------------------------------------------------------------------
void wgrad_gemm_accum_fp32(at::Tensor input, at::Tensor d_output, at::Tensor main_grad) {
  check_cuda(input, "input");
  TORCH_CHECK(main_grad.scalar_type() == at::kFloat, "wgrad_gemm_accum_fp32: main_grad must be fp32");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output.contiguous());
  if (x.scalar_type() == at::kFloat) {
    main_grad.addmm_(dy.t(), x);
  } else {
    at::addmm_out(main_grad, main_grad, dy.t(), x, at::kFloat, 1, 1);
  }
}

void wgrad_gemm_accum_fp16(at::Tensor input, at::Tensor d_output, at::Tensor main_grad) {
  check_cuda(input, "input");
  TORCH_CHECK(main_grad.scalar_type() == input.scalar_type(), "wgrad_gemm_accum_fp16: dtype mismatch");
  main_grad.addmm_(as2d(d_output.contiguous()).t(), as2d(input.contiguous()));
}

// activation helpers exposed for python modules (bias_gelu etc.)
at::Tensor act_forward_py(at::Tensor x, c10::optional<at::Tensor> bias, int act) {
  check_cuda(x, "x");
  auto y = x.contiguous().clone();
  act_inplace(y, bias.has_value() ? bias->contiguous() : at::Tensor(), act);
  return y;
}

std::vector<at::Tensor> act_backward_py(at::Tensor dy, at::Tensor aux, int act, bool want_bgrad) {
  check_cuda(dy, "dy");
  dy = dy.contiguous();
  aux = aux.contiguous();
  auto dx = at::empty_like(dy);
  auto db = act_backward(dy, aux, dx, act, want_bgrad);
  if (act == bh::kActNone) dx = dy;
  return {dx, db.defined() ? db : at::Tensor()};
}

}  // namespace

void register_dense(pybind11::module_& root) {
  namespace py = pybind11;
  auto fd = root.def_submodule("fused_dense_cuda", "GEMM + bias / GELU dense layers");
  fd.def("linear_bias_forward", &linear_bias_forward);
  fd.def("linear_bias_backward", &linear_bias_backward);
  fd.def("linear_gelu_linear_forward", &linear_gelu_linear_forward);
  fd.def("linear_gelu_linear_backward", &linear_gelu_linear_backward);
  fd.def("act_forward", &act_forward_py, py::arg("x"), py::arg("bias"), py::arg("act"));
  fd.def("act_backward", &act_backward_py, py::arg("dy"), py::arg("aux"), py::arg("act"), py::arg("want_bgrad"));
  auto mlp = root.def_submodule("mlp_cuda", "N-layer MLP");
  mlp.def("forward", &mlp_forward);
  mlp.def("backward", &mlp_backward);
  auto wg = root.def_submodule("fused_weight_gradient_mlp_cuda", "weight-gradient GEMM accumulated into main_grad");
  wg.def("wgrad_gemm_accum_fp32", &wgrad_gemm_accum_fp32);
  wg.def("wgrad_gemm_accum_fp16", &wgrad_gemm_accum_fp16);
}

}  // namespace bhb
