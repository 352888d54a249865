// `fused_layer_norm_cuda` front-end (reference API: csrc/layer_norm_cuda.cpp:428-441).
// Kernels: kernels/layer_norm.hip.
#include "common.h"

#include "bh/knobs.h"
#include "bh/ln_api.h"

namespace bhb {
namespace {

struct Dims {
  int64_t n1;
  int n2;
};

Dims dims_of(const at::Tensor& x, at::IntArrayRef normalized_shape) {
  const int nd = (int)normalized_shape.size();
  TORCH_CHECK(nd >= 1 && x.dim() >= nd, "normalized_shape must match the trailing input dims");
  int64_t n2 = 1;
  for (int i = 0; i < nd; ++i) {
    TORCH_CHECK(x.size(x.dim() - nd + i) == normalized_shape[i], "input trailing dims ", x.sizes(),
                " do not match normalized_shape ", normalized_shape);
    n2 *= normalized_shape[i];
  }
  TORCH_CHECK(n2 < INT32_MAX, "normalized size too large");
  return {x.numel() / std::max<int64_t>(n2, 1), (int)n2};
}

bool al16(const at::Tensor& t) { return !t.defined() || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

bool use_vec(int n2, std::initializer_list<at::Tensor> ts) {
  if (n2 % 8) return false;
  for (const auto& t : ts)
    if (!al16(t)) return false;
  return true;
}

int wc(const at::Tensor& w) { return w.defined() ? dtype_code(w.scalar_type()) : -1; }
const void* wp(const at::Tensor& w) { return w.defined() ? w.data_ptr() : nullptr; }

// forward: returns (output, mean, invvar); rms -> mean undefined
std::vector<at::Tensor> fwd_impl(at::Tensor input, at::IntArrayRef shape, at::Tensor gamma, at::Tensor beta,
                                 double eps, bool rms, bool mixed) {
  check_cuda(input, "input");
  input = input.contiguous();
  if (gamma.defined()) gamma = gamma.contiguous();
  if (beta.defined()) beta = beta.contiguous();
  auto d = dims_of(input, shape);
  auto st = (mixed && gamma.defined()) ? gamma.scalar_type() : input.scalar_type();
  auto out = at::empty_like(input, input.options().dtype(st));
  std::vector<int64_t> stat_shape(input.sizes().begin(), input.sizes().end() - shape.size());
  auto fopt = input.options().dtype(at::kFloat);
  at::Tensor mean = rms ? at::Tensor() : at::empty(stat_shape, fopt);
  at::Tensor invvar = at::empty(stat_shape, fopt);
  const bool vec = use_vec(d.n2, {input, gamma, beta, out});
  bh::ln_forward(d.n1, d.n2, dtype_code(input.scalar_type()), input.data_ptr(), wc(gamma), wp(gamma), wp(beta),
                 dtype_code(out.scalar_type()), out.data_ptr(), rms ? nullptr : mean.data_ptr<float>(),
                 invvar.data_ptr<float>(), (float)eps, rms, vec, stream_for(input));
  if (rms) return {out, invvar};
  return {out, mean, invvar};
}

// backward: returns (grad_input, grad_gamma, grad_beta) (grads undefined when not affine)
std::vector<at::Tensor> bwd_impl(at::Tensor dout, at::Tensor mean, at::Tensor invvar, at::Tensor input_or_output,
                                 at::IntArrayRef shape, at::Tensor gamma, at::Tensor beta, double eps, bool rms,
                                 bool memory_efficient, at::Tensor dresid = at::Tensor()) {
  check_cuda(dout, "grad_output");
  dout = dout.contiguous();
  at::Tensor xin = input_or_output.contiguous();
  if (gamma.defined()) gamma = gamma.contiguous();
  if (beta.defined()) beta = beta.contiguous();
  auto d = dims_of(xin, shape);
  auto dx = at::empty_like(xin);
  if (dresid.defined()) {
    dresid = dresid.contiguous();
    TORCH_CHECK(dresid.scalar_type() == dx.scalar_type() && dresid.numel() == dx.numel() && dresid.is_cuda(),
                "layer_norm backward: dresid must match the input's dtype and size");
  }
  const bool vec = use_vec(d.n2, {dout, xin, gamma, beta, dx, dresid});
  hipStream_t s = stream_for(xin);
  // memory-efficient backward recomputes x_hat from the output: mean is not saved and never read
  const float* mp = (rms || memory_efficient) ? nullptr : mean.data_ptr<float>();
  TORCH_CHECK(rms || memory_efficient || mean.numel() == d.n1, "layer_norm backward: mean has ", mean.numel(),
              " elements, expected ", d.n1);
  TORCH_CHECK(invvar.numel() == d.n1, "layer_norm backward: invvar has ", invvar.numel(), " elements, expected ", d.n1);
  // Config.ln_bwd_fused: dx and the parameter-gradient partials in one pass (else two; measured faster in
  // BERT-large, profiles/ln_bwd_fused_ab_r6.txt)
  const int fblocks = gamma.defined() && bh::knob("ln_bwd_fused", 0) ? bh::ln_bwd_fused_blocks(d.n1, d.n2) : 0;
  if (fblocks > 0) {  // one pass for dx and the parameter gradients
    at::Tensor gg = at::empty_like(gamma), gb;
    if (!rms && beta.defined()) gb = at::empty_like(beta);
    auto part = at::empty({2 * (int64_t)fblocks * d.n2}, xin.options().dtype(at::kFloat));
    bh::ln_backward_fused(d.n1, d.n2, dtype_code(dout.scalar_type()), dout.data_ptr(), dtype_code(xin.scalar_type()),
                          xin.data_ptr(), mp, invvar.data_ptr<float>(), wc(gamma), wp(gamma), wp(beta), dx.data_ptr(),
                          gg.data_ptr(), gb.defined() ? gb.data_ptr() : nullptr, part.data_ptr<float>(), fblocks, rms,
                          memory_efficient, vec, s, dresid.defined() ? dresid.data_ptr() : nullptr);
    return {dx, gg, gb};
  }
  bh::ln_backward_dx(d.n1, d.n2, dtype_code(dout.scalar_type()), dout.data_ptr(), dtype_code(xin.scalar_type()),
                     xin.data_ptr(), mp, invvar.data_ptr<float>(), wc(gamma), wp(gamma), wp(beta), dx.data_ptr(), rms,
                     memory_efficient, vec, s, dresid.defined() ? dresid.data_ptr() : nullptr);
  at::Tensor gg, gb;
  if (gamma.defined()) {
    gg = at::empty_like(gamma);
    if (!rms && beta.defined()) gb = at::empty_like(beta);
    const int splits = bh::ln_wgrad_splits(d.n1, d.n2);
    auto part = at::empty({2 * (int64_t)splits * d.n2}, xin.options().dtype(at::kFloat));
    bh::ln_backward_wgrad(d.n1, d.n2, dtype_code(dout.scalar_type()), dout.data_ptr(), dtype_code(xin.scalar_type()),
                          xin.data_ptr(), mp, invvar.data_ptr<float>(), wc(gamma), wp(gamma), wp(beta), gg.data_ptr(),
                          gb.defined() ? gb.data_ptr() : nullptr, part.data_ptr<float>(), splits, rms, memory_efficient,
                          vec, s);
  }
  return {dx, gg, gb};
}

std::vector<at::Tensor> forward_affine(at::Tensor input, at::IntArrayRef shape, at::Tensor gamma, at::Tensor beta,
                                       double eps) {
  return fwd_impl(input, shape, gamma, beta, eps, false, false);
}
std::vector<at::Tensor> forward_affine_mixed_dtypes(at::Tensor input, at::IntArrayRef shape, at::Tensor gamma,
                                                    at::Tensor beta, double eps) {
  return fwd_impl(input, shape, gamma, beta, eps, false, true);
}
std::vector<at::Tensor> forward(at::Tensor input, at::IntArrayRef shape, double eps) {
  return fwd_impl(input, shape, at::Tensor(), at::Tensor(), eps, false, false);
}
std::vector<at::Tensor> rms_forward_affine(at::Tensor input, at::IntArrayRef shape, at::Tensor gamma, double eps) {
  return fwd_impl(input, shape, gamma, at::Tensor(), eps, true, false);
}
std::vector<at::Tensor> rms_forward_affine_mixed_dtypes(at::Tensor input, at::IntArrayRef shape, at::Tensor gamma,
                                                        double eps) {
  return fwd_impl(input, shape, gamma, at::Tensor(), eps, true, true);
}
std::vector<at::Tensor> rms_forward(at::Tensor input, at::IntArrayRef shape, double eps) {
  return fwd_impl(input, shape, at::Tensor(), at::Tensor(), eps, true, false);
}
std::vector<at::Tensor> backward_affine(at::Tensor dout, at::Tensor mean, at::Tensor invvar,
                                        at::Tensor input_or_output, at::IntArrayRef shape, at::Tensor gamma,
                                        at::Tensor beta, double eps, bool memory_efficient,
                                        c10::optional<at::Tensor> dresid) {
  return bwd_impl(dout, mean, invvar, input_or_output, shape, gamma, beta, eps, false, memory_efficient,
                  dresid.has_value() ? *dresid : at::Tensor());
}
at::Tensor backward(at::Tensor dout, at::Tensor mean, at::Tensor invvar, at::Tensor input_or_output,
                    at::IntArrayRef shape, double eps, bool memory_efficient) {
  return bwd_impl(dout, mean, invvar, input_or_output, shape, at::Tensor(), at::Tensor(), eps, false,
                  memory_efficient)[0];
}
std::vector<at::Tensor> rms_backward_affine(at::Tensor dout, at::Tensor invvar, at::Tensor input_or_output,
                                            at::IntArrayRef shape, at::Tensor gamma, double eps,
                                            bool memory_efficient) {
  auto r = bwd_impl(dout, at::Tensor(), invvar, input_or_output, shape, gamma, at::Tensor(), eps, true,
                    memory_efficient);
  return {r[0], r[1]};
}
at::Tensor rms_backward(at::Tensor dout, at::Tensor invvar, at::Tensor input_or_output, at::IntArrayRef shape,
                        double eps, bool memory_efficient) {
  return bwd_impl(dout, at::Tensor(), invvar, input_or_output, shape, at::Tensor(), at::Tensor(), eps, true,
                  memory_efficient)[0];
}

}  // namespace

void register_norms(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("fused_layer_norm_cuda", "LayerNorm / RMSNorm kernels (gfx950)");
  m.def("forward_affine", &forward_affine);
  m.def("forward_affine_mixed_dtypes", &forward_affine_mixed_dtypes);
  m.def("forward", &forward);
  m.def("rms_forward_affine", &rms_forward_affine);
  m.def("rms_forward_affine_mixed_dtypes", &rms_forward_affine_mixed_dtypes);
  m.def("rms_forward", &rms_forward);
  m.def("backward_affine", &backward_affine, py::arg("dout"), py::arg("mean"), py::arg("invvar"),
        py::arg("input_or_output"), py::arg("normalized_shape"), py::arg("gamma"), py::arg("beta"), py::arg("eps"),
        py::arg("memory_efficient") = false, py::arg("dresid") = py::none());
  m.def("backward", &backward, py::arg("dout"), py::arg("mean"), py::arg("invvar"), py::arg("input_or_output"),
        py::arg("normalized_shape"), py::arg("eps"), py::arg("memory_efficient") = false);
  m.def("rms_backward_affine", &rms_backward_affine, py::arg("dout"), py::arg("invvar"), py::arg("input_or_output"),
        py::arg("normalized_shape"), py::arg("gamma"), py::arg("eps"), py::arg("memory_efficient") = false);
  m.def("rms_backward", &rms_backward, py::arg("dout"), py::arg("invvar"), py::arg("input_or_output"),
        py::arg("normalized_shape"), py::arg("eps"), py::arg("memory_efficient") = false);
}

}  // namespace bhb
