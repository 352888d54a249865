// `fused_adam_cuda` front-end (deprecated contrib optimizer extension). Python signatures follow
// apex/contrib/csrc/optimizers/fused_adam_cuda.cpp:79-85; kernels: kernels/legacy_optim.hip.
#include "common.h"

#include <cmath>

#include "bh/legacy_api.h"

namespace bhb {
namespace {

bh::LegacyAdamArgs adam_args(double lr, double beta1, double beta2, double eps, double grad_scale, int64_t step,
                             int64_t mode, int64_t bias_correction, double decay) {
  bh::LegacyAdamArgs a{};
  double step_size = lr;
  if (bias_correction == 1) {
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    step_size = lr * std::sqrt(bc2) / bc1;
  }
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.grad_scale = (float)grad_scale;
  a.step_size = (float)step_size;
  a.decay = (float)decay;
  a.mode = (int)mode;
  return a;
}

void check_same(const at::Tensor& x, int64_t n, const char* name) {
  check_cuda(x, name);
  TORCH_CHECK(x.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(x.numel() == n, "number of elements in ", name, " and p tensors should be equal");
}

int copy_code(const at::Tensor& p_copy, int64_t n) {
  if (p_copy.numel() == 0) return -1;
  check_same(p_copy, n, "p_copy");
  return dtype_code(p_copy.scalar_type());
}

void adam(at::Tensor p, at::Tensor p_copy, at::Tensor m, at::Tensor v, at::Tensor g, double lr, double beta1,
          double beta2, double eps, double grad_scale, int64_t step, int64_t mode, int64_t bias_correction,
          double decay) {
  const int64_t n = p.numel();
  check_same(p, n, "p");
  check_same(m, n, "m");
  check_same(v, n, "v");
  check_same(g, n, "g");
  TORCH_CHECK(m.scalar_type() == p.scalar_type() && v.scalar_type() == p.scalar_type(), "m / v must match p's dtype");
  const int cc = copy_code(p_copy, n);
  bh::legacy_adam(n, dtype_code(p.scalar_type()), p.data_ptr(), cc, cc < 0 ? nullptr : p_copy.data_ptr(),
                  m.data_ptr(), v.data_ptr(), dtype_code(g.scalar_type()), g.data_ptr(),
                  adam_args(lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay), stream_for(p));
}

void reversible_adam(at::Tensor p, at::Tensor p_copy, at::Tensor m, at::Tensor v, at::Tensor g, double lr,
                     double beta1, double beta2, double eps, double grad_scale, int64_t step, int64_t mode,
                     int64_t bias_correction, double decay) {
  const int64_t n = p.numel();
  check_same(p, n, "p");
  check_same(m, n, "m");
  check_same(v, n, "v");
  check_same(g, n, "g");
  const int cc = copy_code(p_copy, n);
  auto scratch = at::zeros({1}, p.options().dtype(at::kInt));
  bh::legacy_reversible_adam(n, dtype_code(p.scalar_type()), p.data_ptr(), cc, cc < 0 ? nullptr : p_copy.data_ptr(),
                             m.data_ptr(), v.data_ptr(), dtype_code(g.scalar_type()), g.data_ptr(),
                             adam_args(lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay),
                             scratch.data_ptr<int>(), stream_for(p));
}

void maybe_adam_undo(at::Tensor overflow_flag, at::Tensor p, at::Tensor m, at::Tensor v, at::Tensor g, double lr,
                     double beta1, double beta2, double eps, double grad_scale, int64_t step, int64_t mode,
                     int64_t bias_correction, double decay) {
  const int64_t n = p.numel();
  check_same(p, n, "p");
  check_same(m, n, "m");
  check_same(v, n, "v");
  check_same(g, n, "g");
  TORCH_CHECK(overflow_flag.is_cuda() && overflow_flag.scalar_type() == at::kInt, "overflow_flag must be GPU int32");
  bh::legacy_adam_undo(n, overflow_flag.data_ptr<int>(), dtype_code(p.scalar_type()), p.data_ptr(), m.data_ptr(),
                       v.data_ptr(), dtype_code(g.scalar_type()), g.data_ptr(),
                       adam_args(lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay), stream_for(p));
}

void adam_mt(int64_t chunk_size, at::Tensor overflow_flag, std::vector<std::vector<at::Tensor>> lists, double lr,
             double beta1, double beta2, double eps, double grad_scale, int64_t step, int64_t mode,
             int64_t bias_correction, double decay) {
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "adam_mt: tensor lists p, m, v, g [, p_copy]");
  (void)overflow_flag;  // accepted for the multi_tensor_applier signature; the legacy Adam never skips
  if (lists[0].empty()) return;
  const int dt_p = list_dtype(lists[0], "adam_mt");
  TORCH_CHECK(list_dtype(lists[1], "adam_mt") == dt_p && list_dtype(lists[2], "adam_mt") == dt_p,
              "adam_mt: m / v must match p's dtype");
  const int dt_g = list_dtype(lists[3], "adam_mt");
  const int dt_c = lists.size() == 5 ? list_dtype(lists[4], "adam_mt") : -1;
  const auto& plan = get_plan(lists, chunk_size);
  bh::legacy_adam_mt(plan.view, dt_g, dt_p, dt_c,
                     adam_args(lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay),
                     stream_for(lists[0][0]));
}

void strided_check_finite(at::Tensor overflow_flag, at::Tensor p_copy, int64_t stride, int64_t clear_overflow_first) {
  check_cuda(p_copy, "p_copy");
  TORCH_CHECK(p_copy.is_contiguous(), "p_copy must be contiguous");
  TORCH_CHECK(overflow_flag.is_cuda() && overflow_flag.scalar_type() == at::kInt, "overflow_flag must be GPU int32");
  bh::strided_check_finite(p_copy.numel(), overflow_flag.data_ptr<int>(), dtype_code(p_copy.scalar_type()),
                           p_copy.data_ptr(), (int)stride, clear_overflow_first != 0, stream_for(p_copy));
}

const int* flag_ptr(const at::Tensor& f) {
  if (!f.defined() || f.numel() == 0) return nullptr;
  TORCH_CHECK(f.is_cuda() && f.scalar_type() == at::kInt, "overflow_flag must be GPU int32");
  return f.data_ptr<int>();
}

void maybe_cast(at::Tensor overflow_flag, at::Tensor p_in, at::Tensor p_out) {
  const int64_t n = p_in.numel();
  check_same(p_in, n, "p_in");
  check_same(p_out, n, "p_out");
  bh::maybe_cast(n, flag_ptr(overflow_flag), dtype_code(p_in.scalar_type()), p_in.data_ptr(),
                 dtype_code(p_out.scalar_type()), p_out.data_ptr(), stream_for(p_in));
}

void maybe_cast_mt(int64_t chunk_size, at::Tensor overflow_flag, std::vector<std::vector<at::Tensor>> lists) {
  TORCH_CHECK(lists.size() == 2, "maybe_cast_mt: tensor lists p_in, p_out");
  if (lists[0].empty()) return;
  const int dt_in = list_dtype(lists[0], "maybe_cast_mt");
  const int dt_out = list_dtype(lists[1], "maybe_cast_mt");
  const auto& plan = get_plan(lists, chunk_size);
  bh::maybe_cast_mt(plan.view, flag_ptr(overflow_flag), dt_in, dt_out, stream_for(lists[0][0]));
}

}  // namespace

void register_legacy_optim(pybind11::module_& root) {
  auto m = root.def_submodule("fused_adam_cuda", "deprecated contrib Adam kernels + e5m2 casts (gfx950)");
  m.def("strided_check_finite", &strided_check_finite, "Strided finite check.");
  m.def("adam", &adam, "Adam (legacy update rule).");
  m.def("reversible_adam", &reversible_adam, "Adam that skips non-finite gradients and flags p_copy[0].");
  m.def("adam_mt", &adam_mt, "Multi-tensor Adam (legacy update rule).");
  m.def("maybe_adam_undo", &maybe_adam_undo, "Undo one Adam step when overflow_flag is set.");
  m.def("maybe_cast", &maybe_cast, "Cast between fp32 / fp16 / bf16 / e5m2 bytes unless overflow_flag is set.");
  m.def("maybe_cast_mt", &maybe_cast_mt, "Multi-tensor maybe_cast.");
}

}  // namespace bhb
