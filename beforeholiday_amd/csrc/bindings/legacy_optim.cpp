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

const int* flag_ptr(const c10::optional<at::Tensor>& f) {
  if (!f.has_value() || !f->defined() || f->numel() == 0) return nullptr;
  TORCH_CHECK(f->is_cuda() && f->scalar_type() == at::kInt, "overflow_flag must be GPU int32");
  return f->data_ptr<int>();
}

void maybe_cast(c10::optional<at::Tensor> overflow_flag, at::Tensor p_in, at::Tensor p_out) {
  const int64_t n = p_in.numel();
  check_same(p_in, n, "p_in");
  check_same(p_out, n, "p_out");
  bh::maybe_cast(n, flag_ptr(overflow_flag), dtype_code(p_in.scalar_type()), p_in.data_ptr(),
                 dtype_code(p_out.scalar_type()), p_out.data_ptr(), stream_for(p_in));
}

void maybe_cast_mt(int64_t chunk_size, c10::optional<at::Tensor> overflow_flag,
                   std::vector<std::vector<at::Tensor>> lists) {
  TORCH_CHECK(lists.size() == 2, "maybe_cast_mt: tensor lists p_in, p_out");
  if (lists[0].empty()) return;
  const int dt_in = list_dtype(lists[0], "maybe_cast_mt");
  const int dt_out = list_dtype(lists[1], "maybe_cast_mt");
  const auto& plan = get_plan(lists, chunk_size);
  bh::maybe_cast_mt(plan.view, flag_ptr(overflow_flag), dt_in, dt_out, stream_for(lists[0][0]));
}

const float* fptr(const at::Tensor& t, const char* name, int64_t n) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() >= n, name,
              " must be a contiguous GPU fp32 tensor with >= ", n, " elements");
  return t.data_ptr<float>();
}

void lamb_compute_update_term(int64_t chunk_size, at::Tensor noop, std::vector<std::vector<at::Tensor>> lists,
                              at::Tensor beta1, at::Tensor beta2, at::Tensor beta3, at::Tensor bias_correction,
                              at::Tensor step, at::Tensor eps, int64_t mode, at::Tensor decay,
                              at::Tensor global_scale, at::Tensor global_grad_norm, double max_grad_norm) {
  TORCH_CHECK(lists.size() == 5, "multi_tensor_lamb_compute_update_term: lists g, p, m, v, u");
  if (lists[0].empty()) return;
  const int64_t T = lists[0].size();
  const int dt_g = list_dtype(lists[0], "lamb_update_term");
  const int dt_p = list_dtype(lists[1], "lamb_update_term");
  TORCH_CHECK(list_dtype(lists[2], "lamb_update_term") == dt_p && list_dtype(lists[3], "lamb_update_term") == dt_p,
              "m / v must match p's dtype");
  TORCH_CHECK(list_dtype(lists[4], "lamb_update_term") == bh::kF32, "update term u must be fp32");
  TORCH_CHECK(bias_correction.scalar_type() == at::kInt && bias_correction.numel() >= T && step.scalar_type() == at::kInt,
              "bias_correction / step must be int32 GPU tensors");
  TORCH_CHECK(noop.is_cuda() && noop.scalar_type() == at::kInt, "noop_flag must be GPU int32");
  bh::DistLambStage1Args a{};
  a.beta1 = fptr(beta1, "per_tensor_beta1", T);
  a.beta2 = fptr(beta2, "per_tensor_beta2", T);
  a.beta3 = fptr(beta3, "per_tensor_beta3", T);
  a.eps = fptr(eps, "per_tensor_epsilon", T);
  a.decay = fptr(decay, "per_tensor_decay", T);
  a.bias_correction = bias_correction.data_ptr<int>();
  a.step = step.data_ptr<int>();
  a.global_scale = fptr(global_scale, "global_scale", 1);
  a.global_grad_norm = fptr(global_grad_norm, "global_grad_norm", 1);
  a.max_grad_norm = (float)max_grad_norm;
  a.mode = (int)mode;
  const auto& plan = get_plan(lists, chunk_size);
  bh::distopt_lamb_stage1(plan.view, dt_g, dt_p, a, noop.data_ptr<int>(), stream_for(lists[1][0]));
}

void lamb_update_weights(int64_t chunk_size, at::Tensor noop, std::vector<std::vector<at::Tensor>> lists,
                         at::Tensor param_norm, at::Tensor update_norm, at::Tensor update_norm_offset,
                         at::Tensor learning_rate, at::Tensor decay, at::Tensor global_grad_norm, bool use_nvlamb) {
  TORCH_CHECK(lists.size() == 2 || lists.size() == 3, "multi_tensor_lamb_update_weights: lists p, u [, p_copy]");
  (void)global_grad_norm;  // accepted for the reference signature (clipping happened in the update term)
  if (lists[0].empty()) return;
  const int64_t T = lists[0].size();
  const int dt_p = list_dtype(lists[0], "lamb_update_weights");
  TORCH_CHECK(list_dtype(lists[1], "lamb_update_weights") == bh::kF32, "update term u must be fp32");
  const int dt_c = lists.size() == 3 ? list_dtype(lists[2], "lamb_update_weights") : -1;
  TORCH_CHECK(update_norm_offset.scalar_type() == at::kLong && update_norm_offset.numel() >= T && update_norm_offset.is_cuda(),
              "update_norm_offset must be a GPU int64 tensor");
  TORCH_CHECK(noop.is_cuda() && noop.scalar_type() == at::kInt, "noop_flag must be GPU int32");
  bh::DistLambStage2Args a{};
  a.param_norm = fptr(param_norm, "per_tensor_param_norm", T);
  a.update_norm = fptr(update_norm, "per_tensor_update_norm", 1);
  a.update_norm_offset = update_norm_offset.data_ptr<int64_t>();
  a.lr = fptr(learning_rate, "learning_rate", 1);
  a.decay = fptr(decay, "per_tensor_decay", T);
  a.use_nvlamb = use_nvlamb;
  const auto& plan = get_plan(lists, chunk_size);
  bh::distopt_lamb_stage2(plan.view, dt_p, dt_c, a, noop.data_ptr<int>(), stream_for(lists[0][0]));
}

void dist_fused_adam(int64_t chunk_size, at::Tensor noop, std::vector<std::vector<at::Tensor>> lists,
                     at::Tensor beta1, at::Tensor beta2, at::Tensor bias_correction, at::Tensor eps,
                     at::Tensor weight_decay, double lr, double grad_scale, int64_t step, int64_t mode) {
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "multi_tensor_fused_adam: lists p, m, v, g [, p_copy]");
  (void)noop;
  if (lists[0].empty()) return;
  const int64_t T = lists[0].size();
  const int dt_p = list_dtype(lists[0], "dist_adam");
  TORCH_CHECK(list_dtype(lists[1], "dist_adam") == dt_p && list_dtype(lists[2], "dist_adam") == dt_p,
              "m / v must match p's dtype");
  const int dt_g = list_dtype(lists[3], "dist_adam");
  const int dt_c = lists.size() == 5 ? list_dtype(lists[4], "dist_adam") : -1;
  TORCH_CHECK(bias_correction.is_cuda() && bias_correction.scalar_type() == at::kInt && bias_correction.numel() >= T,
              "per_tensor_bias_correction must be a GPU int32 tensor");
  bh::DistAdamArgs a{};
  a.beta1 = fptr(beta1, "per_tensor_beta1", T);
  a.beta2 = fptr(beta2, "per_tensor_beta2", T);
  a.eps = fptr(eps, "per_tensor_eps", T);
  a.decay = fptr(weight_decay, "per_tensor_weight_decay", T);
  a.bias_correction = bias_correction.data_ptr<int>();
  a.lr = (float)lr;
  a.grad_scale = (float)grad_scale;
  a.step = (int)step;
  a.mode = (int)mode;
  const auto& plan = get_plan(lists, chunk_size);
  bh::distopt_adam(plan.view, dt_p, dt_g, dt_c, a, stream_for(lists[0][0]));
}

}  // namespace

void register_legacy_optim(pybind11::module_& root) {
  auto da = root.def_submodule("distributed_adam_cuda", "per-tensor hyper-parameter multi-tensor Adam (gfx950)");
  da.def("multi_tensor_fused_adam", &dist_fused_adam, "Multi tensor Adam with per-tensor hyper-parameters.");
  auto dl = root.def_submodule("distributed_lamb_cuda", "ZeRO LAMB stages with device-resident scalars (gfx950)");
  dl.def("multi_tensor_lamb_compute_update_term", &lamb_compute_update_term, "Computes update term for LAMB optimizer");
  dl.def("multi_tensor_lamb_update_weights", &lamb_update_weights, "Applies update term for LAMB optimizer");
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
