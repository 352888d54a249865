// `bn_fold`: kernels of the BatchNorm-backward fold (kernels/bn_fold.hip, bh/bn_fold_api.h).
#include "common.h"

#include "bh/bn_fold_api.h"

namespace bhb {
namespace {

bool half_2d(const at::Tensor& t) {
  return t.is_cuda() && t.dim() == 2 && t.is_contiguous() &&
         (t.scalar_type() == at::kHalf || t.scalar_type() == at::kBFloat16) &&
         (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

// (gram partials [S, K, K], column-sum partials [S, K]) of a' = a or relu(a * pro_scale + pro_shift)
std::vector<at::Tensor> gram(const at::Tensor& a, const c10::optional<at::Tensor>& pro_scale,
                             const c10::optional<at::Tensor>& pro_shift, int64_t s2_h, int64_t s2_w) {
  TORCH_CHECK(half_2d(a) && a.size(1) % 64 == 0 && a.size(0) > 0,
              "bn_fold.gram: a must be a contiguous 16-byte aligned fp16/bf16 [M, K] GPU tensor, K % 64 == 0");
  const int64_t M = s2_h > 0 ? a.size(0) / 4 : a.size(0), K = a.size(1);
  TORCH_CHECK(s2_h == 0 || (s2_h % 2 == 0 && s2_w % 2 == 0 && a.size(0) % (s2_h * s2_w) == 0),
              "bn_fold.gram: stride-2 rows need a [N * s2_h * s2_w, K] input with even s2_h, s2_w");
  TORCH_CHECK(!(s2_h > 0 && pro_scale.has_value() && pro_scale->defined()), "bn_fold.gram: no prologue at stride 2");
  const float *ps = nullptr, *ph = nullptr;
  at::Tensor psc, phc;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "bn_fold.gram: pro_scale and pro_shift together");
    psc = pro_scale->contiguous();
    phc = pro_shift->contiguous();
    TORCH_CHECK(psc.is_cuda() && phc.is_cuda() && psc.scalar_type() == at::kFloat && phc.scalar_type() == at::kFloat &&
                    psc.numel() == K && phc.numel() == K,
                "bn_fold.gram: pro_scale / pro_shift must be fp32 [K] GPU tensors");
    ps = psc.data_ptr<float>();
    ph = phc.data_ptr<float>();
  }
  const int S = bh::gram_splits(M, (int)K);
  auto gp = at::empty({S, K, K}, a.options().dtype(at::kFloat));
  auto cp = at::empty({S, K}, a.options().dtype(at::kFloat));
  bh::gram_partials(dtype_code(a.scalar_type()), a.data_ptr(), M, (int)K, ps, ph, gp.data_ptr<float>(),
                    cp.data_ptr<float>(), stream_for(a), (int)s2_h, (int)s2_w);
  return {gp, cp};
}

// (g * bits, column-sum partials [S, N] of the result)
std::vector<at::Tensor> mask_colsum(const at::Tensor& g, const at::Tensor& bits) {
  TORCH_CHECK(half_2d(g) && g.size(1) % 8 == 0, "bn_fold.mask_colsum: g must be a contiguous fp16/bf16 [M, N] tensor");
  const int64_t M = g.size(0), N = g.size(1);
  TORCH_CHECK(bits.is_cuda() && bits.scalar_type() == at::kByte && bits.is_contiguous() && bits.numel() == M * N / 8 &&
                  bits.device() == g.device(),
              "bn_fold.mask_colsum: bits must be a contiguous uint8 [M, N/8] tensor on g's device");
  const int S = bh::mask_colsum_splits(M, (int)N);
  auto out = at::empty_like(g);
  auto part = at::empty({S, N}, g.options().dtype(at::kFloat));
  bh::mask_colsum(dtype_code(g.scalar_type()), g.data_ptr(), bits.data_ptr<uint8_t>(), out.data_ptr(), M, (int)N,
                  part.data_ptr<float>(), stream_for(g));
  return {out, part};
}

void check_f32(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == numel, "bn_fold: ", what,
              " must be a contiguous fp32 GPU tensor of ", numel, " elements");
}

// stage 1: (P [N, K], Gm [K, K], Sa [K], sums [2N], bn_grads [2N]) from the partials of the weight-gradient,
// Gram and mask kernels; sums = this rank's [sum g, sum g (y - mean)], bn_grads = (dgamma, dbeta) local
std::vector<at::Tensor> fold_reduce(const at::Tensor& W, const at::Tensor& p_ws, const at::Tensor& g_ws,
                                    const at::Tensor& sa_ws, const at::Tensor& sg_ws, const at::Tensor& mean,
                                    const at::Tensor& invstd) {
  TORCH_CHECK(half_2d(W), "bn_fold.fold_reduce: W must be a contiguous fp16/bf16 [N, K] tensor");
  const int64_t N = W.size(0), K = W.size(1);
  TORCH_CHECK(p_ws.dim() == 2 && p_ws.size(1) == N * K && g_ws.dim() == 3 && g_ws.size(1) == K && g_ws.size(2) == K &&
                  sa_ws.dim() == 2 && sa_ws.size(1) == K && sa_ws.size(0) == g_ws.size(0) && sg_ws.dim() == 2 &&
                  sg_ws.size(1) == N,
              "bn_fold.fold_reduce: partial shapes");
  for (const at::Tensor* t : {&p_ws, &g_ws, &sa_ws, &sg_ws}) check_f32(*t, t->numel(), "partials");
  check_f32(mean, N, "mean");
  check_f32(invstd, N, "invstd");
  auto o = W.options().dtype(at::kFloat);
  auto P = at::empty({N, K}, o), Gm = at::empty({K, K}, o), Sa = at::empty({K}, o);
  auto sums = at::empty({2 * N}, o), bn_grads = at::empty({2 * N}, o);
  bh::fold_reduce(dtype_code(W.scalar_type()), W.data_ptr(), p_ws.data_ptr<float>(), (int)p_ws.size(0),
                  g_ws.data_ptr<float>(), sa_ws.data_ptr<float>(), (int)g_ws.size(0), sg_ws.data_ptr<float>(),
                  (int)sg_ws.size(0), mean.data_ptr<float>(), invstd.data_ptr<float>(), (int)N, (int)K,
                  P.data_ptr<float>(), Gm.data_ptr<float>(), Sa.data_ptr<float>(), sums.data_ptr<float>(),
                  bn_grads.data_ptr<float>(), stream_for(W));
  return {P, Gm, Sa, sums, bn_grads};
}

// stage 2 (after the sums' all-reduce): (dW [N, K] in W's dtype, abd [3N] fp32 = (A, B, D)) -- the
// BatchNorm input gradient is A g + B y + D per channel
std::vector<at::Tensor> fold_finish(const at::Tensor& W, const at::Tensor& sums, const at::Tensor& count,
                                    const at::Tensor& mean, const at::Tensor& invstd,
                                    const c10::optional<at::Tensor>& weight, const at::Tensor& P, const at::Tensor& Gm,
                                    const at::Tensor& Sa) {
  TORCH_CHECK(half_2d(W), "bn_fold.fold_finish: W must be a contiguous fp16/bf16 [N, K] tensor");
  const int64_t N = W.size(0), K = W.size(1);
  check_f32(sums, 2 * N, "sums");
  check_f32(count, 1, "count");
  check_f32(mean, N, "mean");
  check_f32(invstd, N, "invstd");
  check_f32(P, N * K, "P");
  check_f32(Gm, K * K, "Gm");
  check_f32(Sa, K, "Sa");
  const float* wp = nullptr;
  if (weight.has_value() && weight->defined()) {
    check_f32(*weight, N, "weight");
    wp = weight->data_ptr<float>();
  }
  auto abd = at::empty({3 * N}, W.options().dtype(at::kFloat));
  auto dW = at::empty({N, K}, W.options());
  bh::fold_finish(dtype_code(W.scalar_type()), W.data_ptr(), sums.data_ptr<float>(), count.data_ptr<float>(),
                  mean.data_ptr<float>(), invstd.data_ptr<float>(), wp, P.data_ptr<float>(), Gm.data_ptr<float>(),
                  Sa.data_ptr<float>(), (int)N, (int)K, abd.data_ptr<float>(), dW.data_ptr(), stream_for(W));
  return {dW, abd};
}

}  // namespace

void register_bn_fold(pybind11::module_& root) {
  auto m = root.def_submodule("bn_fold", "BatchNorm-backward fold: Gram partials, residual-ReLU mask + column sums");
  m.def("gram", &gram, py::arg("a"), py::arg("pro_scale") = py::none(), py::arg("pro_shift") = py::none(),
        py::arg("s2_h") = 0, py::arg("s2_w") = 0);
  m.def("mask_colsum", &mask_colsum, py::arg("g"), py::arg("bits"));
  m.def("fold_reduce", &fold_reduce, py::arg("W"), py::arg("p_ws"), py::arg("g_ws"), py::arg("sa_ws"), py::arg("sg_ws"),
        py::arg("mean"), py::arg("invstd"));
  m.def("fold_finish", &fold_finish, py::arg("W"), py::arg("sums"), py::arg("count"), py::arg("mean"), py::arg("invstd"),
        py::arg("weight"), py::arg("P"), py::arg("Gm"), py::arg("Sa"));
}

}  // namespace bhb
