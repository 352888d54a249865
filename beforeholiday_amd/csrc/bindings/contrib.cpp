// `focal_loss_cuda` and `fused_index_mul_2d` front-ends (reference APIs:
// apex/contrib/csrc/focal_loss/focal_loss_cuda.cpp, apex/contrib/csrc/index_mul_2d/index_mul_2d_cuda.cpp).
// Kernels: kernels/contrib.hip.
#include "common.h"

#include "bh/contrib_api.h"

namespace bhb {
namespace {

std::vector<at::Tensor> focal_fwd(at::Tensor cls_output, at::Tensor cls_targets, at::Tensor num_positives_sum,
                                  int64_t num_real_classes, double alpha, double gamma, double smoothing) {
  check_cuda(cls_output, "cls_output");
  TORCH_CHECK(cls_output.size(-1) >= num_real_classes, "Incorrect number of real classes.");
  TORCH_CHECK(cls_targets.scalar_type() == at::kLong, "Invalid label type.");
  cls_output = cls_output.contiguous();
  cls_targets = cls_targets.contiguous();
  const int64_t C = cls_output.size(-1);
  const int64_t rows = cls_output.numel() / std::max<int64_t>(C, 1);
  TORCH_CHECK(cls_targets.numel() == rows, "focal_loss: expected ", rows, " labels, got ", cls_targets.numel());
  auto num_pos = num_positives_sum.to(at::kFloat).contiguous();
  auto pgrad = at::empty_like(cls_output);
  auto loss = at::empty({}, cls_output.options().dtype(at::kFloat));
  const int parts = bh::focal_loss_parts(cls_output.numel());
  auto part = at::empty({parts}, cls_output.options().dtype(at::kFloat));
  bh::focal_loss_forward(dtype_code(cls_output.scalar_type()), cls_output.data_ptr(), cls_targets.data_ptr<int64_t>(),
                         pgrad.data_ptr(), part.data_ptr<float>(), parts, num_pos.data_ptr<float>(),
                         loss.data_ptr<float>(), rows, (int)C, (int)num_real_classes, (float)alpha, (float)gamma,
                         (float)smoothing, stream_for(cls_output));
  return {loss, pgrad};
}

at::Tensor focal_bwd(at::Tensor grad_output, at::Tensor partial_grad, at::Tensor num_positives_sum) {
  check_cuda(partial_grad, "partial_grad");
  TORCH_CHECK(partial_grad.is_contiguous(), "partial_grad must be contiguous");
  auto gout = grad_output.to(at::kFloat).contiguous();
  auto num_pos = num_positives_sum.to(at::kFloat).contiguous();
  bh::focal_loss_backward(dtype_code(partial_grad.scalar_type()), partial_grad.data_ptr(), gout.data_ptr<float>(),
                          num_pos.data_ptr<float>(), partial_grad.numel(), stream_for(partial_grad));
  return partial_grad;
}

void check_imul(const at::Tensor& in1, const at::Tensor& in2, const at::Tensor& idx) {
  check_cuda(in1, "in1");
  TORCH_CHECK(in1.dim() == 2 && in2.dim() == 2 && idx.dim() == 1, "index_mul_2d: in1/in2 2-D, idx 1-D");
  TORCH_CHECK(in1.size(1) == in2.size(1) && in2.size(0) == idx.size(0), "index_mul_2d: shape mismatch");
  TORCH_CHECK(in1.scalar_type() == in2.scalar_type(), "index_mul_2d: dtype mismatch");
  TORCH_CHECK(in1.is_contiguous() && in2.is_contiguous() && idx.is_contiguous(), "index_mul_2d: contiguous inputs");
  TORCH_CHECK(idx.scalar_type() == at::kLong, "index_mul_2d: idx must be int64");
}

void imul_fwd(at::Tensor out, at::Tensor in1, at::Tensor in2, at::Tensor idx) {
  check_imul(in1, in2, idx);
  bh::index_mul_2d_forward(dtype_code(in1.scalar_type()), out.data_ptr(), in1.data_ptr(), in2.data_ptr(),
                           idx.data_ptr<int64_t>(), in2.size(0), (int)in2.size(1), stream_for(in1));
}

// grad_in1 must be zero-initialised (like the reference)
void imul_bwd(at::Tensor grad_in1, at::Tensor grad_in2, at::Tensor grad_out, at::Tensor in1, at::Tensor in2,
              at::Tensor idx) {
  check_imul(in1, in2, idx);
  grad_out = grad_out.contiguous();
  const bool f32 = grad_in1.scalar_type() == at::kFloat;
  at::Tensor acc = f32 ? grad_in1 : grad_in1.to(at::kFloat);
  bh::index_mul_2d_backward(dtype_code(in1.scalar_type()), acc.data_ptr<float>(), f32 ? nullptr : grad_in1.data_ptr(),
                            in1.size(0), grad_in2.data_ptr(), grad_out.data_ptr(), in1.data_ptr(), in2.data_ptr(),
                            idx.data_ptr<int64_t>(), in2.size(0), (int)in2.size(1), stream_for(in1));
}

void imul_bwd_bwd(at::Tensor grad_grad_out, at::Tensor grad_in1, at::Tensor grad_in2, at::Tensor grad_out,
                  at::Tensor grad_grad_in1, at::Tensor grad_grad_in2, at::Tensor in1, at::Tensor in2, at::Tensor idx) {
  check_imul(in1, in2, idx);
  grad_out = grad_out.contiguous();
  grad_grad_in1 = grad_grad_in1.contiguous();
  grad_grad_in2 = grad_grad_in2.contiguous();
  const bool f32 = grad_in1.scalar_type() == at::kFloat;
  at::Tensor acc = f32 ? grad_in1 : grad_in1.to(at::kFloat);
  bh::index_mul_2d_backward_backward(dtype_code(in1.scalar_type()), grad_grad_out.data_ptr(), acc.data_ptr<float>(),
                                     f32 ? nullptr : grad_in1.data_ptr(), in1.size(0), grad_in2.data_ptr(),
                                     grad_out.data_ptr(), grad_grad_in1.data_ptr(), grad_grad_in2.data_ptr(),
                                     in1.data_ptr(), in2.data_ptr(), idx.data_ptr<int64_t>(), in2.size(0),
                                     (int)in2.size(1), stream_for(in1));
}

}  // namespace

void register_contrib(pybind11::module_& root) {
  auto fl = root.def_submodule("focal_loss_cuda", "sigmoid focal loss");
  fl.def("forward", &focal_fwd);
  fl.def("backward", &focal_bwd);
  auto im = root.def_submodule("fused_index_mul_2d", "out = in1[idx] * in2");
  for (const char* p : {"float_", "half_", "bfloat16_", ""}) {
    im.def((std::string(p) + "forward").c_str(), &imul_fwd);
    im.def((std::string(p) + "backward").c_str(), &imul_bwd);
    im.def((std::string(p) + "backward_backward").c_str(), &imul_bwd_bwd);
  }
}

}  // namespace bhb
