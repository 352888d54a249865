// Megatron fused softmax modules + xentropy front-ends. Reference APIs:
// csrc/megatron/scaled_{upper_triang_masked,masked,}softmax*.cpp, generic_scaled_masked_softmax*.cpp,
// apex/contrib/csrc/xentropy/interface.cpp:50-51. Kernels: kernels/softmax.hip.
#include "common.h"

#include "bh/softmax_api.h"

namespace bhb {
namespace {

bool al16(const at::Tensor& t) { return !t.defined() || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

void check_half(const at::Tensor& t) {
  check_cuda(t, "input");
  TORCH_CHECK(t.scalar_type() == at::kHalf || t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat,
              "fused softmax: fp16 / bf16 / fp32 input expected");
}

// padding mask: input [b, np, sq, sk], mask [b or 1, 1, sq, sk]
at::Tensor masked_fwd(at::Tensor input, at::Tensor mask, double scale) {
  check_half(input);
  TORCH_CHECK(input.dim() == 4, "input must be [b, np, sq, sk]");
  input = input.contiguous();
  const int64_t b = input.size(0), np = input.size(1), sq = input.size(2), sk = input.size(3);
  at::Tensor m;
  int mb = 1;
  if (mask.defined()) {
    TORCH_CHECK(mask.dim() == 4 && mask.size(2) == sq && mask.size(3) == sk && mask.size(1) == 1,
                "mask must be [b or 1, 1, sq, sk]");
    m = (mask.scalar_type() == at::kBool ? mask.view(at::kByte) : mask.to(at::kByte)).contiguous();
    mb = (int)m.size(0);
    TORCH_CHECK(mb == 1 || mb == b, "mask batch must be 1 or b");
  }
  auto y = at::empty_like(input);
  const bool vec = (sk % 8 == 0) && al16(input) && al16(y) && (!m.defined() || reinterpret_cast<uintptr_t>(m.data_ptr()) % 8 == 0);
  bh::softmax_forward(dtype_code(input.scalar_type()), input.data_ptr(), m.defined() ? m.data_ptr<uint8_t>() : nullptr,
                      y.data_ptr(), b * np * sq, (int)sq, (int)sk, (int)np, mb, m.defined() ? 1 : 0, (float)scale, vec,
                      stream_for(input));
  return y;
}

// backward: in place on output_grads (reference semantics)
at::Tensor generic_bwd(at::Tensor dy, at::Tensor y, double scale, int mode, int sq) {
  check_half(y);
  TORCH_CHECK(dy.sizes() == y.sizes(), "grad/output shape mismatch");
  dy = dy.contiguous();
  y = y.contiguous();
  const int64_t sk = y.size(-1);
  const int64_t rows = y.numel() / sk;
  const bool vec = (sk % 8 == 0) && al16(dy) && al16(y);
  bh::softmax_backward(dtype_code(y.scalar_type()), dy.data_ptr(), y.data_ptr(), dy.data_ptr(), rows, sq, (int)sk,
                       mode, (float)scale, vec, stream_for(y));
  return dy;
}

at::Tensor masked_bwd(at::Tensor dy, at::Tensor y, double scale) { return generic_bwd(dy, y, scale, 0, 1); }

at::Tensor softmax_fwd(at::Tensor input, double scale) { return masked_fwd(input.dim() == 4 ? input : input.unsqueeze(0), at::Tensor(), scale).view(input.sizes()); }

// causal: input [attn_batches, sq, sk] with sq == sk
at::Tensor causal_fwd(at::Tensor input, double scale) {
  check_half(input);
  TORCH_CHECK(input.dim() == 3 && input.size(1) == input.size(2), "input must be [attn_batches, sq, sq]");
  input = input.contiguous();
  const int64_t ab = input.size(0), sq = input.size(1);
  auto y = at::empty_like(input);
  const bool vec = (sq % 8 == 0) && al16(input) && al16(y);
  bh::softmax_forward(dtype_code(input.scalar_type()), input.data_ptr(), nullptr, y.data_ptr(), ab * sq, (int)sq,
                      (int)sq, 1, 1, 2, (float)scale, vec, stream_for(input));
  return y;
}

at::Tensor causal_bwd(at::Tensor dy, at::Tensor y, double scale) {
  return generic_bwd(dy, y, scale, 2, (int)y.size(1));
}

int64_t get_batch_per_block(int64_t sq, int64_t sk, int64_t b, int64_t np) {
  // rows are scheduled independently (wave or workgroup per row): no divisibility constraint
  return 1;
}

std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor labels, double smoothing, bool half_to_float) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, V]");
  logits = logits.contiguous();
  labels = labels.to(at::kLong).contiguous();
  const int64_t N = logits.size(0), V = logits.size(1);
  auto ldt = half_to_float ? at::kFloat : logits.scalar_type();
  auto loss = at::empty({N}, logits.options().dtype(ldt));
  auto lse = at::empty({N}, logits.options().dtype(at::kFloat));
  const bool vec = (V % 8 == 0) && al16(logits);
  bh::xentropy_forward(dtype_code(logits.scalar_type()), logits.data_ptr(), labels.data_ptr<int64_t>(),
                       dtype_code(ldt), loss.data_ptr(), lse.data_ptr<float>(), N, (int)V, (float)smoothing, vec,
                       stream_for(logits));
  return {loss, lse};
}

at::Tensor xent_bwd(at::Tensor grad_loss, at::Tensor logits, at::Tensor lse, at::Tensor labels, double smoothing) {
  check_cuda(logits, "logits");
  logits = logits.contiguous();
  grad_loss = grad_loss.contiguous();
  labels = labels.to(at::kLong).contiguous();
  lse = lse.to(at::kFloat).contiguous();
  const int64_t N = logits.size(0), V = logits.size(1);
  auto dx = at::empty_like(logits);
  const bool vec = (V % 8 == 0) && al16(logits) && al16(dx);
  bh::xentropy_backward(dtype_code(logits.scalar_type()), logits.data_ptr(), dtype_code(grad_loss.scalar_type()),
                        grad_loss.data_ptr(), lse.data_ptr<float>(), labels.data_ptr<int64_t>(), dx.data_ptr(), N,
                        (int)V, (float)smoothing, vec, stream_for(logits));
  return dx;
}

// vocab-parallel CE: logits [rows, V] (this rank's shard), target [rows] global ids
at::Tensor vp_stats(at::Tensor logits, at::Tensor target, int64_t start) {
  check_cuda(logits, "logits");
  logits = logits.contiguous();
  target = target.to(at::kLong).contiguous();
  const int64_t V = logits.size(-1), N = logits.numel() / std::max<int64_t>(V, 1);
  TORCH_CHECK(target.numel() == N, "vocab_parallel_xent: target has ", target.numel(), " elements, expected ", N);
  auto stats = at::empty({N, 4}, logits.options().dtype(at::kFloat));
  const bool vec = (V % 8 == 0) && al16(logits);
  bh::vocab_xent_stats(dtype_code(logits.scalar_type()), logits.data_ptr(), target.data_ptr<int64_t>(),
                       stats.data_ptr<float>(), N, (int)V, start, vec, stream_for(logits));
  return stats;
}

// gathered [world, rows, 4] -> (loss[rows] in out_dtype, lse[rows] fp32)
std::vector<at::Tensor> vp_combine(at::Tensor gathered, at::ScalarType out_dtype) {
  check_cuda(gathered, "stats");
  gathered = gathered.contiguous();
  TORCH_CHECK(gathered.dim() == 3 && gathered.size(2) == 4 && gathered.scalar_type() == at::kFloat,
              "vocab_parallel_xent: stats must be float [world, rows, 4]");
  const int64_t rows = gathered.size(1);
  auto loss = at::empty({rows}, gathered.options().dtype(out_dtype));
  auto lse = at::empty({rows}, gathered.options());
  bh::vocab_xent_combine(gathered.data_ptr<float>(), (int)gathered.size(0), rows, dtype_code(out_dtype),
                         loss.data_ptr(), lse.data_ptr<float>(), stream_for(gathered));
  return {loss, lse};
}

}  // namespace

void register_softmax(pybind11::module_& root) {
  namespace py = pybind11;
  auto causal = root.def_submodule("scaled_upper_triang_masked_softmax_cuda", "causal scaled softmax");
  causal.def("forward", &causal_fwd);
  causal.def("backward", &causal_bwd);
  auto masked = root.def_submodule("scaled_masked_softmax_cuda", "padding-masked scaled softmax");
  masked.def("forward", &masked_fwd);
  masked.def("backward", &masked_bwd);
  masked.def("get_batch_per_block", &get_batch_per_block);
  auto plain = root.def_submodule("scaled_softmax_cuda", "scaled softmax");
  plain.def("forward", &softmax_fwd);
  plain.def("backward", &masked_bwd);
  auto generic = root.def_submodule("generic_scaled_masked_softmax_cuda", "masked softmax, any sk");
  generic.def("forward", &masked_fwd);
  generic.def("backward", &masked_bwd);
  auto xent = root.def_submodule("xentropy_cuda", "softmax cross-entropy with label smoothing");
  xent.def("forward", &xent_fwd);
  xent.def("backward", &xent_bwd);
  xent.def("vocab_parallel_stats", &vp_stats);
  xent.def("vocab_parallel_combine", &vp_combine);
}

}  // namespace bhb
