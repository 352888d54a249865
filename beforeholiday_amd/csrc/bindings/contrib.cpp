// `focal_loss_cuda` and `fused_index_mul_2d` front-ends (reference APIs:
// apex/contrib/csrc/focal_loss/focal_loss_cuda.cpp, apex/contrib/csrc/index_mul_2d/index_mul_2d_cuda.cpp).
// Kernels: kernels/contrib.hip.
#include "common.h"

#include "bh/contrib_api.h"
#include "bh/attn_api.h"
#include "bh/mha_api.h"
#include "bh/sparsity_api.h"
#include "bh/transducer_api.h"

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

// scores [B*heads, sq, sk] -> (softmax, dropped probabilities or undefined)
std::vector<at::Tensor> mha_softmax_fwd(at::Tensor scores, c10::optional<at::Tensor> mask, int64_t mask_mode,
                                        int64_t heads, double p_drop, int64_t seed, int64_t offset, bool training) {
  check_cuda(scores, "scores");
  scores = scores.contiguous();
  TORCH_CHECK(scores.dim() == 3, "mha softmax: scores must be [B*heads, sq, sk]");
  const int64_t sq = scores.size(1), sk = scores.size(2), rows = scores.size(0) * sq;
  TORCH_CHECK(sk <= bh::mha_max_sk(), "mha softmax: sk ", sk, " > ", bh::mha_max_sk());
  at::Tensor m;
  int dt_mask = bh::kF32;
  if (mask_mode != 0) {
    TORCH_CHECK(mask.has_value() && mask->defined(), "mha softmax: mask required");
    m = mask->contiguous();
    if (mask_mode == 1 || mask_mode == 3) m = m.to(at::kByte);
    else dt_mask = dtype_code(m.scalar_type());
    const int64_t expect = (mask_mode == 3) ? sq * sk : (scores.size(0) / heads) * sk;
    TORCH_CHECK(m.numel() == expect, "mha softmax: mask has ", m.numel(), " elements, expected ", expect);
  }
  auto sm = at::empty_like(scores);
  at::Tensor dropped;
  const bool drop = training && p_drop > 0.0;
  if (drop) dropped = at::empty_like(scores);
  const bool vec = (sk % 8 == 0) && reinterpret_cast<uintptr_t>(scores.data_ptr()) % 16 == 0;
  bh::mha_softmax_dropout_forward(dtype_code(scores.scalar_type()), scores.data_ptr(), (int)mask_mode, dt_mask,
                                  m.defined() ? m.data_ptr() : nullptr, sm.data_ptr(),
                                  drop ? dropped.data_ptr() : nullptr, rows, (int)sq, (int)sk, (int)heads,
                                  (float)p_drop, (uint64_t)seed, (uint64_t)offset, vec, stream_for(scores));
  return {sm, drop ? dropped : sm};
}

at::Tensor mha_softmax_bwd(at::Tensor dy, at::Tensor sm, double p_drop, int64_t seed, int64_t offset,
                           bool use_dropout) {
  check_cuda(dy, "dy");
  dy = dy.contiguous();
  sm = sm.contiguous();
  const int64_t sk = sm.size(-1), rows = sm.numel() / sk;
  auto dx = at::empty_like(sm);
  const bool vec = (sk % 8 == 0);
  bh::mha_softmax_dropout_backward(dtype_code(sm.scalar_type()), dy.data_ptr(), sm.data_ptr(), dx.data_ptr(), rows,
                                   (int)sk, (float)p_drop, (uint64_t)seed, (uint64_t)offset, use_dropout && p_drop > 0,
                                   vec, stream_for(sm));
  return dx;
}

// transducer loss: returns (alpha, beta, loss)
std::vector<at::Tensor> td_loss_fwd(at::Tensor x, at::Tensor label, at::Tensor f_len, at::Tensor y_len,
                                    at::Tensor batch_offset, int64_t max_f_len, int64_t blank_idx, int64_t opt,
                                    bool packed_input) {
  check_cuda(x, "x");
  x = x.contiguous();
  label = label.to(at::kLong).contiguous();
  auto fl = f_len.to(at::kInt).contiguous();
  auto yl = y_len.to(at::kInt).contiguous();
  const int64_t B = fl.numel();
  const int64_t V = x.size(-1);
  const int64_t max_u1 = packed_input ? (label.size(1) + 1) : x.size(2);
  const int64_t max_t = packed_input ? max_f_len : x.size(1);
  at::Tensor bo;
  if (packed_input) bo = batch_offset.to(at::kLong).contiguous();
  auto fopt = x.options().dtype(at::kFloat);
  auto alpha = at::empty({B, max_t, max_u1}, fopt);
  auto beta = at::empty({B, max_t, max_u1}, fopt);
  auto loss = at::empty({B}, fopt);
  bh::transducer_loss_forward(dtype_code(x.scalar_type()), x.data_ptr(), label.data_ptr<int64_t>(),
                              (int)label.size(1), fl.data_ptr<int>(), yl.data_ptr<int>(),
                              packed_input ? bo.data_ptr<int64_t>() : nullptr, (int)B, (int)max_t, (int)max_u1,
                              (int)V, (int)blank_idx, alpha.data_ptr<float>(), beta.data_ptr<float>(),
                              loss.data_ptr<float>(), stream_for(x));
  return {alpha, beta, loss};
}

at::Tensor td_loss_bwd(at::Tensor x, at::Tensor loss_grad, at::Tensor alpha, at::Tensor beta, at::Tensor f_len,
                       at::Tensor y_len, at::Tensor label, at::Tensor batch_offset, int64_t max_f_len,
                       int64_t blank_idx, int64_t opt, bool fuse_softmax_backward, bool packed_input) {
  check_cuda(x, "x");
  x = x.contiguous();
  label = label.to(at::kLong).contiguous();
  auto fl = f_len.to(at::kInt).contiguous();
  auto yl = y_len.to(at::kInt).contiguous();
  auto lg = loss_grad.to(at::kFloat).contiguous();
  const int64_t B = fl.numel();
  at::Tensor bo;
  if (packed_input) bo = batch_offset.to(at::kLong).contiguous();
  auto dx = packed_input ? at::zeros_like(x) : at::empty_like(x);
  bh::transducer_loss_backward(dtype_code(x.scalar_type()), x.data_ptr(), lg.data_ptr<float>(),
                               alpha.data_ptr<float>(), beta.data_ptr<float>(), label.data_ptr<int64_t>(),
                               (int)label.size(1), fl.data_ptr<int>(), yl.data_ptr<int>(),
                               packed_input ? bo.data_ptr<int64_t>() : nullptr, (int)B, (int)alpha.size(1),
                               (int)alpha.size(2), (int)x.size(-1), (int)blank_idx, fuse_softmax_backward,
                               dx.data_ptr(), stream_for(x));
  return dx;
}

bh::JointArgs joint_args(int64_t B, int64_t T, int64_t U, int64_t H, const at::Tensor& fl, const at::Tensor& gl,
                         const at::Tensor& bo, bool pack, int64_t rows, bool relu, bool dropout, double prob,
                         int64_t seed) {
  bh::JointArgs a{};
  a.B = (int)B;
  a.T = (int)T;
  a.U = (int)U;
  a.H = (int)H;
  a.rows = rows;
  a.f_len = fl.data_ptr<int>();
  a.g_len = gl.data_ptr<int>();
  a.batch_offset = pack ? bo.data_ptr<int64_t>() : nullptr;
  a.relu = relu;
  a.dropout = dropout && prob > 0.0;
  const double keep_thresh = prob * 4294967296.0;
  a.keep_thresh = (uint32_t)std::min(keep_thresh, 4294967295.0);
  a.scale = (a.dropout && prob < 1.0) ? (float)(1.0 / (1.0 - prob)) : 1.f;
  a.seed = (uint32_t)seed;
  return a;
}

// returns (out, mask) -- mask (uint8 per output element) only when want_mask
std::vector<at::Tensor> td_joint_fwd(at::Tensor f, at::Tensor g, at::Tensor f_len, at::Tensor g_len,
                                     at::Tensor batch_offset, int64_t packed_batch, bool pack_output, bool relu,
                                     bool dropout, double dropout_prob, int64_t seed, bool want_mask) {
  check_cuda(f, "f");
  check_cuda(g, "g");
  TORCH_CHECK(f.dim() == 3 && g.dim() == 3 && f.size(0) == g.size(0) && f.size(2) == g.size(2),
              "transducer_joint: f [B, T, H] and g [B, U, H]");
  TORCH_CHECK(f.scalar_type() == g.scalar_type(), "transducer_joint: f and g must share a dtype");
  TORCH_CHECK(f.size(2) % 8 == 0, "transducer_joint: hidden size must be a multiple of 8");
  f = f.contiguous();
  g = g.contiguous();
  auto fl = f_len.to(at::kInt).contiguous();
  auto gl = g_len.to(at::kInt).contiguous();
  TORCH_CHECK(fl.is_cuda() && gl.is_cuda() && fl.numel() == f.size(0) && gl.numel() == f.size(0),
              "transducer_joint: f_len / g_len must be GPU tensors of length B");
  const int64_t B = f.size(0), T = f.size(1), U = g.size(1), H = f.size(2);
  at::Tensor bo;
  at::Tensor out;
  int64_t rows;
  if (pack_output) {
    bo = batch_offset.to(at::kLong).contiguous();
    TORCH_CHECK(bo.is_cuda() && bo.numel() == B, "transducer_joint: batch_offset must be a GPU tensor of length B");
    rows = packed_batch;
    out = at::empty({packed_batch, H}, f.options());
  } else {
    rows = B * T * U;
    out = at::empty({B, T, U, H}, f.options());
  }
  at::Tensor mask;
  if (want_mask) mask = at::zeros(out.sizes(), f.options().dtype(at::kByte));
  auto a = joint_args(B, T, U, H, fl, gl, bo, pack_output, rows, relu, dropout, dropout_prob, seed);
  bh::transducer_joint_forward(a, dtype_code(f.scalar_type()), f.data_ptr(), g.data_ptr(), out.data_ptr(),
                               want_mask ? mask.data_ptr<uint8_t>() : nullptr, stream_for(f));
  return {out, mask};
}

std::vector<at::Tensor> td_joint_bwd(at::Tensor grad, at::Tensor out, at::Tensor f_len, at::Tensor g_len,
                                     at::Tensor batch_offset, int64_t T, int64_t U, bool pack_output, bool relu,
                                     bool dropout, double dropout_prob, int64_t seed) {
  check_cuda(grad, "grad");
  grad = grad.contiguous();
  auto fl = f_len.to(at::kInt).contiguous();
  auto gl = g_len.to(at::kInt).contiguous();
  const int64_t B = fl.numel();
  const int64_t H = grad.size(-1);
  TORCH_CHECK(H % 8 == 0, "transducer_joint: hidden size must be a multiple of 8");
  at::Tensor bo;
  if (pack_output) bo = batch_offset.to(at::kLong).contiguous();
  const int64_t rows = grad.numel() / H;
  TORCH_CHECK(pack_output || rows == B * T * U, "transducer_joint backward: grad must be [B, T, U, H]");
  if (relu) {
    TORCH_CHECK(out.defined() && out.sizes() == grad.sizes(), "transducer_joint backward: relu needs the output");
    out = out.contiguous();
  }
  auto df = at::empty({B, T, H}, grad.options());
  auto dg = at::empty({B, U, H}, grad.options());
  auto a = joint_args(B, T, U, H, fl, gl, bo, pack_output, rows, relu, dropout, dropout_prob, seed);
  bh::transducer_joint_backward(a, dtype_code(grad.scalar_type()), grad.data_ptr(), relu ? out.data_ptr() : nullptr,
                                df.data_ptr(), dg.data_ptr(), stream_for(grad));
  return {df, dg};
}

void check_perm_matrix(const at::Tensor& m) {
  check_cuda(m, "matrix");
  TORCH_CHECK(m.dim() == 2 && m.scalar_type() == at::kFloat && m.is_contiguous(),
              "permutation search: matrix must be a contiguous 2-D fp32 tensor");
  TORCH_CHECK(m.size(1) % 4 == 0, "permutation search: column count must be a multiple of 4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(m.data_ptr()) % 16 == 0, "permutation search: matrix must be 16B aligned");
}

at::Tensor perm_sum24(at::Tensor m) {
  check_perm_matrix(m);
  const int parts = bh::perm_sum_parts(m.size(0), m.size(1));
  auto part = at::empty({parts}, m.options());
  auto out = at::empty({}, m.options());
  bh::perm_sum_after_2to4(m.data_ptr<float>(), m.size(0), m.size(1), part.data_ptr<float>(), out.data_ptr<float>(),
                          stream_for(m));
  return out;
}

std::vector<at::Tensor> perm_pair_gains(at::Tensor m, at::Tensor pairs) {
  check_perm_matrix(m);
  TORCH_CHECK(pairs.is_cuda() && pairs.scalar_type() == at::kInt && pairs.dim() == 2 && pairs.size(1) == 2 &&
                  pairs.is_contiguous(), "permutation search: pairs must be a contiguous int32 [P, 2] GPU tensor");
  const int64_t stripes = m.size(1) / 4;
  if (pairs.numel() > 0) {
    TORCH_CHECK(pairs.min().item<int>() >= 0 && pairs.max().item<int>() < stripes,
                "permutation search: stripe index out of range");
  }
  const int64_t P = pairs.size(0);
  auto gain = at::empty({P}, m.options());
  auto split = at::empty({P}, pairs.options());
  bh::perm_stripe_pair_gains(m.data_ptr<float>(), m.size(0), m.size(1), pairs.data_ptr<int32_t>(), P,
                             gain.data_ptr<float>(), split.data_ptr<int32_t>(), stream_for(m));
  return {gain, split};
}


// ---- fused attention (kernels/attn.hip). q/k/v/outputs are [time, batch*heads, 64] views with a
// contiguous last dim (arbitrary time / batch*heads strides).
void attn_check(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.dim() == 3 && t.size(2) == 64 && t.stride(2) == 1, name, ": expected a [t, bh, 64] view with stride(2)==1");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, ": strides must be multiples of 8 elements and the base 16-byte aligned");
}

bh::AttnArgs attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int mask_mode,
                       const c10::optional<at::Tensor>& mask, int64_t heads, double scale, double p, bool training,
                       int64_t seed, at::Tensor& mask_keep, bool flash = false) {
  attn_check(q, "q");
  attn_check(k, "k");
  attn_check(v, "v");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "attn: dtype mismatch");
  TORCH_CHECK(k.size(0) == v.size(0) && q.size(1) == k.size(1) && q.size(1) == v.size(1), "attn: shape mismatch");
  TORCH_CHECK(flash || k.size(0) <= bh::attn_max_sk(), "attn: sk > ", bh::attn_max_sk());
  TORCH_CHECK(flash || (mask_mode >= 0 && mask_mode <= 3), "attn: short kernels take mask modes 0-3");
  bh::AttnArgs a;
  a.q = q.data_ptr(); a.k = k.data_ptr(); a.v = v.data_ptr();
  a.q_st = q.stride(0); a.q_sbh = q.stride(1);
  a.k_st = k.stride(0); a.k_sbh = k.stride(1);
  a.v_st = v.stride(0); a.v_sbh = v.stride(1);
  a.sq = (int)q.size(0); a.sk = (int)k.size(0); a.BH = (int)q.size(1); a.heads = (int)heads;
  a.mask_mode = mask_mode;
  if (mask_mode != 0) {
    TORCH_CHECK(mask_mode == 5 || (mask.has_value() && mask->defined()), "attn: mask_mode needs a mask");
  }
  if (mask_mode != 0 && mask_mode != 5) {
    if (mask_mode == 2) mask_keep = mask->to(at::kFloat).contiguous();
    else mask_keep = mask->to(at::kByte).contiguous();
    const int64_t B = a.BH / a.heads;
    const int64_t want = mask_mode == 3 ? (int64_t)a.sq * a.sk : mask_mode == 4 ? B * a.sq * a.sk : B * a.sk;
    TORCH_CHECK(mask_keep.numel() == want, "attn: mask has ", mask_keep.numel(), " elements, expected ", want);
    a.mask = mask_keep.data_ptr();
  }
  a.scale = (float)scale;
  a.p_drop = (float)p;
  a.training = training;
  a.seed = (uint64_t)seed;
  return a;
}

at::Tensor attn_fwd(at::Tensor q, at::Tensor k, at::Tensor v, int mask_mode, c10::optional<at::Tensor> mask,
                    int64_t heads, double scale, double p, bool training, int64_t seed) {
  at::Tensor mk;
  auto a = attn_args(q, k, v, mask_mode, mask, heads, scale, p, training, seed, mk);
  auto o = at::empty({q.size(0), q.size(1), 64}, q.options());
  a.o = o.data_ptr();
  a.o_st = o.stride(0);
  a.o_sbh = o.stride(1);
  bh::attn_forward(dtype_code(q.scalar_type()), a, stream_for(q));
  return o;
}

void attn_bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, int mask_mode,
              c10::optional<at::Tensor> mask, int64_t heads, double scale, double p, bool training, int64_t seed,
              at::Tensor dq, at::Tensor dk, at::Tensor dv) {
  at::Tensor mk;
  auto a = attn_args(q, k, v, mask_mode, mask, heads, scale, p, training, seed, mk);
  attn_check(dout, "dout");
  attn_check(dq, "dq");
  attn_check(dk, "dk");
  attn_check(dv, "dv");
  a.dout = dout.data_ptr(); a.do_st = dout.stride(0); a.do_sbh = dout.stride(1);
  a.dq = dq.data_ptr(); a.dq_st = dq.stride(0); a.dq_sbh = dq.stride(1);
  a.dk = dk.data_ptr(); a.dk_st = dk.stride(0); a.dk_sbh = dk.stride(1);
  a.dv = dv.data_ptr(); a.dv_st = dv.stride(0); a.dv_sbh = dv.stride(1);
  bh::attn_backward(dtype_code(q.scalar_type()), a, stream_for(q));
}

void register_contrib_impl(pybind11::module_& root);

// mode 4 on the 32x32 flash kernels: the uint8 mask packed to bits, [bits | bits_t] in one int32
// tensor (AttnArgs::mbits / mbits_t). ``pre`` = the packing done once by flash_mask_bits (a BERT
// forward shares one mask over all layers); otherwise packed here. (The 16-wide kernels reading the
// mask bytes lost: profiles/bert_flash_mode4_wide_ab.txt.)
void attach_mask_bits(bh::AttnArgs& a, const at::Tensor& q, const c10::optional<at::Tensor>& pre, at::Tensor& mb) {
  if (a.mask_mode != 4) return;
  const int64_t B = a.BH / a.heads;
  const int64_t nb = B * a.sq * ((a.sk + 31) / 32), nbt = B * a.sk * ((a.sq + 31) / 32);
  if (pre.has_value() && pre->defined()) {
    check_cuda(*pre, "mask bits");
    TORCH_CHECK(pre->scalar_type() == at::kInt && pre->is_contiguous() && pre->numel() == nb + nbt,
                "flash: mask bits must be the int32 [", nb + nbt, "] tensor of flash_mask_bits for this shape");
    mb = *pre;
  } else {
    mb = at::empty({nb + nbt}, q.options().dtype(at::kInt));
    auto* w = reinterpret_cast<uint32_t*>(mb.data_ptr());
    bh::flash_mask_bits(a, w, w + nb, stream_for(q));
  }
  a.mbits = reinterpret_cast<const uint32_t*>(mb.data_ptr());
  a.mbits_t = a.mbits + nb;
}

// mask [B, sq, sk] (bool / uint8) -> the packed bits for flash_forward / flash_backward (mode 4)
at::Tensor flash_mask_bits_op(at::Tensor mask) {
  check_cuda(mask, "mask");
  TORCH_CHECK(mask.dim() == 3, "flash_mask_bits: mask must be [B, sq, sk]");
  auto m = mask.to(at::kByte).contiguous();
  bh::AttnArgs a;
  a.mask_mode = 4;
  a.mask = m.data_ptr();
  a.heads = 1;
  a.BH = (int)m.size(0);
  a.sq = (int)m.size(1);
  a.sk = (int)m.size(2);
  const int64_t nb = (int64_t)a.BH * a.sq * ((a.sk + 31) / 32), nbt = (int64_t)a.BH * a.sk * ((a.sq + 31) / 32);
  auto mb = at::empty({nb + nbt}, m.options().dtype(at::kInt));
  auto* w = reinterpret_cast<uint32_t*>(mb.data_ptr());
  bh::flash_mask_bits(a, w, w + nb, stream_for(m));
  return mb;
}

// seed_dev: an int64 [1] device tensor (utils/graph_rng.py) that keys the dropout with the step seed
void attach_seed_dev(bh::AttnArgs& a, const at::Tensor& q, const c10::optional<at::Tensor>& seed_dev) {
  if (!seed_dev.has_value() || !seed_dev->defined()) return;
  TORCH_CHECK(seed_dev->scalar_type() == at::kLong && seed_dev->numel() == 1 && seed_dev->device() == q.device(),
              "flash attention: seed_dev must be an int64 [1] tensor on q's device");
  a.seed_dev = seed_dev->data_ptr<int64_t>();
}

std::vector<at::Tensor> flash_fwd(at::Tensor q, at::Tensor k, at::Tensor v, int mask_mode,
                                  c10::optional<at::Tensor> mask, int64_t heads, double scale, double p, bool training,
                                  int64_t seed, double mask_fill, c10::optional<at::Tensor> bits,
                                  c10::optional<at::Tensor> seed_dev) {
  at::Tensor mk;
  auto a = attn_args(q, k, v, mask_mode, mask, heads, scale, p, training, seed, mk, /*flash=*/true);
  attach_seed_dev(a, q, seed_dev);
  a.mask_fill = (float)mask_fill;
  at::Tensor mb;
  attach_mask_bits(a, q, bits, mb);
  auto o = at::empty({q.size(0), q.size(1), 64}, q.options());
  auto lse = at::empty({q.size(1), q.size(0)}, q.options().dtype(at::kFloat));
  a.o = o.data_ptr(); a.o_st = o.stride(0); a.o_sbh = o.stride(1);
  a.lse = lse.data_ptr<float>();
  bh::flash_forward(dtype_code(q.scalar_type()), a, stream_for(q));
  return {o, lse};
}

void flash_bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse, int mask_mode,
               c10::optional<at::Tensor> mask, int64_t heads, double scale, double p, bool training, int64_t seed,
               double mask_fill, at::Tensor dq, at::Tensor dk, at::Tensor dv, c10::optional<at::Tensor> bits,
               c10::optional<at::Tensor> seed_dev) {
  at::Tensor mk;
  auto a = attn_args(q, k, v, mask_mode, mask, heads, scale, p, training, seed, mk, /*flash=*/true);
  attach_seed_dev(a, q, seed_dev);
  a.mask_fill = (float)mask_fill;
  at::Tensor mb;
  attach_mask_bits(a, q, bits, mb);
  attn_check(dout, "dout");
  attn_check(o, "o");
  attn_check(dq, "dq");
  attn_check(dk, "dk");
  attn_check(dv, "dv");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)a.BH * a.sq, "flash_bwd: lse must be [BH, sq]");
  a.o = o.data_ptr(); a.o_st = o.stride(0); a.o_sbh = o.stride(1);
  a.dout = dout.data_ptr(); a.do_st = dout.stride(0); a.do_sbh = dout.stride(1);
  a.dq = dq.data_ptr(); a.dq_st = dq.stride(0); a.dq_sbh = dq.stride(1);
  a.dk = dk.data_ptr(); a.dk_st = dk.stride(0); a.dk_sbh = dk.stride(1);
  a.dv = dv.data_ptr(); a.dv_st = dv.stride(0); a.dv_sbh = dv.stride(1);
  auto delta = at::empty_like(lse);
  a.lse = lse.data_ptr<float>();
  const int dt = dtype_code(q.scalar_type());
  bh::flash_delta(dt, a, delta.data_ptr<float>(), stream_for(q));
  a.delta = delta.data_ptr<float>();
  bh::flash_backward(dt, a, stream_for(q));
}

// varlen: q / k / v / o / dout / dq / dk / dv are packed [total_tokens, heads, 64] views (e.g. the
// slices of one [total, 3, heads, 64] qkv tensor), cu_seqlens int32 [B + 1] on the device. max_s
// (the caller's bound on the lengths, as in fmhalib) sizes the grid; nothing is read back.
bh::AttnArgs varlen_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& cu,
                         int64_t max_s, bool causal, double scale, double p, bool training, int64_t seed) {
  attn_check(q, "q");
  attn_check(k, "k");
  attn_check(v, "v");
  check_cuda(cu, "cu_seqlens");
  TORCH_CHECK(cu.scalar_type() == at::kInt && cu.dim() == 1 && cu.numel() >= 2 && cu.is_contiguous(),
              "flash varlen: cu_seqlens must be a contiguous int32 [B + 1] tensor");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "flash varlen: dtype mismatch");
  TORCH_CHECK(q.sizes() == k.sizes() && q.sizes() == v.sizes(), "flash varlen: q / k / v shape mismatch");
  TORCH_CHECK(max_s >= 1, "flash varlen: max_s must be >= 1");
  bh::AttnArgs a;
  a.q = q.data_ptr(); a.k = k.data_ptr(); a.v = v.data_ptr();
  a.q_st = q.stride(0); a.q_sbh = q.stride(1);
  a.k_st = k.stride(0); a.k_sbh = k.stride(1);
  a.v_st = v.stride(0); a.v_sbh = v.stride(1);
  a.heads = (int)q.size(1);
  a.BH = (int)((cu.numel() - 1) * q.size(1));
  a.sq = a.sk = (int)max_s;
  a.cu_seqlens = cu.data_ptr<int>();
  a.mask_mode = causal ? 5 : 0;
  a.scale = (float)scale;
  a.p_drop = (float)p;
  a.training = training;
  a.seed = (uint64_t)seed;
  return a;
}

std::vector<at::Tensor> flash_varlen_fwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor cu, int64_t max_s,
                                         bool causal, double scale, double p, bool training, int64_t seed) {
  auto a = varlen_args(q, k, v, cu, max_s, causal, scale, p, training, seed);
  auto o = at::empty({q.size(0), q.size(1), 64}, q.options());
  auto lse = at::empty({(int64_t)a.BH, max_s}, q.options().dtype(at::kFloat));
  a.o = o.data_ptr(); a.o_st = o.stride(0); a.o_sbh = o.stride(1);
  a.lse = lse.data_ptr<float>();
  if (q.size(0) > 0) bh::flash_forward(dtype_code(q.scalar_type()), a, stream_for(q));
  return {o, lse};
}

void flash_varlen_bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                      at::Tensor cu, int64_t max_s, bool causal, double scale, double p, bool training, int64_t seed,
                      at::Tensor dq, at::Tensor dk, at::Tensor dv) {
  auto a = varlen_args(q, k, v, cu, max_s, causal, scale, p, training, seed);
  attn_check(dout, "dout");
  attn_check(o, "o");
  attn_check(dq, "dq");
  attn_check(dk, "dk");
  attn_check(dv, "dv");
  for (const auto* t : {&dout, &o, &dq, &dk, &dv})
    TORCH_CHECK(t->sizes() == q.sizes(), "flash varlen backward: gradient / output shape mismatch");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)a.BH * max_s, "flash varlen backward: lse must be [BH, max_s]");
  if (q.size(0) == 0) return;
  a.o = o.data_ptr(); a.o_st = o.stride(0); a.o_sbh = o.stride(1);
  a.dout = dout.data_ptr(); a.do_st = dout.stride(0); a.do_sbh = dout.stride(1);
  a.dq = dq.data_ptr(); a.dq_st = dq.stride(0); a.dq_sbh = dq.stride(1);
  a.dk = dk.data_ptr(); a.dk_st = dk.stride(0); a.dk_sbh = dk.stride(1);
  a.dv = dv.data_ptr(); a.dv_st = dv.stride(0); a.dv_sbh = dv.stride(1);
  auto delta = at::empty_like(lse);
  a.lse = lse.data_ptr<float>();
  const int dt = dtype_code(q.scalar_type());
  bh::flash_delta(dt, a, delta.data_ptr<float>(), stream_for(q));
  a.delta = delta.data_ptr<float>();
  bh::flash_backward(dt, a, stream_for(q));
}

}  // namespace

void register_contrib(pybind11::module_& root) {
  register_contrib_impl(root);
  auto fa = root.def_submodule("fused_attention", "MFMA fused short-sequence attention (head_dim 64, sk <= 128)");
  fa.def("forward", &attn_fwd);
  fa.def("backward", &attn_bwd);
  fa.def("max_sk", &bh::attn_max_sk);
  namespace py = pybind11;
  fa.def("flash_forward", &flash_fwd, "any-length attention forward -> (o, lse)", py::arg("q"), py::arg("k"),
         py::arg("v"), py::arg("mask_mode"), py::arg("mask"), py::arg("heads"), py::arg("scale"), py::arg("p"),
         py::arg("training"), py::arg("seed"), py::arg("mask_fill"), py::arg("bits") = py::none(),
         py::arg("seed_dev") = py::none());
  fa.def("flash_backward", &flash_bwd, "any-length attention backward into dq / dk / dv", py::arg("dout"),
         py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("lse"), py::arg("mask_mode"),
         py::arg("mask"), py::arg("heads"), py::arg("scale"), py::arg("p"), py::arg("training"), py::arg("seed"),
         py::arg("mask_fill"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("bits") = py::none(),
         py::arg("seed_dev") = py::none());
  fa.def("flash_varlen_forward", &flash_varlen_fwd, "packed variable-length attention forward -> (o, lse)",
         py::arg("q"), py::arg("k"), py::arg("v"), py::arg("cu_seqlens"), py::arg("max_s"), py::arg("causal"),
         py::arg("scale"), py::arg("p"), py::arg("training"), py::arg("seed"));
  fa.def("flash_varlen_backward", &flash_varlen_bwd, "packed variable-length attention backward into dq / dk / dv",
         py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("lse"),
         py::arg("cu_seqlens"), py::arg("max_s"), py::arg("causal"), py::arg("scale"), py::arg("p"),
         py::arg("training"), py::arg("seed"), py::arg("dq"), py::arg("dk"), py::arg("dv"));
  fa.def("flash_mask_bits", &flash_mask_bits_op, "mode-4 mask [B, sq, sk] -> packed bits for the flash kernels");
}

namespace {
void register_contrib_impl(pybind11::module_& root) {
  auto fl = root.def_submodule("focal_loss_cuda", "sigmoid focal loss");
  fl.def("forward", &focal_fwd);
  fl.def("backward", &focal_bwd);
  auto mha = root.def_submodule("fast_multihead_attn", "MHA mask + softmax + dropout block");
  mha.def("mask_softmax_dropout_forward", &mha_softmax_fwd);
  mha.def("mask_softmax_dropout_backward", &mha_softmax_bwd);
  mha.def("max_sk", &bh::mha_max_sk);
  auto tl = root.def_submodule("transducer_loss_cuda", "RNN-T loss");
  tl.def("forward", &td_loss_fwd);
  tl.def("backward", &td_loss_bwd);
  auto tj = root.def_submodule("transducer_joint_cuda", "RNN-T joint: broadcast add + pack + ReLU + dropout");
  tj.def("forward", &td_joint_fwd);
  tj.def("backward", &td_joint_bwd);
  auto ps = root.def_submodule("permutation_search_cuda", "2:4 sparsity channel-permutation search");
  ps.def("sum_after_2_to_4", &perm_sum24, "kept |w| after 2:4 pruning along rows of a [R, C] fp32 matrix");
  ps.def("stripe_pair_gains", &perm_pair_gains, "best re-split gain and split index per stripe pair");
  auto im = root.def_submodule("fused_index_mul_2d", "out = in1[idx] * in2");
  for (const char* p : {"float_", "half_", "bfloat16_", ""}) {
    im.def((std::string(p) + "forward").c_str(), &imul_fwd);
    im.def((std::string(p) + "backward").c_str(), &imul_bwd);
    im.def((std::string(p) + "backward_backward").c_str(), &imul_bwd_bwd);
  }
}

}  // namespace

}  // namespace bhb
