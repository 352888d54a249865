// `syncbn` front-end: fused BN statistics / normalisation / backward for SyncBatchNorm.
// Kernels: kernels/batchnorm.hip. Reference API: csrc/syncbn.cpp:98-109 (compat wrappers for those
// names live in python: beforeholiday_amd/ops/syncbn.py).
#include "common.h"
#include "bh/pool_api.h"

#include "bh/bn_api.h"

namespace bhb {
namespace {

struct Layout {
  bh::BNShape s;
  at::Tensor x;  // possibly re-laid-out input
};

bool aligned16(const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

Layout layout_of(const at::Tensor& x_in) {
  TORCH_CHECK(x_in.dim() >= 2, "batchnorm expects at least 2 dims (N, C, ...)");
  Layout L;
  at::Tensor x = x_in;
  const int64_t N = x.size(0);
  const int64_t C = x.size(1);
  int64_t inner = 1;
  for (int d = 2; d < x.dim(); ++d) inner *= x.size(d);
  bool cl = false;
  if (inner == 1) {
    if (!x.is_contiguous()) x = x.contiguous();
    cl = (C % 8 == 0) && aligned16(x);
  } else if (x.is_contiguous()) {
    cl = false;
  } else if ((x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)) ||
             (x.dim() == 5 && x.is_contiguous(at::MemoryFormat::ChannelsLast3d))) {
    cl = (C % 8 == 0) && aligned16(x);
    if (!cl) x = x.contiguous();
  } else {
    x = x.contiguous();
  }
  if (!cl && !aligned16(x)) x = x.clone();
  L.x = x;
  L.s.C = (int)C;
  L.s.channels_last = cl;
  if (cl) {
    L.s.outer = N * inner;
    L.s.inner = 1;
  } else {
    L.s.outer = N;
    L.s.inner = inner;
  }
  return L;
}

// bring `t` into exactly the layout of the (re-laid-out) reference input
at::Tensor like(const at::Tensor& t, const at::Tensor& ref) {
  if (t.strides() == ref.strides() && aligned16(t)) return t;
  at::Tensor o = at::empty_like(ref, t.options());
  o.copy_(t);
  return o;
}

int wcode(const c10::optional<at::Tensor>& w) { return (w.has_value() && w->defined()) ? dtype_code(w->scalar_type()) : bh::kF32; }
const void* wptr(const c10::optional<at::Tensor>& w) { return (w.has_value() && w->defined()) ? w->data_ptr() : nullptr; }
void* wptr_mut(const c10::optional<at::Tensor>& w) { return (w.has_value() && w->defined()) ? w->data_ptr() : nullptr; }

at::TensorOptions fopt(const at::Tensor& x) { return x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous); }

// local stats -> [mean(C), var_biased(C), count(1)] (the all_gather payload)
at::Tensor stats_local(at::Tensor x_in) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  const int C = L.s.C;
  const int splits = bh::bn_num_splits(L.s);
  auto part = at::empty({3 * (int64_t)splits * C + splits}, fopt(L.x));
  float* pm = part.data_ptr<float>();
  float* pm2 = pm + (int64_t)splits * C;
  float* pn = pm2 + (int64_t)splits * C;
  auto out = at::empty({2 * (int64_t)C + 1}, fopt(L.x));
  hipStream_t st = stream_for(L.x);
  bh::bn_stats(L.s, dtype_code(L.x.scalar_type()), L.x.data_ptr(), splits, pm, pm2, pn, st);
  bh::BNFinal fin{};
  bh::bn_stats_finalize(L.s, splits, pm, pm2, pn, out.data_ptr<float>(), fin, bh::kF32, nullptr, nullptr, nullptr,
                        nullptr, st);
  return out;
}

// local shifted sums -> [sum(x-K) (C), sum((x-K)^2) (C), count (1)] (the all_reduce SUM payload);
// K = running_mean (shared by every rank), or 0 when stats are not tracked
at::Tensor stats_local_sums(at::Tensor x_in, c10::optional<at::Tensor> running_mean) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  const int C = L.s.C;
  const int splits = bh::bn_num_splits(L.s);
  const int64_t nslots = L.s.channels_last ? splits : (int64_t)splits * C;
  auto part = at::empty({2 * (int64_t)splits * C + nslots}, fopt(L.x));
  float* pm = part.data_ptr<float>();
  float* pm2 = pm + (int64_t)splits * C;
  float* pn = pm2 + (int64_t)splits * C;
  auto out = at::empty({2 * (int64_t)C + 1}, fopt(L.x));
  hipStream_t st = stream_for(L.x);
  bh::bn_stats(L.s, dtype_code(L.x.scalar_type()), L.x.data_ptr(), splits, pm, pm2, pn, st);
  const bool has_k = running_mean.has_value() && running_mean->defined();
  if (has_k) TORCH_CHECK(running_mean->is_contiguous() && running_mean->numel() == C, "running_mean must be [C]");
  bh::BNFinal fin{};
  bh::bn_stats_finalize(L.s, splits, pm, pm2, pn, nullptr, fin, has_k ? dtype_code(running_mean->scalar_type()) : bh::kF32,
                        nullptr, nullptr, nullptr, nullptr, st, has_k ? running_mean->data_ptr() : nullptr,
                        out.data_ptr<float>());
  return out;
}

// returns (mean, invstd, scale, shift, count)
std::vector<at::Tensor> final_outputs(const at::Tensor& ref, int64_t C) {
  auto o = fopt(ref);
  return {at::empty({C}, o), at::empty({C}, o), at::empty({C}, o), at::empty({C}, o), at::empty({1}, o)};
}
int64_t* counter_ptr(const c10::optional<at::Tensor>& t) {
  if (!(t.has_value() && t->defined())) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->numel() == 1,
              "num_batches_tracked must be a GPU int64 scalar tensor");
  return t->data_ptr<int64_t>();
}

bh::BNFinal fin_of(std::vector<at::Tensor>& r, double eps, double momentum) {
  bh::BNFinal f{};
  f.mean = r[0].data_ptr<float>();
  f.invstd = r[1].data_ptr<float>();
  f.scale = r[2].data_ptr<float>();
  f.shift = r[3].data_ptr<float>();
  f.count = r[4].data_ptr<float>();
  f.eps = (float)eps;
  f.momentum = (float)momentum;
  return f;
}

void check_running(const c10::optional<at::Tensor>& rm, const c10::optional<at::Tensor>& rv,
                   const c10::optional<at::Tensor>& w) {
  if (rm.has_value() && rm->defined()) {
    TORCH_CHECK(rv.has_value() && rv->defined(), "running_var required with running_mean");
    TORCH_CHECK(rm->is_contiguous() && rv->is_contiguous(), "running stats must be contiguous");
    if (w.has_value() && w->defined())
      TORCH_CHECK(rm->scalar_type() == w->scalar_type() && rv->scalar_type() == w->scalar_type(),
                  "running stats must share the weight dtype");
  }
}

// single-rank fused statistics (no all_gather needed)
std::vector<at::Tensor> stats_single(at::Tensor x_in, c10::optional<at::Tensor> w, c10::optional<at::Tensor> b,
                                     c10::optional<at::Tensor> rmean, c10::optional<at::Tensor> rvar,
                                     double momentum, double eps, c10::optional<at::Tensor> num_batches) {
  check_cuda(x_in, "input");
  check_running(rmean, rvar, w);
  Layout L = layout_of(x_in);
  const int C = L.s.C;
  const int splits = bh::bn_num_splits(L.s);
  const int64_t nslots = L.s.channels_last ? splits : (int64_t)splits * C;
  auto part = at::empty({2 * (int64_t)splits * C + nslots}, fopt(L.x));
  float* pm = part.data_ptr<float>();
  float* pm2 = pm + (int64_t)splits * C;
  float* pn = pm2 + (int64_t)splits * C;
  auto r = final_outputs(L.x, C);
  auto fin = fin_of(r, eps, momentum);
  fin.num_batches = counter_ptr(num_batches);
  hipStream_t st = stream_for(L.x);
  bh::bn_stats(L.s, dtype_code(L.x.scalar_type()), L.x.data_ptr(), splits, pm, pm2, pn, st);
  const bool has_run = rmean.has_value() && rmean->defined();
  int dtw = wcode(w);
  if (!(w.has_value() && w->defined()) && has_run) dtw = dtype_code(rmean->scalar_type());
  bh::bn_stats_finalize(L.s, splits, pm, pm2, pn, nullptr, fin, dtw, wptr(w), wptr(b),
                        has_run ? rmean->data_ptr() : nullptr, has_run ? rvar->data_ptr() : nullptr, st);
  return r;
}

// merge gathered [W, 2C+1] rows (+ running stats update)
std::vector<at::Tensor> merge_ranks(at::Tensor gathered, c10::optional<at::Tensor> w, c10::optional<at::Tensor> b,
                                    c10::optional<at::Tensor> rmean, c10::optional<at::Tensor> rvar, double momentum,
                                    double eps, c10::optional<at::Tensor> num_batches) {
  check_cuda(gathered, "gathered");
  TORCH_CHECK(gathered.dim() == 2 && gathered.scalar_type() == at::kFloat, "gathered must be [W, 2C+1] fp32");
  gathered = gathered.contiguous();
  check_running(rmean, rvar, w);
  const int W = (int)gathered.size(0);
  const int C = (int)((gathered.size(1) - 1) / 2);
  auto r = final_outputs(gathered, C);
  auto fin = fin_of(r, eps, momentum);
  fin.num_batches = counter_ptr(num_batches);
  const bool has_run = rmean.has_value() && rmean->defined();
  int dtw = wcode(w);
  if (!(w.has_value() && w->defined()) && has_run) dtw = dtype_code(rmean->scalar_type());
  bh::bn_merge_ranks(W, C, gathered.data_ptr<float>(), fin, dtw, wptr(w), wptr(b),
                     has_run ? rmean->data_ptr() : nullptr, has_run ? rvar->data_ptr() : nullptr, nullptr,
                     stream_for(gathered));
  return r;
}

// finalize all-reduced shifted sums [2C+1] (+ running stats update, scale/shift)
std::vector<at::Tensor> merge_sums(at::Tensor sums, c10::optional<at::Tensor> w, c10::optional<at::Tensor> b,
                                   c10::optional<at::Tensor> rmean, c10::optional<at::Tensor> rvar, double momentum,
                                   double eps, c10::optional<at::Tensor> num_batches) {
  check_cuda(sums, "sums");
  TORCH_CHECK(sums.dim() == 1 && sums.scalar_type() == at::kFloat && sums.numel() % 2 == 1, "sums must be fp32 [2C+1]");
  sums = sums.contiguous();
  check_running(rmean, rvar, w);
  const int C = (int)((sums.numel() - 1) / 2);
  auto r = final_outputs(sums, C);
  auto fin = fin_of(r, eps, momentum);
  fin.num_batches = counter_ptr(num_batches);
  const bool has_run = rmean.has_value() && rmean->defined();
  int dtw = wcode(w);
  if (!(w.has_value() && w->defined()) && has_run) dtw = dtype_code(rmean->scalar_type());
  bh::bn_merge_sums(C, sums.data_ptr<float>(), fin, dtw, wptr(w), wptr(b), has_run ? rmean->data_ptr() : nullptr,
                    has_run ? rvar->data_ptr() : nullptr, stream_for(sums));
  return r;
}

// single rank: finalize straight from conv-epilogue partials [2, G, C] (no [2C+1] sums tensor)
std::vector<at::Tensor> merge_parts(at::Tensor part, double count, c10::optional<at::Tensor> w,
                                    c10::optional<at::Tensor> b, c10::optional<at::Tensor> rmean,
                                    c10::optional<at::Tensor> rvar, double momentum, double eps,
                                    c10::optional<at::Tensor> num_batches, bool bump) {
  check_cuda(part, "part");
  TORCH_CHECK(!bump || momentum >= 0, "merge_parts: bump (num_batches += 1) needs a fixed momentum");
  TORCH_CHECK(part.dim() == 3 && part.size(0) == 2 && part.scalar_type() == at::kFloat && part.is_contiguous(),
              "part must be a contiguous fp32 [2, G, C] tensor");
  check_running(rmean, rvar, w);
  const int G = (int)part.size(1), C = (int)part.size(2);
  auto r = final_outputs(part, C);
  auto fin = fin_of(r, eps, momentum);
  fin.num_batches = counter_ptr(num_batches);
  const bool has_run = rmean.has_value() && rmean->defined();
  int dtw = wcode(w);
  if (!(w.has_value() && w->defined()) && has_run) dtw = dtype_code(rmean->scalar_type());
  const int SG = bh::bn_part_segments(G);
  at::Tensor seg_ws = SG > 1 ? at::empty({SG, 2, C}, part.options()) : at::Tensor();
  bh::bn_merge_parts(G, C, part.data_ptr<float>(), (float)count, fin, dtw, wptr(w), wptr(b),
                     has_run ? rmean->data_ptr() : nullptr, has_run ? rvar->data_ptr() : nullptr, stream_for(part),
                     bump, SG > 1 ? seg_ws.data_ptr<float>() : nullptr);
  return r;
}

at::Tensor forward(at::Tensor x_in, c10::optional<at::Tensor> z, at::Tensor scale, at::Tensor shift, bool relu,
                   c10::optional<at::ScalarType> out_dtype, c10::optional<at::Tensor> num_batches) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  at::Tensor zt;
  if (z.has_value() && z->defined()) zt = like(*z, L.x);
  auto y = at::empty_like(L.x, L.x.options().dtype(out_dtype.value_or(L.x.scalar_type())));
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == L.s.C,
              "scale/shift must be fp32 [C]");
  bh::bn_forward(L.s, dtype_code(L.x.scalar_type()), L.x.data_ptr(), zt.defined() ? dtype_code(zt.scalar_type()) : -1,
                 zt.defined() ? zt.data_ptr() : nullptr, dtype_code(y.scalar_type()), y.data_ptr(),
                 scale.contiguous().data_ptr<float>(), shift.contiguous().data_ptr<float>(), relu,
                 counter_ptr(num_batches), stream_for(L.x));
  return y;
}

// true when the 1-bit ReLU mask path applies (NHWC rows x C with C % 8 == 0)
bool mask_ok(const at::Tensor& x) {
  if (!x.is_cuda()) return false;
  Layout L = layout_of(x);
  return L.s.channels_last && L.s.C % 8 == 0;
}

// forward that also returns the ReLU mask as uint8 [rows, C/8] (bit k: channel 8j+k > 0), so the
// backward of BN + add + ReLU does not keep reading the residual input z
std::vector<at::Tensor> forward_mask(at::Tensor x_in, c10::optional<at::Tensor> z, at::Tensor scale, at::Tensor shift,
                                     c10::optional<at::Tensor> num_batches, c10::optional<at::Tensor> zscale,
                                     c10::optional<at::Tensor> zshift) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  TORCH_CHECK(L.s.channels_last && L.s.C % 8 == 0, "forward_mask: needs channels_last with C % 8 == 0");
  at::Tensor zt;
  if (z.has_value() && z->defined()) zt = like(*z, L.x);
  auto y = at::empty_like(L.x);
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == L.s.C,
              "scale/shift must be fp32 [C]");
  auto mask = at::empty({L.s.outer, (int64_t)(L.s.C / 8)}, L.x.options().dtype(at::kByte).memory_format(at::MemoryFormat::Contiguous));
  at::Tensor zs, zh;
  if (zscale.has_value() && zscale->defined()) {
    TORCH_CHECK(zt.defined() && zshift.has_value() && zshift->defined(), "forward_mask: zscale needs z and zshift");
    zs = zscale->contiguous();
    zh = zshift->contiguous();
    TORCH_CHECK(zs.scalar_type() == at::kFloat && zh.scalar_type() == at::kFloat && zs.numel() == L.s.C &&
                    zh.numel() == L.s.C,
                "forward_mask: zscale / zshift must be fp32 [C]");
  }
  bh::bn_forward(L.s, dtype_code(L.x.scalar_type()), L.x.data_ptr(), zt.defined() ? dtype_code(zt.scalar_type()) : -1,
                 zt.defined() ? zt.data_ptr() : nullptr, dtype_code(y.scalar_type()), y.data_ptr(),
                 scale.contiguous().data_ptr<float>(), shift.contiguous().data_ptr<float>(), true,
                 counter_ptr(num_batches), stream_for(L.x), mask.data_ptr<uint8_t>(),
                 zs.defined() ? zs.data_ptr<float>() : nullptr, zs.defined() ? zh.data_ptr<float>() : nullptr);
  return {y, mask};
}

const uint8_t* mask_ptr(const c10::optional<at::Tensor>& mask, const Layout& L) {
  if (!(mask.has_value() && mask->defined())) return nullptr;
  TORCH_CHECK(mask->scalar_type() == at::kByte && mask->is_contiguous() && L.s.channels_last && L.s.C % 8 == 0 &&
                  mask->numel() == L.s.outer * (L.s.C / 8), "relu mask must be uint8 [rows, C/8] from forward_mask");
  return mask->data_ptr<uint8_t>();
}

// returns (sums[2C], grad_weight, grad_bias) -- grads in weight dtype (undefined if weight undefined)
std::vector<at::Tensor> backward_reduce(at::Tensor dy_in, at::Tensor x_in, c10::optional<at::Tensor> z,
                                        at::Tensor mean, at::Tensor invstd, c10::optional<at::Tensor> scale,
                                        c10::optional<at::Tensor> shift, bool relu, c10::optional<at::Tensor> weight,
                                        bool need_weight_grads, c10::optional<at::Tensor> mask) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  at::Tensor dy = like(dy_in, L.x);
  at::Tensor zt;
  if (relu && z.has_value() && z->defined()) zt = like(*z, L.x);
  if (relu) TORCH_CHECK(scale.has_value() && shift.has_value(), "relu recompute needs scale/shift");
  const int C = L.s.C;
  const bool masked = relu && mask.has_value() && mask->defined();
  const int splits = bh::bn_num_splits_reduce(L.s, masked);
  auto part = at::empty({2 * (int64_t)splits * C}, fopt(L.x));
  auto sums = at::empty({2 * (int64_t)C}, fopt(L.x));
  at::Tensor gw, gb;
  const bool wdef = weight.has_value() && weight->defined();
  if (need_weight_grads && wdef) {
    gw = at::empty_like(*weight, at::MemoryFormat::Contiguous);
    gb = at::empty_like(*weight, at::MemoryFormat::Contiguous);
  }
  hipStream_t st = stream_for(L.x);
  bh::bn_backward_reduce(L.s, dtype_code(L.x.scalar_type()), dy.data_ptr(), L.x.data_ptr(),
                         zt.defined() ? dtype_code(zt.scalar_type()) : -1, zt.defined() ? zt.data_ptr() : nullptr,
                         mean.data_ptr<float>(), relu ? scale->data_ptr<float>() : nullptr,
                         relu ? shift->data_ptr<float>() : nullptr, relu, splits, part.data_ptr<float>(),
                         part.data_ptr<float>() + (int64_t)splits * C, st, relu ? mask_ptr(mask, L) : nullptr);
  bh::bn_backward_reduce_finalize(C, splits, part.data_ptr<float>(), part.data_ptr<float>() + (int64_t)splits * C,
                                  invstd.data_ptr<float>(), sums.data_ptr<float>(),
                                  gw.defined() ? dtype_code(gw.scalar_type()) : bh::kF32,
                                  gw.defined() ? gw.data_ptr() : nullptr, gb.defined() ? gb.data_ptr() : nullptr, st);
  return {sums, gw, gb};
}

// returns (dx, dz) ; dz undefined unless need_dz
std::vector<at::Tensor> backward_dgrad(at::Tensor dy_in, at::Tensor x_in, c10::optional<at::Tensor> z,
                                       at::Tensor mean, at::Tensor invstd, c10::optional<at::Tensor> weight,
                                       at::Tensor sums, at::Tensor count, c10::optional<at::Tensor> scale,
                                       c10::optional<at::Tensor> shift, bool relu, bool need_dz,
                                       c10::optional<at::Tensor> mask) {
  check_cuda(x_in, "input");
  Layout L = layout_of(x_in);
  at::Tensor dy = like(dy_in, L.x);
  at::Tensor zt;
  if (z.has_value() && z->defined()) zt = like(*z, L.x);
  if (relu) TORCH_CHECK(scale.has_value() && shift.has_value(), "relu recompute needs scale/shift");
  TORCH_CHECK(count.scalar_type() == at::kFloat && count.numel() >= 1, "count must be fp32");
  auto dx = at::empty_like(L.x);
  at::Tensor dz;
  if (need_dz) dz = at::empty_like(zt.defined() ? zt : L.x);
  bh::bn_backward_dgrad(L.s, dtype_code(L.x.scalar_type()), dy.data_ptr(), L.x.data_ptr(),
                        zt.defined() ? dtype_code(zt.scalar_type()) : (dz.defined() ? dtype_code(dz.scalar_type()) : -1),
                        zt.defined() ? zt.data_ptr() : nullptr, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                        wcode(weight), wptr(weight), sums.data_ptr<float>(), count.data_ptr<float>(),
                        relu ? scale->data_ptr<float>() : nullptr, relu ? shift->data_ptr<float>() : nullptr, relu,
                        dx.data_ptr(), dz.defined() ? dz.data_ptr() : nullptr, stream_for(L.x),
                        relu ? mask_ptr(mask, L) : nullptr);
  return {dx, dz};
}

// ---- NHWC max pooling, optionally fused with the BN affine + ReLU (kernels/pool.hip) ----
bh::PoolArgs pool_args(const at::Tensor& x, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p, bool relu) {
  bh::PoolArgs a;
  a.N = (int)x.size(0);
  a.C = (int)x.size(1);
  a.H = (int)H;
  a.W = (int)W;
  a.k = (int)k;
  a.stride = (int)s;
  a.pad = (int)p;
  a.OH = (int)((H + 2 * p - k) / s + 1);
  a.OW = (int)((W + 2 * p - k) / s + 1);
  a.relu = relu;
  TORCH_CHECK(a.C % 8 == 0 && k * k <= 255 && p <= k / 2 && a.OH > 0 && a.OW > 0,
              "maxpool_nhwc: needs C % 8 == 0, k*k <= 255, pad <= k/2");
  return a;
}

std::vector<at::Tensor> maxpool_forward(at::Tensor x, c10::optional<at::Tensor> scale, c10::optional<at::Tensor> shift,
                                        bool relu, int64_t k, int64_t s, int64_t p, bool want_idx,
                                        c10::optional<at::Tensor> num_batches) {
  check_cuda(x, "input");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_nhwc: 4-D channels_last input");
  const bool bn = scale.has_value() && scale->defined();
  if (bn)
    TORCH_CHECK(scale->scalar_type() == at::kFloat && shift->scalar_type() == at::kFloat && scale->numel() == x.size(1)
                    && scale->is_contiguous() && shift->is_contiguous(), "scale/shift must be contiguous fp32 [C]");
  bh::PoolArgs a = pool_args(x, x.size(2), x.size(3), k, s, p, relu);
  auto y = at::empty({a.N, a.C, a.OH, a.OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor idx;
  if (want_idx) idx = at::empty({a.N, a.C, a.OH, a.OW}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  bh::maxpool_forward_nhwc(a, dtype_code(x.scalar_type()), x.data_ptr(), bn ? scale->data_ptr<float>() : nullptr,
                           bn ? shift->data_ptr<float>() : nullptr, y.data_ptr(),
                           want_idx ? idx.data_ptr<uint8_t>() : nullptr, counter_ptr(num_batches), stream_for(x));
  return {y, idx};
}

at::Tensor maxpool_backward(at::Tensor gy, at::Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  check_cuda(gy, "grad_output");
  gy = gy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.sizes() == gy.sizes() &&
              idx.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_backward: idx must match grad_output");
  bh::PoolArgs a = pool_args(gy, H, W, k, s, p, false);
  TORCH_CHECK(a.OH == gy.size(2) && a.OW == gy.size(3), "maxpool_backward: output size mismatch");
  auto gx = at::empty({a.N, a.C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  bh::maxpool_backward_nhwc(a, dtype_code(gy.scalar_type()), gy.data_ptr(), idx.data_ptr<uint8_t>(), gx.data_ptr(),
                            stream_for(gy));
  return gx;
}

}  // namespace

void register_syncbn(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("syncbn", "batch-norm statistics / normalisation kernels (gfx950)");
  m.def("stats_local", &stats_local, "local [mean, var_biased, count] of x (all_gather payload)");
  m.def("stats_single", &stats_single, py::arg("x"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("num_batches") = py::none());
  m.def("merge_ranks", &merge_ranks, py::arg("gathered"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("num_batches") = py::none());
  m.def("stats_local_sums", &stats_local_sums, py::arg("x"), py::arg("running_mean") = py::none(),
        "local [sum(x-K), sum((x-K)^2), count] about K = running_mean (all_reduce SUM payload)");
  m.def("merge_parts", &merge_parts, py::arg("part"), py::arg("count"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("num_batches") = py::none(), py::arg("bump") = false,
        "single-rank finalize from conv-epilogue partials [2, G, C] (one launch); bump: num_batches += 1 too");
  m.def("merge_sums", &merge_sums, py::arg("sums"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("num_batches") = py::none());
  m.def("forward", &forward, py::arg("x"), py::arg("z"), py::arg("scale"), py::arg("shift"), py::arg("relu"),
        py::arg("out_dtype") = py::none(), py::arg("num_batches") = py::none());
  m.def("backward_reduce", &backward_reduce, py::arg("dy"), py::arg("x"), py::arg("z"), py::arg("mean"),
        py::arg("invstd"), py::arg("scale"), py::arg("shift"), py::arg("relu"), py::arg("weight"),
        py::arg("need_weight_grads"), py::arg("mask") = py::none());
  m.def("backward_dgrad", &backward_dgrad, py::arg("dy"), py::arg("x"), py::arg("z"), py::arg("mean"),
        py::arg("invstd"), py::arg("weight"), py::arg("sums"), py::arg("count"), py::arg("scale"), py::arg("shift"),
        py::arg("relu"), py::arg("need_dz"), py::arg("mask") = py::none());
  m.def("forward_mask", &forward_mask, py::arg("x"), py::arg("z"), py::arg("scale"), py::arg("shift"),
        py::arg("num_batches") = py::none(), py::arg("zscale") = py::none(), py::arg("zshift") = py::none(),
        "fused BN + (z, or BN(z) with zscale / zshift) + ReLU that also returns the uint8 [rows, C/8] ReLU bit mask");
  m.def("mask_ok", &mask_ok);
  m.def("maxpool_forward", &maxpool_forward, py::arg("x"), py::arg("scale"), py::arg("shift"), py::arg("relu"),
        py::arg("kernel_size"), py::arg("stride"), py::arg("padding"), py::arg("want_idx"),
        py::arg("num_batches") = py::none(),
        "NHWC max pool of (relu)(x*scale+shift): returns (y, uint8 argmax offsets)");
  m.def("maxpool_backward", &maxpool_backward, py::arg("grad_output"), py::arg("idx"), py::arg("H"), py::arg("W"),
        py::arg("kernel_size"), py::arg("stride"), py::arg("padding"));
}

}  // namespace bhb
