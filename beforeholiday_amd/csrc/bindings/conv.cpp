// `conv_cuda`: direct 3x3 / stride 1 / pad 1 NHWC convolution (kernels/conv.hip), used by the fused
// ResNet bottleneck for its middle conv (forward, and data gradient through flipped weights).
#include "common.h"

#include "bh/conv_api.h"
#include "bh/dense_api.h"
#include "bh/igemm_api.h"

namespace bhb {
namespace {

bh::Conv3x3Args conv_args(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y) {
  bh::Conv3x3Args a;
  a.x = x.data_ptr();
  a.w = w.data_ptr();
  a.y = y.data_ptr();
  a.N = (int)x.size(0);
  a.C = (int)x.size(1);
  a.H = (int)x.size(2);
  a.W = (int)x.size(3);
  a.K = (int)w.size(0);
  return a;
}

bool shapes_ok(const at::Tensor& x, const at::Tensor& w) {
  return x.is_cuda() && w.is_cuda() && x.dim() == 4 && w.dim() == 4 && w.size(1) == x.size(1) && w.size(2) == 3 &&
         w.size(3) == 3 && x.scalar_type() == w.scalar_type() &&
         (x.scalar_type() == at::kHalf || x.scalar_type() == at::kBFloat16) &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 64 == 0 && w.size(0) % 64 == 0;
}

// True when conv3x3_forward covers (x, w): channels_last fp16 / bf16, C and K multiples of 64.
bool supported(const at::Tensor& x, const at::Tensor& w) { return shapes_ok(x, w); }

// y = conv2d(x, w, stride 1, padding 1) for channels_last x [N, C, H, W], w [K, C, 3, 3]; y channels_last
at::Tensor conv3x3_forward(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(shapes_ok(x, w), "conv3x3_forward: needs channels_last fp16/bf16 x, w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);  // [K][3][3][C] in memory
  auto y = at::empty({x.size(0), w.size(0), x.size(2), x.size(3)}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const auto a = conv_args(x, wc, y);
  TORCH_CHECK(bh::conv3x3_supported(a), "conv3x3_forward: unaligned tensors");
  bh::conv3x3_forward(dtype_code(x.scalar_type()), a, stream_for(x));
  return y;
}

// dX of y = conv2d(x, w, stride 1, padding 1) from dY (channels_last) and the forward's w
at::Tensor conv3x3_dgrad(const at::Tensor& dy, const at::Tensor& w) {
  TORCH_CHECK(dy.is_cuda() && w.is_cuda() && dy.dim() == 4 && w.dim() == 4 && w.size(0) == dy.size(1) &&
                  w.size(2) == 3 && w.size(3) == 3 && dy.scalar_type() == w.scalar_type() &&
                  (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(0) % 64 == 0 && w.size(1) % 64 == 0,
              "conv3x3_dgrad: needs channels_last fp16/bf16 dy, w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto dx = at::empty({dy.size(0), w.size(1), dy.size(2), dy.size(3)},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  bh::Conv3x3Args a;
  a.x = dy.data_ptr();
  a.w = wc.data_ptr();
  a.y = dx.data_ptr();
  a.N = (int)dy.size(0);
  a.C = (int)dy.size(1);
  a.H = (int)dy.size(2);
  a.W = (int)dy.size(3);
  a.K = (int)w.size(1);
  TORCH_CHECK(bh::conv3x3_supported(a), "conv3x3_dgrad: unaligned tensors");
  bh::conv3x3_dgrad(dtype_code(dy.scalar_type()), a, stream_for(dy));
  return dx;
}

const float* f32_or_null(const c10::optional<at::Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == n, what,
              " must be a contiguous fp32 GPU tensor of ", n, " elements");
  return t->data_ptr<float>();
}

// conv3x3_forward with the BatchNorm folding: x is the producing layer's RAW output when pro_scale /
// pro_shift are given (relu(x * scale + shift) is convolved); stats=True also returns the per-workgroup
// partial sums [2, G, K] of (y - kshift) and (y - kshift)^2 (conv_bn.sum_parts reduces them)
std::vector<at::Tensor> conv3x3_bn_forward(const at::Tensor& x, const at::Tensor& w,
                                           const c10::optional<at::Tensor>& pro_scale,
                                           const c10::optional<at::Tensor>& pro_shift, bool stats,
                                           const c10::optional<at::Tensor>& kshift) {
  TORCH_CHECK(shapes_ok(x, w), "conv3x3_bn_forward: needs channels_last fp16/bf16 x, w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({x.size(0), w.size(0), x.size(2), x.size(3)}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = conv_args(x, wc, y);
  a.pro_scale = f32_or_null(pro_scale, a.C, "pro_scale");
  a.pro_shift = f32_or_null(pro_shift, a.C, "pro_shift");
  at::Tensor part = at::empty({0}, x.options().dtype(at::kFloat));
  if (stats) {
    a.epi = bh::kConvEpiStats;
    a.kshift = f32_or_null(kshift, a.K, "kshift");
    part = at::empty({2, (int64_t)bh::conv3x3_parts(a), (int64_t)a.K}, x.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  TORCH_CHECK(bh::conv3x3_supported(a), "conv3x3_bn_forward: unsupported arguments (C <= 512 with a prologue)");
  bh::conv3x3_forward(dtype_code(x.scalar_type()), a, stream_for(x));
  return {y, part};
}

// y = relu?(conv3x3(x, w) * scale + shift (+ r)) (* r when r_mul): conv + bias / frozen BatchNorm
// (+ residual) (+ ReLU) (x mask) in one kernel
at::Tensor conv3x3_affine(const at::Tensor& x, const at::Tensor& w, const at::Tensor& scale, const at::Tensor& shift,
                          bool relu, const c10::optional<at::Tensor>& r, bool r_mul) {
  TORCH_CHECK(shapes_ok(x, w), "conv3x3_affine: needs channels_last fp16/bf16 x, w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({x.size(0), w.size(0), x.size(2), x.size(3)}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = conv_args(x, wc, y);
  a.epi = bh::kConvEpiAffine;
  a.a_scale = f32_or_null(scale, a.K, "scale");
  a.a_shift = f32_or_null(shift, a.K, "shift");
  a.relu = relu;
  a.r_mul = r_mul;
  if (r.has_value() && r->defined()) {
    TORCH_CHECK(r->is_cuda() && r->device() == x.device() && r->scalar_type() == x.scalar_type() &&
                    r->sizes() == y.sizes() && r->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3_affine: r must be a channels_last tensor shaped like the output");
    a.r = r->data_ptr();
  }
  TORCH_CHECK(bh::conv3x3_supported(a), "conv3x3_affine: unsupported arguments");
  bh::conv3x3_forward(dtype_code(x.scalar_type()), a, stream_for(x));
  return y;
}

// conv3x3_dgrad whose epilogue also reduces the PREVIOUS BatchNorm's backward sums: by is that
// BatchNorm's raw input (same shape as dx), dz = dx * (by * bscale + bshift > 0) (brelu): partials
// [2, G, C] of dz and dz * (by - bmean)
std::vector<at::Tensor> conv3x3_bn_dgrad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& by,
                                         const at::Tensor& bscale, const at::Tensor& bshift, const at::Tensor& bmean,
                                         bool brelu) {
  TORCH_CHECK(dy.is_cuda() && w.is_cuda() && dy.dim() == 4 && w.dim() == 4 && w.size(0) == dy.size(1) &&
                  w.size(2) == 3 && w.size(3) == 3 && dy.scalar_type() == w.scalar_type() &&
                  (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(0) % 64 == 0 && w.size(1) % 64 == 0,
              "conv3x3_bn_dgrad: needs channels_last fp16/bf16 dy, w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto dx = at::empty({dy.size(0), w.size(1), dy.size(2), dy.size(3)},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  TORCH_CHECK(by.is_cuda() && by.device() == dy.device() && by.scalar_type() == dy.scalar_type() &&
                  by.sizes() == dx.sizes() && by.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_bn_dgrad: by must be a channels_last tensor shaped like dx");
  bh::Conv3x3Args a;
  a.x = dy.data_ptr();
  a.w = wc.data_ptr();
  a.y = dx.data_ptr();
  a.N = (int)dy.size(0);
  a.C = (int)dy.size(1);
  a.H = (int)dy.size(2);
  a.W = (int)dy.size(3);
  a.K = (int)w.size(1);
  a.epi = bh::kConvEpiBwd;
  a.by = by.data_ptr();
  a.bscale = f32_or_null(bscale, a.K, "bscale");
  a.bshift = f32_or_null(bshift, a.K, "bshift");
  a.bmean = f32_or_null(bmean, a.K, "bmean");
  a.brelu = brelu;
  auto part = at::empty({2, (int64_t)bh::conv3x3_parts(a), (int64_t)a.K}, dy.options().dtype(at::kFloat));
  a.part = part.data_ptr<float>();
  TORCH_CHECK(bh::conv3x3_supported(a), "conv3x3_bn_dgrad: unaligned tensors");
  bh::conv3x3_dgrad(dtype_code(dy.scalar_type()), a, stream_for(dy));
  return {dx, part};
}

// dW of y = conv2d(x, w, stride 1, padding (R-1)/2) for channels_last x [N, C, H, W], dy [N, K, H, W];
// returns [K, C, R, R] channels_last (memory [K][R][R][C])
bool wgrad_ok(const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride = 1) {
  return x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4 && x.size(0) == dy.size(0) &&
         (stride == 1 || stride == 2) && x.size(2) == stride * dy.size(2) &&
         x.size(3) == stride * dy.size(3) && x.scalar_type() == dy.scalar_type() &&
         (x.scalar_type() == at::kHalf || x.scalar_type() == at::kBFloat16) &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
         (R == 1 || R == 3) && x.size(1) % 64 == 0 && dy.size(1) % 64 == 0 &&
         x.numel() < (int64_t(1) << 40);
}

bh::ConvWgradArgs wgrad_args(const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride) {
  bh::ConvWgradArgs a;
  a.x = x.data_ptr();
  a.dy = dy.data_ptr();
  a.N = (int)x.size(0);
  a.C = (int)x.size(1);
  a.H = (int)dy.size(2);  // output (dY) geometry; x is stride x larger
  a.W = (int)dy.size(3);
  a.K = (int)dy.size(1);
  a.R = (int)R;
  a.stride = (int)stride;
  return a;
}

bool wgrad_supported(const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride) {
  if (!wgrad_ok(x, dy, R, stride)) return false;
  bh::ConvWgradGeo g;
  auto a = wgrad_args(x, dy, R, stride);
  a.out = x.data_ptr();  // alignment probe only
  return bh::conv_wgrad_plan(a, &g);
}

// defer = true: the split partials are returned instead of summed ([out, ws or None]); the caller sums
// them with conv_wgrad_reduce (on a side stream: nothing on the critical path waits for them)
std::vector<at::Tensor> conv_wgrad_impl(const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride,
                                        const c10::optional<at::Tensor>& pro_scale,
                                        const c10::optional<at::Tensor>& pro_shift, bool defer, bool f32 = false) {
  TORCH_CHECK(wgrad_ok(x, dy, R, stride), "conv_wgrad: needs channels_last fp16/bf16 x [N, C, sH, sW], "
                                          "dy [N, K, H, W], C and K % 64 == 0, R in {1, 3}, stride in {1, 2}");
  auto out = at::empty({dy.size(1), x.size(1), R, R}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = wgrad_args(x, dy, R, stride);
  a.out = out.data_ptr();
  at::Tensor ps, ph;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined() && (stride == 1 || R == 3),
                "conv_wgrad: the BatchNorm prologue needs pro_scale and pro_shift (1x1: stride 1)");
    ps = pro_scale->contiguous();
    ph = pro_shift->contiguous();
    TORCH_CHECK(ps.is_cuda() && ph.is_cuda() && ps.device() == x.device() && ph.device() == x.device() &&
                    ps.scalar_type() == at::kFloat && ph.scalar_type() == at::kFloat && ps.numel() == x.size(1) &&
                    ph.numel() == x.size(1),
                "conv_wgrad: pro_scale / pro_shift must be fp32 [C] tensors on x's device");
    a.pro_scale = ps.data_ptr<float>();
    a.pro_shift = ph.data_ptr<float>();
  }
  bh::ConvWgradGeo g;
  TORCH_CHECK(bh::conv_wgrad_plan(a, &g), "conv_wgrad: shape not covered (window does not fit in LDS / unaligned)");
  g.f32 = f32;
  const int64_t nws = bh::conv_wgrad_workspace(g, a);
  at::Tensor ws;
  if (nws > 0) ws = at::empty({nws}, x.options().dtype(at::kFloat));
  bh::conv_wgrad(dtype_code(x.scalar_type()), a, g, nws > 0 ? ws.data_ptr<float>() : nullptr, stream_for(x), !defer);
  if (!defer || nws == 0) return {out, at::Tensor()};
  return {out, ws.view({(int64_t)g.parts, -1})};
}

at::Tensor conv_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride,
                      const c10::optional<at::Tensor>& pro_scale, const c10::optional<at::Tensor>& pro_shift) {
  return conv_wgrad_impl(x, dy, R, stride, pro_scale, pro_shift, false)[0];
}

// out (the [K, C, R, R] gradient conv_wgrad_deferred returned) = sum over the rows of ws [parts, n],
// on the current stream
void conv_wgrad_reduce(const at::Tensor& ws, const at::Tensor& out) {
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.dim() == 2 && ws.is_contiguous() &&
                  out.is_cuda() && ws.size(1) == out.numel() && ws.size(1) % 4 == 0,
              "conv_wgrad_reduce: ws [parts, n] fp32 and out with n elements");
  bh::conv_wgrad_reduce(dtype_code(out.scalar_type()), ws.data_ptr<float>(), out.data_ptr(), ws.size(1),
                        (int)ws.size(0), stream_for(out));
}

bool stem_ok(const at::Tensor& x, const at::Tensor& w) {
  return x.is_cuda() && w.is_cuda() && x.dim() == 4 && w.dim() == 4 && x.scalar_type() == w.scalar_type() &&
         (x.scalar_type() == at::kHalf || x.scalar_type() == at::kBFloat16) &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
         bh::conv_stem_supported((int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)w.size(0)) &&
         (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0;
}

// conv2d(x, w, stride 2, padding 3) of the ResNet stem (x [N, 3, 224, 224] channels_last, w [64, 3, 7, 7])
at::Tensor stem_forward(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(stem_ok(x, w), "stem_forward: needs channels_last fp16/bf16 x [N, 3, 224, 224], w [64, 3, 7, 7]");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);  // [64][7][7][3]
  auto y = at::empty({x.size(0), 64, 112, 112}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  bh::conv_stem_forward(dtype_code(x.scalar_type()), x.data_ptr(), wc.data_ptr(), y.data_ptr(), (int)x.size(0),
                        stream_for(x));
  return y;
}

// stem forward + the BatchNorm statistics partials of its output ([2, G, 64] about kshift)
std::vector<at::Tensor> stem_forward_stats(const at::Tensor& x, const at::Tensor& w,
                                           const c10::optional<at::Tensor>& kshift) {
  TORCH_CHECK(stem_ok(x, w), "stem_forward_stats: needs channels_last fp16/bf16 x [N, 3, 224, 224], w [64, 3, 7, 7]");
  const float* kp = nullptr;
  at::Tensor kc;
  if (kshift.has_value() && kshift->defined()) {
    kc = kshift->contiguous();
    TORCH_CHECK(kc.is_cuda() && kc.device() == x.device() && kc.scalar_type() == at::kFloat && kc.numel() == 64,
                "stem_forward_stats: kshift must be an fp32 [64] tensor on x's device");
    kp = kc.data_ptr<float>();
  }
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({x.size(0), 64, 112, 112}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int G = bh::conv_stem_parts((int)x.size(0));
  auto part = at::empty({2, G, 64}, x.options().dtype(at::kFloat));
  bh::conv_stem_forward(dtype_code(x.scalar_type()), x.data_ptr(), wc.data_ptr(), y.data_ptr(), (int)x.size(0),
                        stream_for(x), kp, part.data_ptr<float>());
  return {y, part};
}

bool gemm_n64_ok(const at::Tensor& a, const at::Tensor& b) {
  auto al = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  return a.is_cuda() && b.is_cuda() && a.device() == b.device() && a.dim() == 2 && b.dim() == 2 && a.scalar_type() == b.scalar_type() &&
         (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16) && a.is_contiguous() && b.is_contiguous() &&
         a.size(1) == b.size(1) && al(a) && al(b) && bh::gemm_n64_supported(a.size(0), (int)a.size(1), (int)b.size(0));
}

at::Tensor gemm_n64(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& resid) {
  TORCH_CHECK(gemm_n64_ok(a, b), "gemm_n64: contiguous aligned fp16/bf16 a [M, K], b [64, K], K in {64, 128, 256}, "
                                 "M % 32 == 0");
  auto c = at::empty({a.size(0), 64}, a.options());
  const void* r = nullptr;
  if (resid.has_value()) {
    TORCH_CHECK(resid->is_cuda() && resid->device() == a.device() && resid->sizes() == c.sizes() &&
                    resid->is_contiguous() && resid->scalar_type() == a.scalar_type() &&
                    (reinterpret_cast<uintptr_t>(resid->data_ptr()) & 15) == 0,
                "gemm_n64: resid must be a contiguous aligned [M, 64] tensor of a's dtype on a's device");
    r = resid->data_ptr();
  }
  bh::gemm_n64(dtype_code(a.scalar_type()), a.data_ptr(), b.data_ptr(), r, c.data_ptr(), a.size(0), (int)a.size(1),
               stream_for(a));
  return c;
}

// weight gradient of stem_forward: [64, 3, 7, 7] channels_last from x and dy [N, 64, 112, 112] channels_last
at::Tensor stem_wgrad(const at::Tensor& x, const at::Tensor& dy) {
  TORCH_CHECK(x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4 && x.scalar_type() == dy.scalar_type() &&
                  (x.scalar_type() == at::kHalf || x.scalar_type() == at::kBFloat16) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  bh::conv_stem_supported((int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), 64) &&
                  dy.size(0) == x.size(0) && dy.size(1) == 64 && dy.size(2) == 112 && dy.size(3) == 112 &&
                  (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "stem_wgrad: needs channels_last fp16/bf16 x [N, 3, 224, 224], dy [N, 64, 112, 112]");
  auto out = at::empty({64, 3, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto ws = at::empty({(int64_t)bh::conv_stem_wgrad_parts((int)x.size(0)) * 64 * 7 * 21}, x.options().dtype(at::kFloat));
  bh::conv_stem_wgrad(dtype_code(x.scalar_type()), x.data_ptr(), dy.data_ptr(), out.data_ptr(), ws.data_ptr<float>(),
                      (int)x.size(0), stream_for(x));
  return out;
}

// ---- stride-2 3x3 / pad 1 (kernels/conv_igemm.hip) ----
bool s2_ok(const at::Tensor& x, const at::Tensor& w) {
  return shapes_ok(x, w) && w.size(0) % 64 == 0 && x.size(2) % 2 == 0 && x.size(3) % 2 == 0 && w.device() == x.device();
}

bool s2_supported(const at::Tensor& x, const at::Tensor& w) {
  if (!s2_ok(x, w)) return false;
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto a = bh::igemm_conv3x3_s2_fwd(x.data_ptr(), wc.data_ptr(), x.data_ptr(), (int)x.size(0), (int)x.size(2),
                                    (int)x.size(3), (int)x.size(1), (int)w.size(0));
  return bh::igemm_supported(a);
}

// conv2d(x, w, stride 2, padding 1) of channels_last x [N, C, H, W] (H, W even), w [K, C, 3, 3]; with
// pro_scale / pro_shift x is the raw input of a BatchNorm + ReLU applied on the fly (padding stays zero);
// stats: also the statistics partials [2, G, K] of the output about kshift
std::vector<at::Tensor> conv3x3_s2_forward(const at::Tensor& x, const at::Tensor& w,
                                           const c10::optional<at::Tensor>& pro_scale,
                                           const c10::optional<at::Tensor>& pro_shift, bool stats,
                                           const c10::optional<at::Tensor>& kshift) {
  TORCH_CHECK(s2_ok(x, w), "conv3x3_s2_forward: needs channels_last fp16/bf16 x [N, C, H, W] (H, W even), "
                           "w [K, C, 3, 3], C and K % 64 == 0");
  const at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({x.size(0), w.size(0), x.size(2) / 2, x.size(3) / 2},
                     x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = bh::igemm_conv3x3_s2_fwd(x.data_ptr(), wc.data_ptr(), y.data_ptr(), (int)x.size(0), (int)x.size(2),
                                    (int)x.size(3), (int)x.size(1), (int)w.size(0));
  at::Tensor ps, ph, kc, part;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "conv3x3_s2_forward: pro_scale needs pro_shift");
    ps = pro_scale->contiguous();
    ph = pro_shift->contiguous();
    TORCH_CHECK(ps.scalar_type() == at::kFloat && ph.scalar_type() == at::kFloat && ps.numel() == x.size(1) &&
                    ph.numel() == x.size(1) && ps.device() == x.device() && ph.device() == x.device(),
                "conv3x3_s2_forward: pro_scale / pro_shift must be fp32 [C] on x's device");
    a.pro_scale = ps.data_ptr<float>();
    a.pro_shift = ph.data_ptr<float>();
  }
  if (stats) {
    if (kshift.has_value() && kshift->defined()) {
      kc = kshift->contiguous();
      TORCH_CHECK(kc.scalar_type() == at::kFloat && kc.numel() == w.size(0) && kc.device() == x.device(),
                  "conv3x3_s2_forward: kshift must be fp32 [K] on x's device");
      a.kshift = kc.data_ptr<float>();
    }
    part = at::empty({2, (int64_t)bh::igemm_parts(a), w.size(0)}, x.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  } else {
    part = at::empty({0}, x.options().dtype(at::kFloat));
  }
  TORCH_CHECK(bh::igemm_supported(a), "conv3x3_s2_forward: unsupported arguments (alignment / size)");
  bh::igemm_run(dtype_code(x.scalar_type()), a, stream_for(x));
  return {y, part};
}

// grad of conv2d(x, w, stride 2, padding 1) w.r.t. x (x [N, C, H, W], H and W even) from dy [N, K, H/2, W/2]
at::Tensor conv3x3_s2_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && w.is_cuda() && dy.dim() == 4 && w.dim() == 4 && w.size(0) == dy.size(1) &&
                  w.size(2) == 3 && w.size(3) == 3 && dy.scalar_type() == w.scalar_type() &&
                  (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.size(1) % 64 == 0 && w.size(1) % 64 == 0 &&
                  H % 2 == 0 && W % 2 == 0 && dy.size(2) == H / 2 && dy.size(3) == W / 2,
              "conv3x3_s2_dgrad: needs channels_last fp16/bf16 dy [N, K, H/2, W/2], w [K, C, 3, 3], C and K % 64 == 0");
  // [C][3][3][K]: the weights with input and output channels swapped (a 9 C K-element copy)
  const at::Tensor wt = w.transpose(0, 1).contiguous(at::MemoryFormat::ChannelsLast);
  auto dx = at::empty({dy.size(0), w.size(1), H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = bh::igemm_conv3x3_s2_dgrad(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), (int)dy.size(0), (int)H, (int)W,
                                      (int)w.size(1), (int)w.size(0));
  TORCH_CHECK(bh::igemm_supported(a), "conv3x3_s2_dgrad: unsupported arguments (alignment / size)");
  bh::igemm_run(dtype_code(dy.scalar_type()), a, stream_for(dy));
  return dx;
}

}  // namespace

// The dense layers' weight gradient dW [N, K] = dy [T, N]^T . x [T, K] on the 1x1 weight-gradient kernel
// (tokens as a 1 x 1 x T image); false when the kernel does not take the shape (dense.cpp weight_grad)
bool dense_wgrad_conv(const at::Tensor& dy, const at::Tensor& x, at::Tensor& out) {
  if (!(dy.dim() == 2 && x.dim() == 2 && dy.is_contiguous() && x.is_contiguous() && dy.size(0) == x.size(0)))
    return false;
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  const at::Tensor x4 = x.view({1, 1, T, K}).permute({0, 3, 1, 2});
  const at::Tensor dy4 = dy.view({1, 1, T, N}).permute({0, 3, 1, 2});
  if (!wgrad_supported(x4, dy4, 1, 1)) return false;
  out = conv_wgrad(x4, dy4, 1, 1, c10::nullopt, c10::nullopt).view({N, K});
  return true;
}

void register_conv(pybind11::module_& root) {
  auto m = root.def_submodule("conv_cuda", "direct 3x3 stride-1 NHWC convolution (MFMA implicit GEMM)");
  m.def("conv3x3_forward", &conv3x3_forward, py::arg("x"), py::arg("weight"),
        "conv2d(x, weight, stride=1, padding=1) for channels_last fp16 / bf16, C and K multiples of 64");
  m.def("conv3x3_dgrad", &conv3x3_dgrad, py::arg("grad_out"), py::arg("weight"),
        "grad of conv2d(x, weight, stride=1, padding=1) w.r.t. x, straight from the forward weight");
  m.def("supported", &supported, py::arg("x"), py::arg("weight"));
  m.def("conv3x3_bn_forward", &conv3x3_bn_forward, py::arg("x"), py::arg("weight"), py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("stats") = false, py::arg("kshift") = py::none());
  m.def("conv3x3_affine", &conv3x3_affine, py::arg("x"), py::arg("weight"), py::arg("scale"), py::arg("shift"),
        py::arg("relu") = true, py::arg("r") = py::none(), py::arg("r_mul") = false);
  m.def("conv3x3_bn_dgrad", &conv3x3_bn_dgrad, py::arg("grad_out"), py::arg("weight"), py::arg("by"),
        py::arg("bscale"), py::arg("bshift"), py::arg("bmean"), py::arg("brelu") = true);
  m.def("stem_forward_stats", &stem_forward_stats, py::arg("x"), py::arg("weight"), py::arg("kshift") = py::none(),
        "ResNet stem conv (7x7/2, 3 -> 64) + BatchNorm statistics partials [2, G, 64] of its output about kshift");
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("grad_out"), py::arg("R"), py::arg("stride") = 1,
        py::arg("pro_scale") = py::none(), py::arg("pro_shift") = py::none(),
        "weight gradient of conv2d(x', w, stride, padding=(R-1)//2), R in {1, 3}, stride in {1, 2}, x' = x or "
        "relu(x * pro_scale + pro_shift) per channel: [K, C, R, R] channels_last");
  m.def("conv_wgrad_deferred", [](const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride,
                                  const c10::optional<at::Tensor>& ps, const c10::optional<at::Tensor>& ph) {
    return conv_wgrad_impl(x, dy, R, stride, ps, ph, true);
  }, py::arg("x"), py::arg("grad_out"), py::arg("R"), py::arg("stride") = 1, py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(),
        "conv_wgrad without the split-partials sum: [out (not yet written when ws is returned), ws [parts, n] or None]");
  m.def("conv_wgrad_reduce", &conv_wgrad_reduce, py::arg("ws"), py::arg("out"));
  m.def("conv_wgrad_f32", [](const at::Tensor& x, const at::Tensor& dy, int64_t R, int64_t stride,
                             const c10::optional<at::Tensor>& ps, const c10::optional<at::Tensor>& ph) {
    return conv_wgrad_impl(x, dy, R, stride, ps, ph, true, true)[1];
  }, py::arg("x"), py::arg("grad_out"), py::arg("R"), py::arg("stride") = 1, py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(),
        "the weight-gradient product as fp32 split partials [parts, K * C * R * R] (never rounded to 16 bits; "
        "sum over dim 0 in any fixed order)");
  m.def("wgrad_supported", &wgrad_supported, py::arg("x"), py::arg("grad_out"), py::arg("R"), py::arg("stride") = 1);
  m.def("gemm_n64", &gemm_n64, py::arg("a"), py::arg("b"), py::arg("resid") = c10::nullopt,
        "a [M, K] . b[64, K]^T (+ resid [M, 64]), K in {64, 128, 256}, M % 32 == 0 (kernels/gemm_n64.hip)");
  m.def("gemm_n64_supported", &gemm_n64_ok, py::arg("a"), py::arg("b"));
  m.def("stem_forward", &stem_forward, py::arg("x"), py::arg("weight"),
        "ResNet stem conv2d(x, w, stride=2, padding=3), 3 -> 64 channels at 224x224, channels_last fp16 / bf16");
  m.def("conv3x3_s2_forward", &conv3x3_s2_forward, py::arg("x"), py::arg("weight"), py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("stats") = false, py::arg("kshift") = py::none(),
        "conv2d(x', w, stride=2, padding=1) on the implicit-GEMM MFMA kernel (x' = x or relu(x * pro_scale + "
        "pro_shift)); returns [y, statistics partials [2, G, K] about kshift (empty unless stats)]");
  m.def("conv3x3_s2_dgrad", &conv3x3_s2_dgrad, py::arg("grad_out"), py::arg("weight"), py::arg("H"), py::arg("W"),
        "grad of conv2d(x, w, stride=2, padding=1) w.r.t. x [N, C, H, W]: four stride-1 phase convolutions in one launch");
  m.def("s2_supported", &s2_supported, py::arg("x"), py::arg("weight"));
  m.def("stem_supported", &stem_ok, py::arg("x"), py::arg("weight"));
  m.def("stem_wgrad", &stem_wgrad, py::arg("x"), py::arg("grad_out"),
        "weight gradient of the ResNet stem conv (7x7 / 2, 3 -> 64 at 224x224): [64, 3, 7, 7] channels_last");
}

}  // namespace bhb
