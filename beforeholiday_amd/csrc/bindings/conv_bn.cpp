// `conv_bn`: 1x1 convolution GEMMs with BatchNorm prologue / statistics epilogues
// (kernels/conv_bn.hip, bh/conv_bn_api.h) on [pixels, channels] views of NHWC activations.
#include "common.h"

#include "bh/conv_bn_api.h"
#include "bh/gemm_api.h"

namespace bhb {
namespace {

const float* fptr(const c10::optional<at::Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == n, what,
              " must be a contiguous fp32 GPU tensor of ", n, " elements");
  return t->data_ptr<float>();
}

bh::C1x1Args make_args(const at::Tensor& a, const at::Tensor& b, bool b_trans, int64_t M,
                       const c10::optional<at::Tensor>& pro_scale,
                       const c10::optional<at::Tensor>& pro_shift, const c10::optional<at::Tensor>& resid,
                       int64_t s2_h, int64_t s2_w, int64_t epi, const c10::optional<at::Tensor>& kshift,
                       const c10::optional<at::Tensor>& by, const c10::optional<at::Tensor>& bscale,
                       const c10::optional<at::Tensor>& bshift, const c10::optional<at::Tensor>& bmean, bool brelu) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.device() == b.device() && a.dim() == 2 && b.dim() == 2 &&
                  a.is_contiguous() && b.is_contiguous() && a.scalar_type() == b.scalar_type() &&
                  a.size(1) == b.size(b_trans ? 0 : 1),
              "conv_bn.c1x1: a [rows, K] and b [N, K] ([K, N] with b_trans) contiguous GPU tensors of one dtype");
  bh::C1x1Args p;
  p.A = a.data_ptr();
  p.B = b.data_ptr();
  p.b_trans = b_trans;
  p.M = M;
  p.K = (int)a.size(1);
  p.N = (int)b.size(b_trans ? 1 : 0);
  p.pro_scale = fptr(pro_scale, p.K, "pro_scale");
  p.pro_shift = fptr(pro_shift, p.K, "pro_shift");
  TORCH_CHECK((p.pro_scale == nullptr) == (p.pro_shift == nullptr), "conv_bn.c1x1: pro_scale and pro_shift together");
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->is_cuda() && resid->device() == a.device() && resid->scalar_type() == a.scalar_type() &&
                    resid->is_contiguous() && resid->numel() == M * p.N,
                "conv_bn.c1x1: resid must be a contiguous [M, N] tensor of a's dtype on a's device");
    p.R = resid->data_ptr();
  }
  p.s2_H = (int)s2_h;
  p.s2_W = (int)s2_w;
  if (s2_h > 0) {
    TORCH_CHECK(a.size(0) * (s2_h / 2) * (s2_w / 2) == M * s2_h * s2_w, "conv_bn.c1x1: stride-2 rows");
  } else {
    TORCH_CHECK(a.size(0) == M, "conv_bn.c1x1: a has M rows");
  }
  p.epi = (int)epi;
  p.kshift = fptr(kshift, p.N, "kshift");
  if (epi == bh::kC1x1Bwd) {
    TORCH_CHECK(by.has_value() && by->defined() && by->is_cuda() && by->device() == a.device() &&
                    by->scalar_type() == a.scalar_type() && by->is_contiguous() && by->numel() == M * p.N,
                "conv_bn.c1x1: by must be a contiguous [M, N] tensor of a's dtype");
    p.by = by->data_ptr();
    p.bscale = fptr(bscale, p.N, "bscale");
    p.bshift = fptr(bshift, p.N, "bshift");
    p.bmean = fptr(bmean, p.N, "bmean");
    p.brelu = brelu;
  }
  return p;
}

// returns (C [M, N], partials [2, G, N] fp32 or an empty tensor for the plain epilogue)
std::vector<at::Tensor> c1x1(const at::Tensor& a, const at::Tensor& b, bool b_trans, int64_t M,
                             const c10::optional<at::Tensor>& pro_scale, const c10::optional<at::Tensor>& pro_shift,
                             const c10::optional<at::Tensor>& resid, int64_t s2_h, int64_t s2_w, int64_t epi,
                             const c10::optional<at::Tensor>& kshift, const c10::optional<at::Tensor>& by,
                             const c10::optional<at::Tensor>& bscale, const c10::optional<at::Tensor>& bshift,
                             const c10::optional<at::Tensor>& bmean, bool brelu, bool s2_scatter,
                             const c10::optional<at::Tensor>& a_scale, const c10::optional<at::Tensor>& a_shift,
                             bool relu, bool r_mul, const c10::optional<at::Tensor>& bnb,
                             const c10::optional<at::Tensor>& bnb_y, const c10::optional<at::Tensor>& mbits,
                             int64_t lda) {
  at::Tensor c;
  if (s2_scatter) {
    // accumulate into the full-resolution tensor `resid` in place: a is [M, K], resid [4M, N]
    TORCH_CHECK(s2_h > 0 && resid.has_value() && resid->defined() && resid->is_cuda() &&
                    resid->device() == a.device() && resid->scalar_type() == a.scalar_type() &&
                    resid->is_contiguous() && resid->dim() == 2 && resid->size(0) == 4 * M &&
                    a.size(0) == M,
                "conv_bn.c1x1: the stride-2 scatter accumulates into a contiguous [4M, N] resid");
    c = *resid;
  }
  // lda > 0: a (and bnb_y) are [M, K] column slices of row-major [M, lda] tensors
  TORCH_CHECK(lda == 0 || (a.dim() == 2 && a.stride(1) == 1 && a.stride(0) == lda &&
                           (!bnb_y.has_value() || !bnb_y->defined() ||
                            (bnb_y->dim() == 2 && bnb_y->stride(1) == 1 && bnb_y->stride(0) == lda))),
              "conv_bn.c1x1: lda must equal the row stride of a (and bnb_y)");
  bh::C1x1Args p = make_args(lda ? a.as_strided({a.size(0), a.size(1)}, {a.size(1), 1}) : a, b, b_trans, M, pro_scale,
                             pro_shift, s2_scatter ? c10::optional<at::Tensor>() : resid,
                             s2_scatter ? 0 : s2_h, s2_scatter ? 0 : s2_w, epi, kshift, by, bscale, bshift, bmean,
                             brelu);
  if (s2_scatter) {
    p.s2_H = (int)s2_h;
    p.s2_W = (int)s2_w;
    p.s2_scatter = true;
    p.R = c.data_ptr();
  } else {
    c = at::empty({M, (int64_t)p.N}, a.options());
  }
  p.C = c.data_ptr();
  if (epi == bh::kC1x1Affine) {
    p.a_scale = fptr(a_scale, p.N, "a_scale");
    p.a_shift = fptr(a_shift, p.N, "a_shift");
    p.relu = relu;
    p.r_mul = r_mul;
  }
  if (bnb.has_value() && bnb->defined()) {
    p.bnb = fptr(bnb, 3 * (int64_t)p.K, "bnb");
    TORCH_CHECK(bnb_y.has_value() && bnb_y->defined() && bnb_y->is_cuda() && bnb_y->device() == a.device() &&
                    bnb_y->scalar_type() == a.scalar_type() && (lda ? true : bnb_y->is_contiguous()) &&
                    bnb_y->sizes() == a.sizes(),
                "conv_bn.c1x1: bnb_y must be a tensor shaped (and strided) like a, of a's dtype");
    p.bnb_y = bnb_y->data_ptr();
  }
  p.lda = (int)lda;
  if (epi == bh::kC1x1Mask) {
    TORCH_CHECK(mbits.has_value() && mbits->defined() && mbits->is_cuda() && mbits->device() == a.device() &&
                    mbits->scalar_type() == at::kByte && mbits->is_contiguous() && mbits->numel() == M * p.N / 8,
                "conv_bn.c1x1: the mask epilogue needs mbits, a contiguous uint8 [M, N/8] tensor");
    p.mbits = mbits->data_ptr<uint8_t>();
  }
  at::Tensor part;
  if (epi == bh::kC1x1Stats || epi == bh::kC1x1Bwd || epi == bh::kC1x1Mask) {
    const int G = bh::c1x1_parts(p);
    TORCH_CHECK(G > 0, "conv_bn.c1x1: unsupported shape");
    part = at::empty({2, (int64_t)G, (int64_t)p.N}, a.options().dtype(at::kFloat));
    p.part = part.data_ptr<float>();
  } else {
    part = at::empty({0}, a.options().dtype(at::kFloat));
  }
  TORCH_CHECK(bh::c1x1_supported(p), "conv_bn.c1x1: unsupported shape / alignment / argument combination (M=", M,
              ", K=", p.K, ", N=", p.N, ")");
  bh::c1x1_run(dtype_code(a.scalar_type()), p, stream_for(a));
  return {c, part};
}

bool c1x1_supported(const at::Tensor& a, const at::Tensor& b, bool b_trans, int64_t M, bool pro, bool resid,
                    int64_t s2_h, int64_t s2_w, int64_t epi, bool s2_scatter, bool bnb) {
  if (!(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() &&
        a.scalar_type() == b.scalar_type() && a.size(1) == b.size(b_trans ? 0 : 1) &&
        (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16)))
    return false;
  static float dummy[1];
  bh::C1x1Args p;
  p.A = a.data_ptr();
  p.B = b.data_ptr();
  p.C = a.data_ptr();  // alignment of the future output: at::empty is 16-byte aligned
  p.b_trans = b_trans;
  p.M = M;
  p.K = (int)a.size(1);
  p.N = (int)b.size(b_trans ? 1 : 0);
  p.pro_scale = pro ? dummy : nullptr;
  p.pro_shift = pro ? dummy : nullptr;
  p.bnb = bnb ? dummy : nullptr;
  p.bnb_y = bnb ? a.data_ptr() : nullptr;
  p.R = resid ? a.data_ptr() : nullptr;
  if (s2_scatter) p.R = p.C;
  p.s2_scatter = s2_scatter;
  p.s2_H = (int)s2_h;
  p.s2_W = (int)s2_w;
  p.epi = (int)epi;
  p.part = dummy;
  if (epi == bh::kC1x1Affine) p.a_scale = p.a_shift = dummy;
  if (epi == bh::kC1x1Bwd) {
    p.by = a.data_ptr();
    p.bscale = p.bshift = p.bmean = dummy;
  }
  if (epi == bh::kC1x1Mask) p.mbits = reinterpret_cast<const uint8_t*>(dummy);
  return bh::c1x1_supported(p);
}

// [2N+1] (count >= 0) or [2N] sums over the G partial rows of c1x1's statistics
at::Tensor sum_parts(const at::Tensor& part, double count) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 3 && part.size(0) == 2 &&
                  part.is_contiguous(),
              "conv_bn.sum_parts: part must be a contiguous fp32 [2, G, N] GPU tensor");
  const int64_t G = part.size(1), N = part.size(2);
  auto out = at::empty({2 * N + (count >= 0 ? 1 : 0)}, part.options());
  bh::c1x1_sum_parts((int)G, (int)N, part.data_ptr<float>(), out.data_ptr<float>(), (float)count, stream_for(part));
  return out;
}

// sum_parts plus the BatchNorm's fp32 parameter gradients from the same launch: (sums, gw = sums[N:] * invstd,
// gb = sums[:N] as a separate tensor -- this rank's own, the sums may be all-reduced in place afterwards)
std::vector<at::Tensor> sum_parts_grads(const at::Tensor& part, double count, const at::Tensor& invstd) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 3 && part.size(0) == 2 &&
                  part.is_contiguous(),
              "conv_bn.sum_parts: part must be a contiguous fp32 [2, G, N] GPU tensor");
  const int64_t G = part.size(1), N = part.size(2);
  TORCH_CHECK(invstd.is_cuda() && invstd.scalar_type() == at::kFloat && invstd.is_contiguous() && invstd.numel() == N,
              "conv_bn.sum_parts: invstd must be a contiguous fp32 [N] GPU tensor");
  auto out = at::empty({2 * N + (count >= 0 ? 1 : 0)}, part.options());
  auto gw = at::empty({N}, part.options()), gb = at::empty({N}, part.options());
  bh::c1x1_sum_parts((int)G, (int)N, part.data_ptr<float>(), out.data_ptr<float>(), (float)count, stream_for(part),
                     invstd.data_ptr<float>(), gw.data_ptr<float>(), gb.data_ptr<float>());
  return {out, gw, gb};
}

// C = A . B^T (+ resid) on the tiled MFMA GEMM (kernels/gemm.hip) with a BatchNorm epilogue (epi 0: none;
// 1: forward statistics centred on kshift; 2: the previous BatchNorm's backward sums with by / bscale /
// bshift / bmean) -- the compute-bound 1x1 layers. Returns (C [M, N], partials [2, slabs, N] or empty).
std::vector<at::Tensor> gemm_bn(const at::Tensor& a, const at::Tensor& b, int64_t epi,
                                const c10::optional<at::Tensor>& kshift, const c10::optional<at::Tensor>& by,
                                const c10::optional<at::Tensor>& bscale, const c10::optional<at::Tensor>& bshift,
                                const c10::optional<at::Tensor>& bmean, bool brelu,
                                const c10::optional<at::Tensor>& resid) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.device() == b.device() && a.dim() == 2 && b.dim() == 2 &&
                  a.is_contiguous() && b.is_contiguous() && a.scalar_type() == b.scalar_type() &&
                  (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16) && a.size(1) == b.size(1),
              "conv_bn.gemm_bn: a [M, K] and b [N, K] contiguous fp16/bf16 GPU tensors");
  TORCH_CHECK(epi >= 0 && epi <= 2, "conv_bn.gemm_bn: epi must be 0 (none), 1 (statistics) or 2 (backward sums)");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  auto c = at::empty({M, N}, a.options());
  TORCH_CHECK(bh::gemm_supported(M, N, K, K, K, N, a.data_ptr(), b.data_ptr(), c.data_ptr()) && N % 64 == 0,
              "conv_bn.gemm_bn: unsupported shape");
  bh::GemmEpilogue e;
  at::Tensor part;
  if (epi) {
    const int64_t slabs = bh::gemm_bgrad_slabs(M);
    part = at::empty({2, slabs, N}, a.options().dtype(at::kFloat));
    e.bn_stats = (int)epi;
    e.stat_part = part.data_ptr<float>();
    e.kshift = fptr(kshift, N, "kshift");
  }
  if (epi == 2) {
    TORCH_CHECK(by.has_value() && by->defined() && by->is_cuda() && by->scalar_type() == a.scalar_type() &&
                    by->is_contiguous() && by->numel() == M * N,
                "conv_bn.gemm_bn: by must be a contiguous [M, N] tensor of a's dtype");
    e.bn_y = by->data_ptr();
    e.bn_scale = fptr(bscale, N, "bscale");
    e.bn_shift = fptr(bshift, N, "bshift");
    e.bn_mean = fptr(bmean, N, "bmean");
    TORCH_CHECK(e.bn_scale && e.bn_shift && e.bn_mean, "conv_bn.gemm_bn: bscale / bshift / bmean required");
    e.bn_relu = brelu;
  }
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->is_cuda() && resid->scalar_type() == a.scalar_type() && resid->is_contiguous() &&
                    resid->numel() == M * N && K % 64 == 0,
                "conv_bn.gemm_bn: resid must be a contiguous [M, N] tensor of a's dtype (and K % 64 == 0)");
    e.resid = resid->data_ptr();
  }
  bh::gemm_nt(dtype_code(a.scalar_type()), a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, M, N, K, e,
              stream_for(a));
  return {c, part};
}

}  // namespace

void register_conv_bn(pybind11::module_& root) {
  auto m = root.def_submodule("conv_bn", "1x1 convolution GEMMs with BatchNorm prologue / statistics epilogues");
  m.attr("EPI_PLAIN") = (int)bh::kC1x1Plain;
  m.attr("EPI_STATS") = (int)bh::kC1x1Stats;
  m.attr("EPI_BWD") = (int)bh::kC1x1Bwd;
  m.def("c1x1", &c1x1, py::arg("a"), py::arg("b"), py::arg("b_trans"), py::arg("M"), py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("resid") = py::none(), py::arg("s2_h") = 0, py::arg("s2_w") = 0,
        py::arg("epi") = 0, py::arg("kshift") = py::none(), py::arg("by") = py::none(), py::arg("bscale") = py::none(),
        py::arg("bshift") = py::none(), py::arg("bmean") = py::none(), py::arg("brelu") = true,
        py::arg("s2_scatter") = false, py::arg("a_scale") = py::none(), py::arg("a_shift") = py::none(),
        py::arg("relu") = false, py::arg("r_mul") = false, py::arg("bnb") = py::none(), py::arg("bnb_y") = py::none(),
        py::arg("mbits") = py::none(), py::arg("lda") = 0);
  m.attr("EPI_MASK") = (int)bh::kC1x1Mask;
  m.attr("EPI_AFFINE") = (int)bh::kC1x1Affine;
  m.def("c1x1_supported", &c1x1_supported, py::arg("a"), py::arg("b"), py::arg("b_trans"), py::arg("M"), py::arg("pro") = false,
        py::arg("resid") = false, py::arg("s2_h") = 0, py::arg("s2_w") = 0, py::arg("epi") = 0,
        py::arg("s2_scatter") = false, py::arg("bnb") = false);
  m.def("sum_parts", &sum_parts, py::arg("part"), py::arg("count") = -1.0);
  m.def("sum_parts_grads", &sum_parts_grads, py::arg("part"), py::arg("count"), py::arg("invstd"));
  // x: NCHW-shaped channels_last 16-bit; returns the channels_last [n, c, h / 2, w / 2] stride-2 gather
  m.def("s2_gather", [](at::Tensor x) {
    TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0 &&
                    x.size(2) % 2 == 0 && x.size(3) % 2 == 0 && x.element_size() == 2,
                "conv_bn.s2_gather: channels_last 16-bit [n, c, h, w] with c % 8 == 0 and even h, w");
    auto q = at::empty({x.size(0), x.size(1), x.size(2) / 2, x.size(3) / 2},
                       x.options().memory_format(at::MemoryFormat::ChannelsLast));
    bh::s2_pixels(dtype_code(x.scalar_type()), x.data_ptr(), q.data_ptr(), x.size(0), (int)q.size(2), (int)q.size(3),
                  (int)x.size(1), false, stream_for(x));
    return q;
  }, py::arg("x"));
  m.def("pool_broadcast", [](at::Tensor g, int64_t h, int64_t w, double scale) {
    TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && g.size(1) % 8 == 0 && g.element_size() == 2,
                "conv_bn.pool_broadcast: contiguous 16-bit [n, c] with c % 8 == 0");
    auto out = at::empty({g.size(0), g.size(1), h, w}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
    bh::pool_bcast(dtype_code(g.scalar_type()), g.data_ptr(), out.data_ptr(), g.size(0), h * w, (int)g.size(1),
                   (float)scale, stream_for(g));
    return out;
  }, py::arg("g"), py::arg("h"), py::arg("w"), py::arg("scale"),
     "channels_last [n, c, h, w] = g[n, c] * scale: the global-average-pool backward in one vectorised pass");
  // full [n * h * w, c] (+)= quarter [n * h/2 * w/2, c] at the even pixels, in place; returns full
  m.def("s2_scatter_add", [](at::Tensor full, at::Tensor quarter, int64_t n, int64_t h, int64_t w) {
    TORCH_CHECK(full.is_cuda() && quarter.is_cuda() && full.is_contiguous() && quarter.is_contiguous() &&
                    full.scalar_type() == quarter.scalar_type() && full.element_size() == 2 && full.dim() == 2 &&
                    quarter.dim() == 2 && full.size(1) == quarter.size(1) && full.size(1) % 8 == 0 && h % 2 == 0 &&
                    w % 2 == 0 && full.size(0) == n * h * w && quarter.size(0) == n * (h / 2) * (w / 2),
                "conv_bn.s2_scatter_add: contiguous 16-bit [n*h*w, c] and [n*h/2*w/2, c], c % 8 == 0");
    bh::s2_pixels(dtype_code(full.scalar_type()), full.data_ptr(), quarter.data_ptr(), n, (int)(h / 2), (int)(w / 2),
                  (int)full.size(1), true, stream_for(full));
    return full;
  }, py::arg("full"), py::arg("quarter"), py::arg("n"), py::arg("h"), py::arg("w"));
  m.def("gemm_bn", &gemm_bn, py::arg("a"), py::arg("b"), py::arg("epi"), py::arg("kshift") = py::none(),
        py::arg("by") = py::none(), py::arg("bscale") = py::none(), py::arg("bshift") = py::none(),
        py::arg("bmean") = py::none(), py::arg("brelu") = true, py::arg("resid") = py::none());
}

}  // namespace bhb
