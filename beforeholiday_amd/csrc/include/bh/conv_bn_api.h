// 1x1 convolution GEMMs with BatchNorm folded into their prologue / epilogue (kernels/conv_bn.hip).
//
// C[M, N] = f(A)[M, K] . B[N, K]^T on NHWC activations viewed as [pixels, channels], fp32 accumulation:
//   * prologue (pro_scale != null): f(a) = relu(a * pro_scale[k] + pro_shift[k]) -- the BatchNorm(+ReLU)
//     of the producing layer applied while the operand is loaded, so the normalised activation is never
//     written to HBM; or (bnb != null) the BatchNorm-backward prologue f(a) = A[k] a + B[k] y + D[k];
//   * stride-2 gather (s2_H > 0): output row (n, y, x) reads input row (n, 2y, 2x) of an [N, s2_H, s2_W, K]
//     tensor (the ResNet downsample branch), no gathered copy;
//   * epilogue, optional residual R[M, N] added before rounding;
//   * epilogue statistics, per output column over the rows (deterministic per-workgroup partials,
//     part[g][n] and part[G + g][n], g < G = c1x1_parts()):
//       kStats: sums of (c - kshift[n]) and (c - kshift[n])^2 of the ROUNDED stored value c -- the
//               BatchNorm statistics of this conv's output, centred on the running mean;
//       kBwd:   with y = by[m, n] (the raw input of the previous BatchNorm), mask = (y * bscale[n] +
//               bshift[n] > 0) when brelu: sums of dz = c * mask and dz * (y - bmean[n]) -- that
//               BatchNorm's backward reduction, computed on the data gradient as it is produced.
//       kMask:  c = c * bit(m, n) of the saved ReLU bit mask mbits [M, N/8] (bit n % 8 of byte n / 8) and
//               sums of the masked c (second statistic zero) -- the gradient through a residual block's
//               BatchNorm + add + ReLU output, masked where it is produced (models/resnet.py _ConvBNResFn).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

enum C1x1Epi { kC1x1Plain = 0, kC1x1Stats = 1, kC1x1Bwd = 2, kC1x1Affine = 3, kC1x1Mask = 4 };

struct C1x1Args {
  const void* A = nullptr;  // [rows, K] (rows = M, or N * s2_H * s2_W with the stride-2 gather)
  const void* B = nullptr;  // [N, K], or [K, N] with b_trans
  bool b_trans = false;
  void* C = nullptr;        // [M, N]
  const void* R = nullptr;  // optional residual [M, N]
  int64_t M = 0;
  int K = 0, N = 0;
  const float* pro_scale = nullptr;  // [K] prologue BatchNorm (with ReLU)
  const float* pro_shift = nullptr;
  // BatchNorm-backward prologue (instead of pro_scale / pro_shift): f(a) = A[k] a + B[k] bnb_y + D[k], with
  // bnb = [A (K), B (K), D (K)] fp32 and bnb_y [M, K] -- the data gradient of a convolution whose output y
  // went through a training BatchNorm, formed per fragment from the BatchNorm's output gradient a and its
  // input y (kernels/bn_fold.hip: the BatchNorm input gradient is never written)
  const float* bnb = nullptr;
  const void* bnb_y = nullptr;
  const uint8_t* mbits = nullptr;  // kMask: [M, N/8] ReLU bit mask (N % 32 == 0, 4-byte aligned)
  // row stride (elements) of A and bnb_y when they are a K-column slice of wider rows (0: K). The split-K
  // data gradient runs the BatchNorm-backward prologue over column ranges of a wider gradient.
  int lda = 0;
  int s2_H = 0, s2_W = 0;  // > 0: stride-2 gather from an [.., s2_H, s2_W, K] input; output is [.., s2_H/2, s2_W/2, N]
  // with s2_H > 0: scatter instead -- row (n, y, x) of the [M, N] result is ADDED into row (n, 2y, 2x) of
  // the full-resolution C [.., s2_H, s2_W, N] (R must equal C): the data gradient of a 1x1 / stride-2
  // convolution accumulated onto the other branch's gradient of the same input
  bool s2_scatter = false;
  int epi = kC1x1Plain;
  float* part = nullptr;            // [2][G][N] fp32 partials (kStats / kBwd)
  const float* kshift = nullptr;    // kStats centre per column (may be null = 0)
  const void* by = nullptr;         // kBwd: [M, N] raw input of the previous BatchNorm
  const float* bscale = nullptr;    // kBwd: its scale / shift (ReLU mask) and batch mean
  const float* bshift = nullptr;
  const float* bmean = nullptr;
  bool brelu = true;
  // kC1x1Affine: c = relu?(acc * a_scale[n] + a_shift[n] (+ R)) (* R when r_mul) -- conv + bias / frozen
  // BatchNorm (+ residual) (+ ReLU) (x mask) in one pass (contrib conv_bias_relu / bottleneck)
  const float* a_scale = nullptr;
  const float* a_shift = nullptr;
  bool relu = false;
  bool r_mul = false;
  // A-operand loads: 0 nontemporal (streaming hint), 1 ordinary cached loads (set by c1x1_run from
  // BH_C1X1_ALOAD when left at -1)
  int a_load = -1;
};

// whether the kernel covers the shape (K % 64, N % 64, M % 32, LDS budget, 16-byte alignment)
bool c1x1_supported(const C1x1Args& a);
// number of partial rows G per statistic for this shape (part holds 2 * G * N floats)
int c1x1_parts(const C1x1Args& a);
void c1x1_run(int dt, const C1x1Args& a, hipStream_t st);

// sums[n] = sum_g part[g][n], sums[N + n] = sum_g part[G + g][n], sums[2N] = count (if count >= 0):
// the [2N+1] layout of syncbn.stats_local_sums (forward) or [2N] (sum_dy, sum_dy_xmu) (backward)
void c1x1_sum_parts(int G, int N, const float* part, float* sums, float count, hipStream_t st,
                    const float* invstd = nullptr, float* gw = nullptr, float* gb = nullptr);

// stride-2 pixels of an NHWC tensor full [n, 2 ho, 2 wo, c] <-> quarter [n, ho, wo, c] (16-bit, c % 8 == 0):
// add = false: quarter = full[:, ::2, ::2]; add = true: full[:, ::2, ::2] += quarter
void s2_pixels(int dt, void* full, void* quarter, int64_t n, int ho, int wo, int c, bool add, hipStream_t st);

// out (channels_last [n, c, h, w], 16-bit) = g [n, c] * scale broadcast over the hw pixels (c % 8 == 0)
void pool_bcast(int dt, const void* g, void* out, int64_t n, int64_t hw, int c, float scale, hipStream_t st);

}  // namespace bh
