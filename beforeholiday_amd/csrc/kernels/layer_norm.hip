// LayerNorm / RMSNorm forward + backward for gfx950 (fused_layer_norm_cuda equivalent).
//
// Reference behaviour: csrc/layer_norm_cuda_kernel.cu (cuWelfordMuSigma2 :70/:180, cuApplyLayerNorm
// :362-447, cuComputePartGradGammaBeta :549, cuComputeGradGammaBeta :626, cuComputeGradInput :687;
// hosts HostApplyLayerNorm :876, HostApplyRMSNorm :908, HostLayerNormGradient :996,
// HostRMSNormGradient :1083).
//
// MI355X design:
//  * one wave64 per row: the whole row lives in registers (8 elements / lane / vector, 16-byte
//    loads), so mean and variance are an exact two-pass computation with two wave reductions and
//    the row is read from HBM exactly once (rows up to 8192 elements; longer rows use a
//    block-per-row streaming kernel).
//  * backward dx is the same wave-per-row structure (dy and x read once); the parameter gradients
//    are a column reduction over rows done like the channels_last BN reduce: a thread owns 8
//    contiguous columns, per-(split, column) partials, then a tiny finalize. Deterministic.
//  * memory_efficient: x_hat is recomputed from the saved OUTPUT ((y - beta) / gamma) instead of the
//    input, so the input need not be kept alive (reference semantics).
#include "bh/api.h"
#include "bh/device.h"
#include "bh/ln_api.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;
constexpr int kRowsPerBlock = kBlock / kWave;

#define LN_DISPATCH(code, T, ...)                                         \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    default: throw std::runtime_error("layer_norm: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
BH_DEVICE void load8(const T* p, int col, int n2, bool vec, float (&r)[8]) {
  if (vec && col + 8 <= n2) {
    VecIO<T>::load(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = (col + k < n2) ? to_f<T>(p[col + k]) : 0.f;
  }
}
template <typename T>
BH_DEVICE void store8(T* p, int col, int n2, bool vec, const float (&r)[8]) {
  if (vec && col + 8 <= n2) {
    VecIO<T>::store(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (col + k < n2) p[col + k] = from_f<T>(r[k]);
  }
}

// ------------------------------------------------------------------------------------------
// forward, one wave per row, VPT 8-element vectors per lane
// ------------------------------------------------------------------------------------------
template <typename T, typename Tw, typename Ty, int VPT, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_fwd(const T* __restrict__ x, const Tw* __restrict__ g,
                                                   const Tw* __restrict__ b, Ty* __restrict__ y,
                                                   float* __restrict__ mean_out, float* __restrict__ invvar_out,
                                                   int64_t n1, int n2, float eps, bool vec) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= n1) return;
  const T* xr = x + row * n2;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    load8(xr, (j * kWave + lane) * 8, n2, vec, v[j]);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[j][k];
  }
  const float inv_n = 1.f / (float)n2;
  const float mean = RMS ? 0.f : wave_sum(s) * inv_n;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int col = (j * kWave + lane) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = (col + k < n2) ? v[j][k] - mean : 0.f;
      q = fmaf(d, d, q);
    }
  }
  const float invvar = rsqrtf(wave_sum(q) * inv_n + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    invvar_out[row] = invvar;
  }
  Ty* yr = y + row * n2;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int col = (j * kWave + lane) * 8;
    if (col >= n2) break;
    float gv[8], bv[8], o[8];
    if (g) load8(g, col, n2, vec, gv);
    if (b && !RMS) load8(b, col, n2, vec, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = (v[j][k] - mean) * invvar;
      if (g) t *= gv[k];
      if (b && !RMS) t += bv[k];
      o[k] = t;
    }
    store8(yr, col, n2, vec, o);
  }
}

// block per row for long rows: pass 1 sums, pass 2 centred squares, pass 3 normalise
template <typename T, typename Tw, typename Ty, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_fwd_long(const T* __restrict__ x, const Tw* __restrict__ g,
                                                        const Tw* __restrict__ b, Ty* __restrict__ y,
                                                        float* __restrict__ mean_out, float* __restrict__ invvar_out,
                                                        int n2, float eps) {
  __shared__ float red[kBlock / kWave];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * n2;
  float s = 0.f;
  if (!RMS)
    for (int i = threadIdx.x; i < n2; i += kBlock) s += to_f<T>(xr[i]);
  const float mean = RMS ? 0.f : block_sum(s, red) / (float)n2;
  float q = 0.f;
  for (int i = threadIdx.x; i < n2; i += kBlock) {
    const float d = to_f<T>(xr[i]) - mean;
    q = fmaf(d, d, q);
  }
  const float invvar = rsqrtf(block_sum(q, red) / (float)n2 + eps);
  if (threadIdx.x == 0) {
    if (!RMS) mean_out[row] = mean;
    invvar_out[row] = invvar;
  }
  Ty* yr = y + row * n2;
  for (int i = threadIdx.x; i < n2; i += kBlock) {
    float t = (to_f<T>(xr[i]) - mean) * invvar;
    if (g) t *= to_f<Tw>(g[i]);
    if (b && !RMS) t += to_f<Tw>(b[i]);
    yr[i] = from_f<Ty>(t);
  }
}

// ------------------------------------------------------------------------------------------
// backward dx, one wave per row.  x_hat from x (mean/invvar) or, memory-efficient, from y.
//   LN:  dx = invvar * (dyg - mean(dyg) - xhat * mean(dyg * xhat)),  dyg = dy * gamma
//   RMS: dx = invvar * (dyg - xhat * mean(dyg * xhat))
// ------------------------------------------------------------------------------------------
template <typename T, typename Tw, typename Tdy, int VPT, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_bwd_dx(const Tdy* __restrict__ dy, const T* __restrict__ xin,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ invvar_in, const Tw* __restrict__ g,
                                                      const Tw* __restrict__ b, T* __restrict__ dx, int64_t n1, int n2,
                                                      bool from_output, bool vec, const T* __restrict__ dres) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= n1) return;
  const float mean = (RMS || from_output) ? 0.f : mean_in[row];  // memory-efficient: mean not saved
  const float invvar = invvar_in[row];
  float xh[VPT][8], dg[VPT][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int col = (j * kWave + lane) * 8;
    float dv[8], xv[8], gv[8], bv[8];
    load8(dy + row * n2, col, n2, vec, dv);
    load8(xin + row * n2, col, n2, vec, xv);
    if (g) load8(g, col, n2, vec, gv);
    if (from_output && b && !RMS) load8(b, col, n2, vec, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gg = g ? gv[k] : 1.f;
      float h;
      if (from_output) {
        float yv = xv[k];
        if (b && !RMS) yv -= bv[k];
        h = (gg != 0.f) ? yv / gg : 0.f;
      } else {
        h = (xv[k] - mean) * invvar;
      }
      const bool ok = col + k < n2;
      xh[j][k] = ok ? h : 0.f;
      dg[j][k] = ok ? dv[k] * gg : 0.f;
      s1 += dg[j][k];
      s2 = fmaf(dg[j][k], xh[j][k], s2);
    }
  }
  const float inv_n = 1.f / (float)n2;
  const float m1 = RMS ? 0.f : wave_sum(s1) * inv_n;
  const float m2 = wave_sum(s2) * inv_n;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int col = (j * kWave + lane) * 8;
    if (col >= n2) break;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = invvar * (dg[j][k] - m1 - xh[j][k] * m2);
    if (dres) {  // + the residual branch's gradient of the same input, one rounding
      float rv[8];
      load8(dres + row * n2, col, n2, vec, rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] += rv[k];
    }
    store8(dx + row * n2, col, n2, vec, o);
  }
}

// backward dx AND the parameter-gradient partials in one pass: every wave walks rows blockIdx.x * 4 + wave,
// + 4 gridDim.x, ... with the same per-row math as k_ln_bwd_dx, and keeps dy * x_hat and dy for its lane's
// columns in registers; the block sums its four waves through LDS into ONE partial row (pg[block][n2],
// pb[block][n2]) for k_ln_wgrad_finalize. dy and x are read once for dx and the gradients together (the
// separate k_ln_wgrad_partials pass re-read both).
template <typename T, typename Tw, typename Tdy, int VPT, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_bwd_fused(const Tdy* __restrict__ dy, const T* __restrict__ xin,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ invvar_in, const Tw* __restrict__ g,
                                                         const Tw* __restrict__ b, T* __restrict__ dx, int64_t n1,
                                                         int n2, bool from_output, bool vec,
                                                         const T* __restrict__ dres, float* __restrict__ pg,
                                                         float* __restrict__ pb) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [waves][2][VPT * 512]
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  constexpr int kCols = VPT * kWave * 8;
  float ag[VPT][8], ab[VPT][8], gv[VPT][8], bv[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int col = (j * kWave + lane) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[j][k] = ab[j][k] = 0.f;
    if (g) load8(g, col, n2, vec, gv[j]);
    else
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[j][k] = 1.f;
    if (from_output && b && !RMS) load8(b, col, n2, vec, bv[j]);
  }
  const float inv_n = 1.f / (float)n2;
  // software-pipelined over the wave's rows: the next row's dy, x, residual gradient and statistics are
  // requested (clamped row: unconditional loads) before this row's math, so each wave keeps two rows of
  // loads in flight instead of two dependent round trips per row (one wave per SIMD: latency bound)
  const int64_t stride = (int64_t)gridDim.x * kRowsPerBlock;
  float dvA[VPT][8], xvA[VPT][8], rvA[VPT][8], meanA = 0.f, invA = 0.f;
  auto load_row = [&](int64_t r, float (&dv)[VPT][8], float (&xv)[VPT][8], float (&rv)[VPT][8], float& mean,
                      float& invvar) __attribute__((always_inline)) {
    mean = (RMS || from_output) ? 0.f : mean_in[r];
    invvar = invvar_in[r];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int col = (j * kWave + lane) * 8;
      load8(dy + r * n2, col, n2, vec, dv[j]);
      load8(xin + r * n2, col, n2, vec, xv[j]);
      if (dres) load8(dres + r * n2, col, n2, vec, rv[j]);
    }
  };
  int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + wave;
  if (row < n1) load_row(row, dvA, xvA, rvA, meanA, invA);
  for (; row < n1; row += stride) {
    float dvB[VPT][8], xvB[VPT][8], rvB[VPT][8], meanB, invB;
    load_row(min(row + stride, n1 - 1), dvB, xvB, rvB, meanB, invB);
    const float mean = meanA, invvar = invA;
    float xh[VPT][8], dg[VPT][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int col = (j * kWave + lane) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gg = gv[j][k];
        float h;
        if (from_output) {
          const float yv = (b && !RMS) ? xvA[j][k] - bv[j][k] : xvA[j][k];
          h = (gg != 0.f) ? yv / gg : 0.f;
        } else {
          h = (xvA[j][k] - mean) * invvar;
        }
        const bool ok = col + k < n2;
        xh[j][k] = ok ? h : 0.f;
        const float d = ok ? dvA[j][k] : 0.f;
        dg[j][k] = d * gg;
        ag[j][k] = fmaf(d, xh[j][k], ag[j][k]);
        ab[j][k] += d;
        s1 += dg[j][k];
        s2 = fmaf(dg[j][k], xh[j][k], s2);
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) * inv_n;
    const float m2 = wave_sum(s2) * inv_n;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int col = (j * kWave + lane) * 8;
      if (col >= n2) break;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = invvar * (dg[j][k] - m1 - xh[j][k] * m2) + (dres ? rvA[j][k] : 0.f);
      store8(dx + row * n2, col, n2, vec, o);
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dvA[j][k] = dvB[j][k];
        xvA[j][k] = xvB[j][k];
        rvA[j][k] = rvB[j][k];
      }
    meanA = meanB;
    invA = invB;
  }
  // the block's four waves -> one partial row (fixed order: deterministic)
  float* mine = red + (size_t)wave * 2 * kCols;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mine[(j * kWave + lane) * 8 + k] = ag[j][k];
      mine[kCols + (j * kWave + lane) * 8 + k] = ab[j][k];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < n2; c += kBlock) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < kRowsPerBlock; ++w) {
      sg += red[(size_t)w * 2 * kCols + c];
      sb += red[(size_t)w * 2 * kCols + kCols + c];
    }
    pg[(int64_t)blockIdx.x * n2 + c] = sg;
    pb[(int64_t)blockIdx.x * n2 + c] = sb;
  }
}

template <typename T, typename Tw, typename Tdy, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_bwd_dx_long(const Tdy* __restrict__ dy, const T* __restrict__ xin,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ invvar_in,
                                                           const Tw* __restrict__ g, const Tw* __restrict__ b,
                                                           T* __restrict__ dx, int n2, bool from_output,
                                                           const T* __restrict__ dres) {
  __shared__ float red[kBlock / kWave];
  const int64_t row = blockIdx.x;
  const float mean = (RMS || from_output) ? 0.f : mean_in[row];  // memory-efficient: mean not saved
  const float invvar = invvar_in[row];
  auto xhat = [&](int i) -> float {
    const float xv = to_f<T>(xin[row * n2 + i]);
    if (from_output) {
      const float gg = g ? to_f<Tw>(g[i]) : 1.f;
      const float yv = (b && !RMS) ? xv - to_f<Tw>(b[i]) : xv;
      return gg != 0.f ? yv / gg : 0.f;
    }
    return (xv - mean) * invvar;
  };
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n2; i += kBlock) {
    const float dgv = to_f<Tdy>(dy[row * n2 + i]) * (g ? to_f<Tw>(g[i]) : 1.f);
    s1 += dgv;
    s2 = fmaf(dgv, xhat(i), s2);
  }
  const float m1 = RMS ? 0.f : block_sum(s1, red) / (float)n2;
  const float m2 = block_sum(s2, red) / (float)n2;
  for (int i = threadIdx.x; i < n2; i += kBlock) {
    const float dgv = to_f<Tdy>(dy[row * n2 + i]) * (g ? to_f<Tw>(g[i]) : 1.f);
    const float rv = dres ? to_f<T>(dres[row * n2 + i]) : 0.f;
    dx[row * n2 + i] = from_f<T>(invvar * (dgv - m1 - xhat(i) * m2) + rv);
  }
}

// ------------------------------------------------------------------------------------------
// gamma/beta gradients: column reduction. grid (column tiles of 8*cvb, splits)
//   pg[s][n2] = sum_rows dy * xhat, pb[s][n2] = sum_rows dy
// ------------------------------------------------------------------------------------------
template <typename T, typename Tw, typename Tdy, bool RMS>
__global__ __launch_bounds__(kBlock) void k_ln_wgrad_partials(const Tdy* __restrict__ dy, const T* __restrict__ xin,
                                                              const float* __restrict__ mean_in,
                                                              const float* __restrict__ invvar_in,
                                                              const Tw* __restrict__ g, const Tw* __restrict__ b,
                                                              int64_t n1, int n2, int cvb, int R, int64_t rows_per_split,
                                                              bool from_output, bool vec, float* __restrict__ pg,
                                                              float* __restrict__ pb) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int v = threadIdx.x % cvb, r = threadIdx.x / cvb;
  const int c0 = (blockIdx.x * cvb + v) * 8;
  const int split = blockIdx.y;
  const int64_t row0 = (int64_t)split * rows_per_split;
  const int64_t row1 = min(n1, row0 + rows_per_split);
  float ag[8], ab[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) ag[k] = ab[k] = 0.f;
  const bool active = (r < R) && (c0 < n2);
  if (active) {
    float gv[8], bv[8];
    if (from_output) {
      if (g) load8(g, c0, n2, vec, gv);
      if (b && !RMS) load8(b, c0, n2, vec, bv);
    }
    auto body = [&](const float (&dv)[8], const float (&xv)[8], float mean, float invvar) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float h;
        if (from_output) {
          const float gg = g ? gv[k] : 1.f;
          const float yv = (b && !RMS) ? xv[k] - bv[k] : xv[k];
          h = gg != 0.f ? yv / gg : 0.f;
        } else {
          h = (xv[k] - mean) * invvar;
        }
        ag[k] = fmaf(dv[k], h, ag[k]);
        ab[k] += dv[k];
      }
    };
    // 4 rows of dy / x loads in flight per lane before any arithmetic
    int64_t row = row0 + r;
    for (; row + 3 * (int64_t)R < row1; row += 4 * (int64_t)R) {
      float dv[4][8], xv[4][8], mu[4], iv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t rr = row + u * (int64_t)R;
        load8(dy + rr * n2, c0, n2, vec, dv[u]);
        load8(xin + rr * n2, c0, n2, vec, xv[u]);
        mu[u] = (RMS || from_output) ? 0.f : mean_in[rr];
        iv[u] = from_output ? 0.f : invvar_in[rr];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) body(dv[u], xv[u], mu[u], iv[u]);
    }
    for (; row < row1; row += R) {
      float dv[8], xv[8];
      load8(dy + row * n2, c0, n2, vec, dv);
      load8(xin + row * n2, c0, n2, vec, xv);
      body(dv, xv, (RMS || from_output) ? 0.f : mean_in[row], from_output ? 0.f : invvar_in[row]);
    }
  }
  float* sa = smem;
  float* sb = smem + R * cvb * 8;
  if (r < R) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sa[(r * cvb + v) * 8 + k] = ag[k];
      sb[(r * cvb + v) * 8 + k] = ab[k];
    }
  }
  __syncthreads();
  for (int s = R / 2; s > 0; s >>= 1) {
    if (r < s) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sa[(r * cvb + v) * 8 + k] += sa[((r + s) * cvb + v) * 8 + k];
        sb[(r * cvb + v) * 8 + k] += sb[((r + s) * cvb + v) * 8 + k];
      }
    }
    __syncthreads();
  }
  if (r == 0 && c0 < n2) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (c0 + k < n2) {
        pg[(int64_t)split * n2 + c0 + k] = sa[v * 8 + k];
        pb[(int64_t)split * n2 + c0 + k] = sb[v * 8 + k];
      }
    }
  }
}

template <typename Tw>
__global__ __launch_bounds__(64 * kColsumLanes) void k_ln_wgrad_finalize(int n2, int splits, const float* __restrict__ pg,
                                                                          const float* __restrict__ pb,
                                                                          Tw* __restrict__ gg, Tw* __restrict__ gb) {
  __shared__ float sh[kColsumLanes][64];
  colsum_partials_block<Tw>(pg, splits, n2, gg, sh);
  colsum_partials_block<Tw>(pb, splits, n2, gb, sh);
}

// vectors per lane for the wave-per-row kernels; 0 selects the block-per-row kernel. The backward
// keeps two row copies (x_hat and dy*gamma) in registers, so it caps at 8 (rows <= 4096).
int vpt_for(int n2, int max_vpt) {
  const int vecs = (n2 + 8 * kWave - 1) / (8 * kWave);
  int v = 1;
  while (v < vecs) v *= 2;
  return v <= max_vpt ? v : 0;
}

#define LN_VPT_DISPATCH(vpt, V, ...)                  \
  switch (vpt) {                                       \
    case 1: { constexpr int V = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int V = 2; __VA_ARGS__; } break; \
    case 4: { constexpr int V = 4; __VA_ARGS__; } break; \
    case 8: { constexpr int V = 8; __VA_ARGS__; } break; \
    case 16: { constexpr int V = 16; __VA_ARGS__; } break; \
    default: break;                                    \
  }
// the fused backward keeps ~10 register rows: rows of <= 2048 columns (vpt <= 4, ln_bwd_fused_blocks)
#define LN_VPT4_DISPATCH(vpt, V, ...)                 \
  switch (vpt) {                                       \
    case 1: { constexpr int V = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int V = 2; __VA_ARGS__; } break; \
    case 4: { constexpr int V = 4; __VA_ARGS__; } break; \
    default: break;                                    \
  }

}  // namespace

void ln_forward(int64_t n1, int n2, int dt_x, const void* x, int dt_w, const void* gamma, const void* beta,
                int dt_y, void* y, float* mean, float* invvar, float eps, bool rms, bool vec, hipStream_t st) {
  if (n1 == 0 || n2 == 0) return;
  if (dt_w < 0) dt_w = dt_x;
  const int vpt = vpt_for(n2, 16);
  const int grid = (int)((n1 + kRowsPerBlock - 1) / kRowsPerBlock);
  LN_DISPATCH(dt_x, T, LN_DISPATCH(dt_w, Tw, LN_DISPATCH(dt_y, Ty,
      if (vpt) {
        LN_VPT_DISPATCH(vpt, V,
            if (rms) hipLaunchKernelGGL((k_ln_fwd<T, Tw, Ty, V, true>), dim3(grid), dim3(kBlock), 0, st, (const T*)x,
                                        (const Tw*)gamma, (const Tw*)beta, (Ty*)y, mean, invvar, n1, n2, eps, vec);
            else hipLaunchKernelGGL((k_ln_fwd<T, Tw, Ty, V, false>), dim3(grid), dim3(kBlock), 0, st, (const T*)x,
                                    (const Tw*)gamma, (const Tw*)beta, (Ty*)y, mean, invvar, n1, n2, eps, vec));
      } else {
        if (rms) hipLaunchKernelGGL((k_ln_fwd_long<T, Tw, Ty, true>), dim3(n1), dim3(kBlock), 0, st, (const T*)x,
                                    (const Tw*)gamma, (const Tw*)beta, (Ty*)y, mean, invvar, n2, eps);
        else hipLaunchKernelGGL((k_ln_fwd_long<T, Tw, Ty, false>), dim3(n1), dim3(kBlock), 0, st, (const T*)x,
                                (const Tw*)gamma, (const Tw*)beta, (Ty*)y, mean, invvar, n2, eps);
      })));
  check_launch("ln_forward");
}

void ln_backward_dx(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                    const float* invvar, int dt_w, const void* gamma, const void* beta, void* dx, bool rms,
                    bool from_output, bool vec, hipStream_t st, const void* dresid) {
  if (n1 == 0 || n2 == 0) return;
  if (dt_w < 0) dt_w = dt_x;
  const int vpt = vpt_for(n2, 4);
  const int grid = (int)((n1 + kRowsPerBlock - 1) / kRowsPerBlock);
  LN_DISPATCH(dt_x, T, LN_DISPATCH(dt_w, Tw, LN_DISPATCH(dt_dy, Tdy,
      if (vpt) {
        LN_VPT_DISPATCH(vpt, V,
            if (rms) hipLaunchKernelGGL((k_ln_bwd_dx<T, Tw, Tdy, V, true>), dim3(grid), dim3(kBlock), 0, st,
                                        (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma,
                                        (const Tw*)beta, (T*)dx, n1, n2, from_output, vec, (const T*)dresid);
            else hipLaunchKernelGGL((k_ln_bwd_dx<T, Tw, Tdy, V, false>), dim3(grid), dim3(kBlock), 0, st,
                                    (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta,
                                    (T*)dx, n1, n2, from_output, vec, (const T*)dresid));
      } else {
        if (rms) hipLaunchKernelGGL((k_ln_bwd_dx_long<T, Tw, Tdy, true>), dim3(n1), dim3(kBlock), 0, st,
                                    (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta,
                                    (T*)dx, n2, from_output, (const T*)dresid);
        else hipLaunchKernelGGL((k_ln_bwd_dx_long<T, Tw, Tdy, false>), dim3(n1), dim3(kBlock), 0, st,
                                (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta,
                                (T*)dx, n2, from_output, (const T*)dresid);
      })));
  check_launch("ln_backward_dx");
}

int ln_bwd_fused_blocks(int64_t n1, int n2) {
  // wave-per-row rows only (x_hat and dy * gamma in registers, <= 2048 columns), >= 8 rows per wave, and
  // about one block per CU: 256 partial rows for the finalize
  if (n2 > 2048 || vpt_for(n2, 4) == 0) return 0;
  const int64_t by_rows = n1 / (8 * kRowsPerBlock);
  return (int)std::max<int64_t>(1, std::min<int64_t>(256, by_rows));
}

void ln_backward_fused(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                       const float* invvar, int dt_w, const void* gamma, const void* beta, void* dx, void* grad_gamma,
                       void* grad_beta, float* partials, int blocks, bool rms, bool from_output, bool vec,
                       hipStream_t st, const void* dresid) {
  if (n1 == 0 || n2 == 0) return;
  if (dt_w < 0) dt_w = dt_x;
  const int vpt = vpt_for(n2, 4);
  if (!vpt || blocks < 1) throw std::runtime_error("ln_backward_fused: row too long");
  float* pg = partials;
  float* pb = partials + (int64_t)blocks * n2;
  const size_t shm = sizeof(float) * kRowsPerBlock * 2 * vpt * kWave * 8;
  LN_DISPATCH(dt_x, T, LN_DISPATCH(dt_w, Tw, LN_DISPATCH(dt_dy, Tdy,
      LN_VPT4_DISPATCH(vpt, V,
          if (rms) hipLaunchKernelGGL((k_ln_bwd_fused<T, Tw, Tdy, V, true>), dim3(blocks), dim3(kBlock), shm, st,
                                      (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta,
                                      (T*)dx, n1, n2, from_output, vec, (const T*)dresid, pg, pb);
          else hipLaunchKernelGGL((k_ln_bwd_fused<T, Tw, Tdy, V, false>), dim3(blocks), dim3(kBlock), shm, st,
                                  (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta,
                                  (T*)dx, n1, n2, from_output, vec, (const T*)dresid, pg, pb));
      hipLaunchKernelGGL((k_ln_wgrad_finalize<Tw>), dim3((n2 + 63) / 64), dim3(64 * kColsumLanes), 0, st, n2, blocks,
                         pg, pb, (Tw*)grad_gamma, (Tw*)grad_beta))));
  check_launch("ln_backward_fused");
}

int ln_wgrad_splits(int64_t n1, int n2) {
  const int cv = (n2 + 7) / 8;
  const int cvb = std::min(cv, kBlock);
  int R = kBlock / cvb, p = 1;
  while (p * 2 <= R) p *= 2;
  const int gx = (cv + cvb - 1) / cvb;
  // >= 8 rows per row lane (16 -> 8 took the 8192 x 1024 fp16 backward from 85 to 66 us,
  // benchmarks/bench_ln_bwd.py; profiles/ln_bwd_wgrad_split_sweep.txt) and ~512 workgroups
  constexpr int rows_min = 8, target = 512;
  int64_t splits = std::max<int64_t>(1, target / gx);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, n1 / (p * rows_min)));
  return (int)splits;
}

void ln_backward_wgrad(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                       const float* invvar, int dt_w, const void* gamma, const void* beta, void* grad_gamma,
                       void* grad_beta, float* partials, int splits, bool rms, bool from_output, bool vec,
                       hipStream_t st) {
  if (n2 == 0) return;
  if (dt_w < 0) dt_w = dt_x;
  const int cv = (n2 + 7) / 8;
  const int cvb = std::min(cv, kBlock);
  int R = kBlock / cvb, p = 1;
  while (p * 2 <= R) p *= 2;
  R = p;
  const int gx = (cv + cvb - 1) / cvb;
  const int64_t rps = (n1 + splits - 1) / splits;
  const size_t shm = sizeof(float) * 2 * R * cvb * 8;
  float* pg = partials;
  float* pb = partials + (int64_t)splits * n2;
  LN_DISPATCH(dt_x, T, LN_DISPATCH(dt_w, Tw, LN_DISPATCH(dt_dy, Tdy,
      if (rms) hipLaunchKernelGGL((k_ln_wgrad_partials<T, Tw, Tdy, true>), dim3(gx, splits), dim3(kBlock), shm, st,
                                  (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta, n1,
                                  n2, cvb, R, rps, from_output, vec, pg, pb);
      else hipLaunchKernelGGL((k_ln_wgrad_partials<T, Tw, Tdy, false>), dim3(gx, splits), dim3(kBlock), shm, st,
                              (const Tdy*)dy, (const T*)xin, mean, invvar, (const Tw*)gamma, (const Tw*)beta, n1, n2,
                              cvb, R, rps, from_output, vec, pg, pb);
      hipLaunchKernelGGL((k_ln_wgrad_finalize<Tw>), dim3((n2 + 63) / 64), dim3(64 * kColsumLanes), 0, st, n2, splits,
                         pg, pb, (Tw*)grad_gamma, (Tw*)grad_beta))));
  check_launch("ln_backward_wgrad");
}

}  // namespace bh
