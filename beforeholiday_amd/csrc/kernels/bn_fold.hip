// Kernels of the BatchNorm-backward fold (bh/bn_fold_api.h): the Gram matrix of a convolution input
// with an optional BatchNorm + ReLU prologue, and the residual-ReLU mask applied to an output gradient
// with its column sums.
#include "bh/api.h"
#include "bh/bn_fold_api.h"
#include "bh/device.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));

template <typename T> struct Mf;
template <> struct Mf<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mf<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 256;
constexpr int kGramTargetWG = 512;  // two workgroups per CU

// ------------------------------------------------------------------------------------------------
// Gram partials. Workgroup = (channel block pair (jb, kb) of BJ x BJ outputs, row split). Per RM-row chunk
// a staging thread loads an 8 x 8 (rows x channels) block with eight 16-byte loads, applies the prologue and
// writes it TRANSPOSED into LDS ([channel][row]) as eight 16-byte stores (one per channel: its 8 rows), so
// both MFMA operands -- rows of a^T -- are contiguous 16-byte reads: C[i][j] += sum_m aT_J[i][m] aT_K[j][m].
// A wave owns (BJ/64)^2 32x32 output tiles. The next chunk's blocks are loaded while the current one is
// multiplied. Row ranges per split are contiguous and summed in order, the splits reduced by the caller in
// a fixed order: deterministic. Diagonal workgroups (jb == kb) also sum their channels (the column sums
// of a'). Rows past M are loaded clamped and zeroed by a select (no divergent branches).
// ONE: K == BJ (a single, diagonal block pair: one slice to stage), else two slices. Rows per chunk such
// that every one of the 256 threads stages exactly one 8x8 block per chunk.
template <int BJ, bool ONE> struct GramGeo {
  static constexpr int RM = (ONE ? 16384 : 8192) / BJ;
  static constexpr int PITCH = (RM + 8) * 2;       // bytes per channel row (16-byte aligned, staggered banks)
  static constexpr int ITEMS = (BJ / 8) * (RM / 8);  // 8x8 blocks per slice
};

// s2_H > 0: row m of the [M, K] problem is pixel (n, 2y, 2x) of an [.., s2_H, s2_W, K] input (the 1x1 / stride-2
// downsample convolution's input, read in place)
template <typename T, bool PRO, int BJ, bool ONE>
__global__ __launch_bounds__(kThreads, 2) void k_gram(const T* __restrict__ a, int64_t M, int K,
                                                      const float* __restrict__ pro_scale,
                                                      const float* __restrict__ pro_shift, int splits,
                                                      float* __restrict__ gram_part, float* __restrict__ colsum_part,
                                                      int s2_H, int s2_W) {
  using G = GramGeo<BJ, ONE>;
  constexpr int RM = G::RM, PITCH = G::PITCH, ITEMS = G::ITEMS;
  constexpr int IPT = ((ONE ? 1 : 2) * ITEMS + kThreads - 1) / kThreads;  // staging items per thread
  static_assert(IPT == 1, "one 8x8 block per thread and chunk");
  constexpr int TPW = BJ / 64;                                 // 32-wide tiles per wave per dimension
  __shared__ __attribute__((aligned(16))) char img[ONE ? 1 : 2][BJ * PITCH];

  const int nb = K / BJ;
  const int pair = blockIdx.x % (nb * nb), split = blockIdx.x / (nb * nb);
  const int jb = pair / nb, kb = pair % nb;
  const bool diag = jb == kb;
  const int nitems = diag ? ITEMS : 2 * ITEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t nchunks = (M + RM - 1) / RM;
  const int64_t per = (nchunks + splits - 1) / splits;
  const int64_t ch0 = (int64_t)split * per, ch1 = std::min<int64_t>(nchunks, ch0 + per);
  typedef T t8 __attribute__((ext_vector_type(8)));

  // staging item q of this thread: slice sl, channel chunk c8, row group rg (8 rows); its prologue
  // constants stay in registers
  int it_sl[IPT], it_c8[IPT], it_rg[IPT];
  bool it_on[IPT];
  float psc[IPT][8], psh[IPT][8], cs[IPT][8];
#pragma unroll
  for (int q = 0; q < IPT; ++q) {
    const int item = tid + kThreads * q;
    it_on[q] = item < nitems;
    const int it = it_on[q] ? item : 0;
    it_sl[q] = it / ITEMS;
    const int w = it - it_sl[q] * ITEMS;
    it_c8[q] = w % (BJ / 8);
    it_rg[q] = w / (BJ / 8);
    const int cbase = (it_sl[q] == 0 ? jb : kb) * BJ + it_c8[q] * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      psc[q][e] = PRO ? pro_scale[cbase + e] : 1.f;
      psh[q][e] = PRO ? pro_shift[cbase + e] : 0.f;
      cs[q][e] = 0.f;
    }
  }

  f16v acc[TPW][TPW];
#pragma unroll
  for (int x = 0; x < TPW; ++x)
#pragma unroll
    for (int y = 0; y < TPW; ++y)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[x][y][i] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  const int jt0 = (wave >> 1) * TPW, kt0 = (wave & 1) * TPW;

  auto load = [&](int64_t ch, t8 (&v)[IPT][8]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
      const int cb = (it_sl[q] == 0 ? jb : kb) * BJ + it_c8[q] * 8;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        int64_t m = std::min<int64_t>(ch * RM + it_rg[q] * 8 + rr, M - 1);
        if (s2_H > 0) {
          const int Wo = s2_W >> 1, HWo = (s2_H >> 1) * Wo;
          const int64_t n = m / HWo;
          const int rem = (int)(m - n * HWo), yo = rem / Wo, xo = rem - yo * Wo;
          m = (n * s2_H + 2 * yo) * s2_W + 2 * xo;
        }
        if (it_on[q]) v[q][rr] = *reinterpret_cast<const t8*>(a + m * K + cb);
      }
    }
  };
  auto process = [&](int64_t ch, t8 (&v)[IPT][8]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
      if (!it_on[q]) continue;
      const int64_t m0 = ch * RM + it_rg[q] * 8;
      t8 col[8];  // col[e] = the 8 rows of channel e
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const bool ok = m0 + rr < M;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float f = to_f<T>(v[q][rr][e]);
          if constexpr (PRO) f = to_f<T>(from_f<T>(fmaxf(fmaf(f, psc[q][e], psh[q][e]), 0.f)));
          f = ok ? f : 0.f;
          cs[q][e] += f;
          col[e][rr] = from_f<T>(f);
        }
      }
      char* base = img[ONE ? 0 : it_sl[q]] + (it_c8[q] * 8) * PITCH + it_rg[q] * 16;
#pragma unroll
      for (int e = 0; e < 8; ++e) *reinterpret_cast<t8*>(base + e * PITCH) = col[e];
    }
    __syncthreads();
    const char* iJ = img[0];
    const char* iK = (diag || ONE) ? img[0] : img[ONE ? 0 : 1];
#pragma unroll
    for (int ks = 0; ks < RM / 16; ++ks) {
      i4v fa[TPW], fb[TPW];
#pragma unroll
      for (int x = 0; x < TPW; ++x) {
        fa[x] = *reinterpret_cast<const i4v*>(iJ + (32 * (jt0 + x) + r) * PITCH + (16 * ks + 8 * h) * 2);
        fb[x] = *reinterpret_cast<const i4v*>(iK + (32 * (kt0 + x) + r) * PITCH + (16 * ks + 8 * h) * 2);
      }
#pragma unroll
      for (int x = 0; x < TPW; ++x)
#pragma unroll
        for (int y = 0; y < TPW; ++y) acc[x][y] = Mf<T>::run(fa[x], fb[y], acc[x][y]);
    }
    __syncthreads();
  };
  t8 va[IPT][8], vb[IPT][8];
  if (ch0 < ch1) load(ch0, va);
  for (int64_t ch = ch0; ch < ch1; ch += 2) {
    if (ch + 1 < ch1) load(ch + 1, vb);
    process(ch, va);
    if (ch + 1 < ch1) {
      if (ch + 2 < ch1) load(ch + 2, va);
      process(ch + 1, vb);
    }
  }

  // lane holds C[8 jj + 4 h + ii][r] of each tile in acc[4 jj + ii]
  float* gp = gram_part + (int64_t)split * K * K;
#pragma unroll
  for (int x = 0; x < TPW; ++x)
#pragma unroll
    for (int y = 0; y < TPW; ++y)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int gi = jb * BJ + 32 * (jt0 + x) + 8 * jj + 4 * h + ii;
          const int gj = kb * BJ + 32 * (kt0 + y) + r;
          gp[(int64_t)gi * K + gj] = acc[x][y][4 * jj + ii];
        }
  if (diag) {
    // column sums: items (c8, rg) of one channel chunk merge in row-group order through LDS
    float* red = reinterpret_cast<float*>(img[0]);  // [ITEMS][8] (the images are free after the loop)
#pragma unroll
    for (int q = 0; q < IPT; ++q)
      if (it_on[q] && it_sl[q] == 0) {
        const int w = it_c8[q] + (BJ / 8) * it_rg[q];
#pragma unroll
        for (int e = 0; e < 8; ++e) red[w * 8 + e] = cs[q][e];
      }
    __syncthreads();
    for (int c = tid; c < BJ; c += kThreads) {
      float t = 0.f;
      for (int rg = 0; rg < RM / 8; ++rg) t += red[((c >> 3) + (BJ / 8) * rg) * 8 + (c & 7)];
      colsum_part[(int64_t)split * K + jb * BJ + c] = t;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// g_pre = g * bit, column sums of g_pre. Block = cvb 8-channel chunks x R row lanes; split y owns a
// contiguous run of rows; 4 rows in flight per lane; the R lanes of a chunk merge through LDS in order.
template <typename T>
__global__ __launch_bounds__(kThreads) void k_mask_colsum(const T* __restrict__ g, const uint8_t* __restrict__ bits,
                                                          T* __restrict__ out, int64_t M, int N, int cvb,
                                                          int64_t rows_per_split, float* __restrict__ part) {
  __shared__ float red[kThreads * 8];
  const int tid = threadIdx.x, v = tid % cvb, rl = tid / cvb, R = kThreads / cvb;
  const int c0 = (blockIdx.x * cvb + v) * 8;
  const int N8 = N >> 3;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split, r1 = std::min<int64_t>(M, r0 + rows_per_split);
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  typedef T t8 __attribute__((ext_vector_type(8)));
  const bool active = rl < R && c0 < N;
  if (active) {
    int64_t m = r0 + rl;
    for (; m + 3 * (int64_t)R < r1; m += 4 * (int64_t)R) {
      t8 x[4];
      uint32_t b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x[u] = *reinterpret_cast<const t8*>(g + (m + u * R) * N + c0);
        b[u] = bits[(m + u * R) * N8 + (c0 >> 3)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (!((b[u] >> e) & 1u)) x[u][e] = from_f<T>(0.f);
          s[e] += to_f<T>(x[u][e]);
        }
        *reinterpret_cast<t8*>(out + (m + u * R) * N + c0) = x[u];
      }
    }
    for (; m < r1; m += R) {
      t8 x = *reinterpret_cast<const t8*>(g + m * N + c0);
      const uint32_t b = bits[m * N8 + (c0 >> 3)];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (!((b >> e) & 1u)) x[e] = from_f<T>(0.f);
        s[e] += to_f<T>(x[e]);
      }
      *reinterpret_cast<t8*>(out + m * N + c0) = x;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = s[e];
  __syncthreads();
  if (rl == 0 && c0 < N) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = 0.f;
      for (int q = 0; q < R; ++q) t += red[(q * cvb + v) * 8 + e];
      part[(int64_t)blockIdx.y * N + c0 + e] = t;
    }
  }
}


// ------------------------------------------------------------------------------------------------
// combine kernels (ops/bn_fold.py FoldCombine)

constexpr int kSumLanes = 16;  // split-lanes per 64-column block of sum_partials

__global__ __launch_bounds__(64 * kSumLanes) void k_sum_partials(SumPartials s, int b1, int b2, int b3) {
  // blocks [0, b1) -> array 0, [b1, b2) -> 1, [b2, b3) -> 2, [b3, ..) -> 3; 64 columns per block, kSumLanes
  // lanes over the rows (8 loads in flight each), merged in lane order through LDS
  __shared__ float sh[kSumLanes][64];
  const int b = blockIdx.x;
  const int i = b < b1 ? 0 : (b < b2 ? 1 : (b < b3 ? 2 : 3));
  const int lb = b - (i == 0 ? 0 : (i == 1 ? b1 : (i == 2 ? b2 : b3)));
  const float* part = s.part[i];
  const int64_t rows = s.rows[i], cols = s.cols[i];
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int64_t c = (int64_t)lb * 64 + cl;
  float acc = 0.f;
  if (c < cols) {
    int64_t r = lane;
    for (; r + 7 * kSumLanes < rows; r += 8 * kSumLanes) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(r + u * kSumLanes) * cols + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; r < rows; r += kSumLanes) acc += part[r * cols + c];
  }
  sh[lane][cl] = acc;
  __syncthreads();
  if (lane == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < kSumLanes; ++l) t += sh[l][cl];
    s.out[i][c] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_fold_sums(const T* __restrict__ W, const float* __restrict__ P,
                                                   const float* __restrict__ Sg, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd, int N, int K,
                                                   float* __restrict__ sums, float* __restrict__ bn_grads) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;  // one wave per channel
  if (n >= N) return;
  float d = 0.f;
  for (int k = lane; k < K; k += 64) d = fmaf(to_f<T>(W[(int64_t)n * K + k]), P[(int64_t)n * K + k], d);
  d = wave_sum(d);
  if (lane == 0) {
    const float s1 = Sg[n], s2 = d - mean[n] * s1;
    sums[n] = s1;
    sums[N + n] = s2;
    bn_grads[n] = s2 * invstd[n];
    bn_grads[N + n] = s1;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_fold_coef(const T* __restrict__ W, const float* __restrict__ sums,
                                                   const float* __restrict__ count, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd, const float* __restrict__ weight,
                                                   int N, int K, float* __restrict__ abd, float* __restrict__ BW) {
  const int n = blockIdx.x;
  const float inv_n = 1.f / count[0];
  const float is = invstd[n], wv = weight ? weight[n] : 1.f;
  const float mdy = sums[n] * inv_n, mdyx = sums[N + n] * inv_n;
  const float A = is * wv, B = -is * is * A * mdyx, D = A * (mean[n] * is * is * mdyx - mdy);
  if (threadIdx.x == 0) {
    abd[n] = A;
    abd[N + n] = B;
    abd[2 * N + n] = D;
  }
  for (int k = threadIdx.x; k < K; k += blockDim.x) BW[(int64_t)n * K + k] = B * to_f<T>(W[(int64_t)n * K + k]);
}

template <typename T>
__global__ __launch_bounds__(256) void k_fold_final(const float* __restrict__ abd, const float* __restrict__ P,
                                                    const float* __restrict__ X, const float* __restrict__ Sa, int N,
                                                    int K, T* __restrict__ dW) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * K) return;
  const int n = (int)(i / K), k = (int)(i - (int64_t)n * K);
  dW[i] = from_f<T>(fmaf(abd[n], P[i], fmaf(abd[2 * N + n], Sa[k], X[i])));
}

int mask_cvb(int N) { return std::min(N / 8, 64); }

}  // namespace

int gram_splits(int64_t M, int K) {
  const int BJ = K % 128 == 0 ? 128 : 64;
  const int pairs = (K / BJ) * (K / BJ);
  const bool one = K == BJ;
  const int RM = BJ == 64 ? (one ? GramGeo<64, true>::RM : GramGeo<64, false>::RM)
                          : (one ? GramGeo<128, true>::RM : GramGeo<128, false>::RM);
  const int64_t nchunks = (M + RM - 1) / RM;
  return (int)std::max<int64_t>(1, std::min<int64_t>(nchunks, kGramTargetWG / pairs));
}

void gram_partials(int dt, const void* a, int64_t M, int K, const float* pro_scale, const float* pro_shift,
                   float* gram_part, float* colsum_part, hipStream_t st, int s2_H, int s2_W) {
  if (K % 64 != 0 || K <= 0 || M <= 0) throw std::runtime_error("gram_partials: K % 64 == 0, M > 0");
  const int BJ = K % 128 == 0 ? 128 : 64;
  const int nb = K / BJ, splits = gram_splits(M, K);
  const dim3 grid(nb * nb * splits), block(kThreads);
  const bool pro = pro_scale != nullptr;
  const bool one = K == BJ;
  auto go = [&](auto tag) {
    using T = decltype(tag);
    const T* ap = reinterpret_cast<const T*>(a);
    auto L = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, block, 0, st, ap, M, K, pro_scale, pro_shift, splits, gram_part, colsum_part,
                         s2_H, s2_W);
    };
    if (BJ == 128) {
      if (one) { if (pro) L(k_gram<T, true, 128, true>); else L(k_gram<T, false, 128, true>); }
      else { if (pro) L(k_gram<T, true, 128, false>); else L(k_gram<T, false, 128, false>); }
    } else {
      if (one) { if (pro) L(k_gram<T, true, 64, true>); else L(k_gram<T, false, 64, true>); }
      else { if (pro) L(k_gram<T, true, 64, false>); else L(k_gram<T, false, 64, false>); }
    }
  };
  switch (dt) {
    case kF16: go(f16{}); break;
    case kBF16: go(bf16{}); break;
    default: throw std::runtime_error("gram_partials: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("gram_partials: ") + hipGetErrorString(e));
}

int mask_colsum_splits(int64_t M, int N) {
  const int cvb = mask_cvb(N), R = kThreads / cvb;
  const int gx = (N / 8 + cvb - 1) / cvb;
  const int64_t want = std::max<int64_t>(1, 1024 / gx);
  const int64_t max_splits = std::max<int64_t>(1, M / (4 * R));
  return (int)std::min(want, max_splits);
}

void mask_colsum(int dt, const void* g, const uint8_t* bits, void* g_pre, int64_t M, int N, float* colsum_part,
                 hipStream_t st) {
  if (N % 8 != 0 || N <= 0 || M <= 0) throw std::runtime_error("mask_colsum: N % 8 == 0, M > 0");
  const int cvb = mask_cvb(N);
  const int gx = (N / 8 + cvb - 1) / cvb;
  const int splits = mask_colsum_splits(M, N);
  const int64_t rps = (M + splits - 1) / splits;
  const dim3 grid(gx, splits), block(kThreads);
  switch (dt) {
    case kF16:
      hipLaunchKernelGGL(k_mask_colsum<f16>, grid, block, 0, st, (const f16*)g, bits, (f16*)g_pre, M, N, cvb, rps,
                         colsum_part);
      break;
    case kBF16:
      hipLaunchKernelGGL(k_mask_colsum<bf16>, grid, block, 0, st, (const bf16*)g, bits, (bf16*)g_pre, M, N, cvb, rps,
                         colsum_part);
      break;
    default: throw std::runtime_error("mask_colsum: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("mask_colsum: ") + hipGetErrorString(e));
}

void sum_partials(const SumPartials& s, hipStream_t st) {
  int nb[4];
  for (int i = 0; i < 4; ++i) nb[i] = s.part[i] ? (int)((s.cols[i] + 63) / 64) : 0;
  const int b1 = nb[0], b2 = b1 + nb[1], b3 = b2 + nb[2], tot = b3 + nb[3];
  if (tot == 0) return;
  hipLaunchKernelGGL(k_sum_partials, dim3(tot), dim3(64 * kSumLanes), 0, st, s, b1, b2, b3);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("sum_partials: ") + hipGetErrorString(e));
}

#define BH_FOLD_DT(dt, T, ...)                                   \
  switch (dt) {                                                  \
    case kF16: { using T = f16; __VA_ARGS__; } break;            \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;          \
    default: throw std::runtime_error("bn_fold: fp16 / bf16 only"); \
  }

void fold_sums(int dt, const void* W, const float* P, const float* Sg, const float* mean, const float* invstd, int N,
               int K, float* sums, float* bn_grads, hipStream_t st) {
  BH_FOLD_DT(dt, T, hipLaunchKernelGGL(k_fold_sums<T>, dim3((N + 3) / 4), dim3(256), 0, st, (const T*)W, P, Sg, mean,
                                       invstd, N, K, sums, bn_grads));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fold_sums: ") + hipGetErrorString(e));
}

void fold_coef(int dt, const void* W, const float* sums, const float* count, const float* mean, const float* invstd,
               const float* weight, int N, int K, float* abd, float* BW, hipStream_t st) {
  BH_FOLD_DT(dt, T, hipLaunchKernelGGL(k_fold_coef<T>, dim3(N), dim3(std::min(256, std::max(64, K))), 0, st,
                                       (const T*)W, sums, count, mean, invstd, weight, N, K, abd, BW));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fold_coef: ") + hipGetErrorString(e));
}

void fold_final(int dt, const float* abd, const float* P, const float* X, const float* Sa, int N, int K, void* dW,
                hipStream_t st) {
  const int64_t tot = (int64_t)N * K;
  BH_FOLD_DT(dt, T, hipLaunchKernelGGL(k_fold_final<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, abd, P,
                                       X, Sa, N, K, (T*)dW));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fold_final: ") + hipGetErrorString(e));
}

}  // namespace bh
