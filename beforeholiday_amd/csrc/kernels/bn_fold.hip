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
  // (prefetches unconditional, clamped to the last chunk -- re-read, never used -- so the compiler's
  // vmcnt bookkeeping stays exact instead of merging the paths into vmcnt(0))
  if (ch0 < ch1) {
    const int64_t last = ch1 - 1;
    load(ch0, va);
    for (int64_t ch = ch0; ch < ch1; ch += 2) {
      load(ch + 1 < ch1 ? ch + 1 : last, vb);
      process(ch, va);
      load(ch + 2 < ch1 ? ch + 2 : last, va);
      if (ch + 1 < ch1) process(ch + 1, vb);
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

// fold_reduce in one launch. Blocks [0, N): row n of P = sum of the S1 weight-gradient partial rows (CW columns x
// L lanes over the rows, merged in lane order), Sg[n], and from them the row's sums and BatchNorm gradients:
//   sums[n] = Sg[n], sums[N + n] = W[n] . P[n] - mean[n] Sg[n], bn_grads = (sums[N + n] invstd[n], Sg[n]).
// Blocks [N, ..): 64-column chunks of Gm (K x K) and Sa (K), 4 lanes over their S2 partial rows.
// Every sum runs in a fixed order: deterministic.
constexpr int kFoldThreads = 256;

template <typename T>
__global__ __launch_bounds__(kFoldThreads) void k_fold_reduce(const T* __restrict__ W, const float* __restrict__ p_ws,
                                                              int S1, const float* __restrict__ g_ws,
                                                              const float* __restrict__ sa_ws, int S2,
                                                              const float* __restrict__ sg_ws, int S3,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, int N, int K,
                                                              float* __restrict__ P, float* __restrict__ Gm,
                                                              float* __restrict__ Sa, float* __restrict__ sums,
                                                              float* __restrict__ bn_grads) {
  __shared__ float red[kFoldThreads];
  const int tid = threadIdx.x, b = blockIdx.x;
  if (b < N) {
    const int n = b;
    const int CW = K < kFoldThreads ? K : kFoldThreads, L = kFoldThreads / CW;
    const int c = tid % CW, l = tid / CW;
    const int64_t NK = (int64_t)N * K;
    float d = 0.f;
    for (int k0 = 0; k0 < K; k0 += CW) {
      const int k = k0 + c;
      float a = 0.f;
      if (l < L && k < K) {
        const float* src = p_ws + (int64_t)n * K + k;
        int s = l;
        for (; s + 3 * L < S1; s += 4 * L) {
          const float u0 = src[s * NK], u1 = src[(s + L) * NK], u2 = src[(s + 2 * L) * NK], u3 = src[(s + 3 * L) * NK];
          a += u0;
          a += u1;
          a += u2;
          a += u3;
        }
        for (; s < S1; s += L) a += src[s * NK];
      }
      red[tid] = a;
      __syncthreads();
      if (l == 0 && k < K) {
        float t = 0.f;
        for (int q = 0; q < L; ++q) t += red[q * CW + c];
        P[(int64_t)n * K + k] = t;
        d = fmaf(to_f<T>(W[(int64_t)n * K + k]), t, d);
      }
      __syncthreads();
    }
    float sg = 0.f;
    for (int s = tid; s < S3; s += kFoldThreads) sg += sg_ws[(int64_t)s * N + n];
    d = block_sum(d, red);
    sg = block_sum(sg, red);
    if (tid == 0) {
      const float s2 = d - mean[n] * sg;
      sums[n] = sg;
      sums[N + n] = s2;
      bn_grads[n] = s2 * invstd[n];
      bn_grads[N + n] = sg;
    }
    return;
  }
  // Gm / Sa chunks: 64 columns x 4 lanes over the S2 rows
  const int nbG = (K * K + 63) / 64;
  const int cb = b - N;
  const bool isG = cb < nbG;
  const float* part = isG ? g_ws : sa_ws;
  float* out = isG ? Gm : Sa;
  const int64_t cols = isG ? (int64_t)K * K : K;
  const int64_t col = (int64_t)(isG ? cb : cb - nbG) * 64 + (tid & 63);
  const int lane = tid >> 6;
  float a = 0.f;
  if (col < cols) {
    int s = lane;
    for (; s + 12 < S2; s += 16) {
      const float u0 = part[s * cols + col], u1 = part[(s + 4) * cols + col], u2 = part[(s + 8) * cols + col],
                  u3 = part[(s + 12) * cols + col];
      a += u0;
      a += u1;
      a += u2;
      a += u3;
    }
    for (; s < S2; s += 4) a += part[s * cols + col];
  }
  red[tid] = a;
  __syncthreads();
  if (lane == 0 && col < cols) out[col] = red[tid] + red[tid + 64] + red[tid + 128] + red[tid + 192];
}

// fold_finish in one launch, block n: (A, B, D) of channel n from the all-reduced sums, then row n of
// dW = A P + (B W) Gm + D (x) Sa in fp32 ((B W) Gm formed here: no separate fp32 GEMM), rounded once.
template <typename T>
__global__ __launch_bounds__(kFoldThreads) void k_fold_finish(const T* __restrict__ W, const float* __restrict__ sums,
                                                              const float* __restrict__ count,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ weight,
                                                              const float* __restrict__ P, const float* __restrict__ Gm,
                                                              const float* __restrict__ Sa, int N, int K,
                                                              float* __restrict__ abd, T* __restrict__ dW) {
  extern __shared__ float bw[];  // B W[n, :]
  const int n = blockIdx.x, tid = threadIdx.x;
  const float inv_n = 1.f / count[0];
  const float is = invstd[n], wv = weight ? weight[n] : 1.f;
  const float mdy = sums[n] * inv_n, mdyx = sums[N + n] * inv_n;
  const float A = is * wv, B = -is * is * A * mdyx, D = A * (mean[n] * is * is * mdyx - mdy);
  if (tid == 0) {
    abd[n] = A;
    abd[N + n] = B;
    abd[2 * N + n] = D;
  }
  for (int j = tid; j < K; j += kFoldThreads) bw[j] = B * to_f<T>(W[(int64_t)n * K + j]);
  __syncthreads();
  for (int k = tid; k < K; k += kFoldThreads) {
    float x = 0.f;
    for (int j = 0; j < K; ++j) x = fmaf(bw[j], Gm[(int64_t)j * K + k], x);
    dW[(int64_t)n * K + k] = from_f<T>(fmaf(A, P[(int64_t)n * K + k], fmaf(D, Sa[k], x)));
  }
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

#define BH_FOLD_DT(dt, T, ...)                                   \
  switch (dt) {                                                  \
    case kF16: { using T = f16; __VA_ARGS__; } break;            \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;          \
    default: throw std::runtime_error("bn_fold: fp16 / bf16 only"); \
  }

void fold_reduce(int dt, const void* W, const float* p_ws, int S1, const float* g_ws, const float* sa_ws, int S2,
                 const float* sg_ws, int S3, const float* mean, const float* invstd, int N, int K, float* P, float* Gm,
                 float* Sa, float* sums, float* bn_grads, hipStream_t st) {
  const int grid = N + (K * K + 63) / 64 + (K + 63) / 64;
  BH_FOLD_DT(dt, T, hipLaunchKernelGGL(k_fold_reduce<T>, dim3(grid), dim3(kFoldThreads), 0, st, (const T*)W, p_ws, S1,
                                       g_ws, sa_ws, S2, sg_ws, S3, mean, invstd, N, K, P, Gm, Sa, sums, bn_grads));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fold_reduce: ") + hipGetErrorString(e));
}

void fold_finish(int dt, const void* W, const float* sums, const float* count, const float* mean, const float* invstd,
                 const float* weight, const float* P, const float* Gm, const float* Sa, int N, int K, float* abd,
                 void* dW, hipStream_t st) {
  BH_FOLD_DT(dt, T, hipLaunchKernelGGL(k_fold_finish<T>, dim3(N), dim3(kFoldThreads), sizeof(float) * K, st,
                                       (const T*)W, sums, count, mean, invstd, weight, P, Gm, Sa, N, K, abd, (T*)dW));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fold_finish: ") + hipGetErrorString(e));
}

}  // namespace bh
