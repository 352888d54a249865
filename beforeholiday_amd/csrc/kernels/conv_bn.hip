// 1x1 convolution GEMMs with the neighbouring BatchNorms folded in (see bh/conv_bn_api.h): the
// ResNet-50 bottleneck's 1x1 convolutions, which are HBM bound at batch 256 (K, N <= 512 against
// M = 50k - 800k pixels), so every separate BatchNorm pass over their inputs or outputs costs as much
// as the convolution itself.
//
// Layout (MFMA v_mfma_f32_32x32x16): a wave owns whole 32-row strips of the output with NC columns
// (a column slice of N). Lane (r, h) = (lane & 31, lane >> 5) loads row r of the strip, channels
// 16 s + 8 h .. + 7 of k-step s straight from global memory into its A fragment (16-byte loads), so
// the BatchNorm prologue is a register transform on the fragment (scale / shift held in LDS). The
// column slice of the weights stays in LDS for the life of the persistent workgroup (rows padded by 16
// bytes: the 16-lane phases of a ds_read_b128 hit distinct banks), one B-fragment read per MFMA. The
// next strip's rows are loaded while the current strip's epilogue runs.
//
// Epilogue: lane holds C[8 j + 4 h + i][32 t + r] in acc[t][4 j + i], i.e. ONE column per 32-column
// tile, 16 rows of it. The rounded values go through a wave-private 16 x 64 LDS tile (adjacent lanes
// swap one value so each writes 32-bit words) and leave as 128-byte row segments: NC / 16 stores per strip, so
// the vmcnt wait for the next strip's A rows does not have to drain the stores (vmcnt counts both on
// gfx9; 2-byte column stores were NC * 2 per strip, past vmcnt's range). The per-column statistics are
// accumulated per lane across all strips the wave processes (2 floats per tile), then reduced over the
// lane halves, the 4 waves (LDS) and written as one partial row per workgroup: deterministic, no
// atomics, and the statistics of an 800k-row output cost one extra read of nothing.
#include "bh/api.h"
#include "bh/conv_bn_api.h"
#include "bh/device.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));

template <typename T> struct Mf;
template <> struct Mf<f16> {
  typedef h8v v8;
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mf<bf16> {
  typedef b8v v8;
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kStageBytes = 16 * 128;  // per wave: 16 rows x 64 fp16 columns of output

struct Geo {
  int nslices;  // column slices of NC
  int G;        // workgroups per slice (multiple of 8)
  int strips;   // M / 32
  int ss_off;   // LDS byte offset of the prologue scale / shift
  int red_off;  // LDS byte offset of the cross-wave reduction buffer
  int stage_off;  // LDS byte offset of the output staging tiles (kStageBytes per wave)
};

// S2: 0 none, 1 stride-2 gather of the A rows, 2 stride-2 scatter of the C rows (output row (n, y, x)
// of the quarter-resolution problem lands in row (n, 2y, 2x) of the full-resolution C)
// PRO: 0 none, 1 BatchNorm + ReLU of the A operand, 2 BatchNorm backward (A a + B y + D from a second stream)
template <typename T, int KC, int NC, int EPI, int PRO, int S2, bool RES>
__global__ __launch_bounds__(kThreads, 2) void k_c1x1(C1x1Args p, Geo g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NC / 32;  // 32-column tiles per wave
  constexpr int KS = KC / 16;  // k-steps per register chunk
  using V8 = typename Mf<T>::v8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  // workgroup -> (column slice, strip group), XCD-aware: consecutive ids land on different XCDs
  // (id % 8), so the slices of one strip group are given the same id % 8 and share that XCD's L2
  const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
  const int slice = idx % g.nslices;
  const int grp = (idx / g.nslices) * 8 + xcd;
  const int K = p.K, N = p.N;
  const int nch = K / KC;
  const int col0 = slice * NC;
  const int RS = 2 * K + 16;
  char* bl = smem;
  float* ss = reinterpret_cast<float*>(smem + g.ss_off);
  float* se = ss + (PRO == 1 ? 2 * K : (PRO == 2 ? 3 * K : 0));  // the epilogue's per-column constants
  {
    if (!p.b_trans) {
      const T* Bp = reinterpret_cast<const T*>(p.B) + (int64_t)col0 * K;
      const int per_row = K >> 3;
      for (int c = threadIdx.x; c < NC * per_row; c += kThreads) {
        const int row = c / per_row, c8 = c - row * per_row;
        *reinterpret_cast<i4v*>(bl + row * RS + c8 * 16) =
            *reinterpret_cast<const i4v*>(Bp + (int64_t)row * K + c8 * 8);
      }
    } else {
      // B given as [K, N] (a forward weight read as its transpose, the data-gradient case): each thread
      // reads 8 consecutive n of one k (16 bytes) and scatters them down 8 LDS rows
      const T* Bp = reinterpret_cast<const T*>(p.B) + col0;
      constexpr int per_k = NC / 8;
      for (int c = threadIdx.x; c < K * per_k; c += kThreads) {
        const int k = c / per_k, n8 = c - k * per_k;
        typedef T t8 __attribute__((ext_vector_type(8)));
        const t8 v = *reinterpret_cast<const t8*>(Bp + (int64_t)k * N + n8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<T*>(bl + (n8 * 8 + j) * RS + 2 * k) = v[j];
      }
    }
    if constexpr (PRO == 1) {
      for (int c = threadIdx.x; c < K; c += kThreads) {
        ss[c] = p.pro_scale[c];
        ss[K + c] = p.pro_shift[c];
      }
    }
    if constexpr (PRO == 2) {
      for (int c = threadIdx.x; c < 3 * K; c += kThreads) ss[c] = p.bnb[c];
    }
    if constexpr (EPI == kC1x1Affine) {  // frozen per-column scale / shift of the epilogue
      for (int c = threadIdx.x; c < NC; c += kThreads) {
        se[c] = p.a_scale[col0 + c];
        se[NC + c] = p.a_shift[col0 + c];
      }
    }
    if constexpr (EPI == kC1x1Bwd) {  // the previous BatchNorm's per-column constants, read per tile
      for (int c = threadIdx.x; c < NC; c += kThreads) {
        se[c] = p.bscale[col0 + c];
        se[NC + c] = p.bshift[col0 + c];
        se[2 * NC + c] = p.bmean[col0 + c];
      }
    }
  }
  __syncthreads();

  // per-lane statistics of column col0 + 32 t + r
  float s1[NT], s2[NT], e0[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    s1[t] = s2[t] = 0.f;
    e0[t] = 0.f;
    if constexpr (EPI == kC1x1Stats) e0[t] = p.kshift ? p.kshift[col0 + 32 * t + r] : 0.f;
  }

  const T* __restrict__ A = reinterpret_cast<const T*>(p.A);
  T* __restrict__ Cp = reinterpret_cast<T*>(p.C);
  const T* __restrict__ Rp = reinterpret_cast<const T*>(p.R);
  const T* __restrict__ Yp = reinterpret_cast<const T*>(p.by);
  auto arow = [&](int sp) -> int64_t {
    const int64_t m = (int64_t)sp * 32 + r;
    if constexpr (S2 == 1) {
      const int Wo = p.s2_W >> 1, HWo = (p.s2_H >> 1) * Wo;
      const int64_t n = m / HWo;
      const int rem = (int)(m - n * HWo), yo = rem / Wo, xo = rem - yo * Wo;
      return (n * p.s2_H + 2 * yo) * p.s2_W + 2 * xo;
    } else {
      return m;
    }
  };
  // The wave's work is a flat sequence of (strip, chunk) steps; A fragments are double-buffered in
  // registers so that the loads of step i + 1 are in flight during step i's MFMAs (and epilogue).
  const int stride = g.G * kWaves;
  const int first = grp * kWaves + wave;
  const int total = (first < g.strips ? (g.strips - first + stride - 1) / stride : 0) * nch;
  i4v a0[KS], a1[KS];
  i4v y0[PRO == 2 ? KS : 1], y1[PRO == 2 ? KS : 1];  // PRO 2: the BatchNorm input's fragments
  const T* __restrict__ BY = reinterpret_cast<const T*>(p.bnb_y);
  auto load = [&](int i, i4v(&a)[KS], i4v(&yv)[PRO == 2 ? KS : 1]) {
    const int q = i / nch, c = i - q * nch;
    const int64_t off = arow(first + q * stride) * (p.lda ? p.lda : K) + c * KC + 8 * h;
    const T* src = A + off;
    if (p.a_load == 1) {
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s] = *reinterpret_cast<const i4v*>(src + 16 * s);
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s] = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(src + 16 * s));
    }
    if constexpr (PRO == 2) {
#pragma unroll
      for (int s = 0; s < KS; ++s) yv[s] = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(BY + off + 16 * s));
    }
  };
  // Output staging (all but the scatter variant): the lane-per-column MFMA result leaves as 128-byte
  // row segments (whole cache lines: 64-byte half lines measured ~20% slower on the HBM-bound shapes)
  // through a wave-private [16 rows][64 columns] LDS tile. A pair of 32-column tiles fills it twice --
  // rows 0-15 (j < 2 of both tiles), then rows 16-31; the even tile's upper rows wait in 4 registers
  // until the odd tile is done with its lower ones. A strip of 32 x NC outputs leaves in NC / 16
  // dwordx4 stores instead of NC * 2 2-byte ones: few enough that the next strip's loads are waited
  // for precisely (vmcnt counts stores too on gfx9) instead of draining every store of the strip.
  // Rows 4 apart (the two lane halves) are XOR-swizzled by half a row: conflict-free 32-bit writes.
  char* stage = smem + g.stage_off + wave * kStageBytes;
  auto put = [&](int row, int half_col, unsigned int word) __attribute__((always_inline)) {
    const int rr = row & 15, wd = half_col * 16 + (r >> 1);
    *reinterpret_cast<unsigned int*>(stage + rr * 128 + 4 * (wd ^ (((rr >> 2) & 1) << 4))) = word;
  };
  auto flush = [&](int strip, int pair, int half) __attribute__((always_inline)) {
    const int ch = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rr = 8 * q + (lane >> 3);
      const i4v v = *reinterpret_cast<const i4v*>(stage + rr * 128 + 16 * (ch ^ (((rr >> 2) & 1) << 2)));
      *reinterpret_cast<i4v*>(Cp + ((int64_t)strip * 32 + 16 * half + rr) * N + col0 + 64 * pair + ch * 8) = v;
    }
  };
  // the lane pair (r, r ^ 1) swaps one value of rows v - 1, v (v odd) so that each lane holds one
  // 32-bit word of two adjacent columns: the even lane row v - 1's, the odd lane row v's
  auto pair_word = [&](int v, unsigned int o_even, unsigned int o_odd, int* row) __attribute__((always_inline)) {
    const bool odd = r & 1;
    const unsigned int keep = odd ? o_odd : o_even, send = odd ? o_even : o_odd;
    const unsigned int got = (unsigned int)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    const int vv = odd ? v : v - 1;
    *row = 8 * (vv >> 2) + 4 * h + (vv & 3);
    return odd ? (got | (keep << 16)) : (keep | (got << 16));
  };
  f16v acc[NT];
  // Narrow tiles (NC = 64): the residual / previous-output values the epilogue reads are loaded at the
  // top of the strip's last chunk, so their HBM latency hides behind that chunk's MFMAs instead of
  // stalling the epilogue (one 2-byte column load per row: nothing to coalesce them into). Wider tiles
  // keep the per-tile loads (hoisting 64+ values spills).
  // (not next to the BatchNorm-backward prologue's second fragment stream: registers)
  constexpr bool kHoist = (RES != (EPI == kC1x1Bwd)) && S2 != 2 && NT * 16 <= 32 && PRO != 2;
  auto process = [&](int i, i4v(&a)[KS], i4v(&yv)[PRO == 2 ? KS : 1]) {
    const int q = i / nch, c = i - q * nch;
    const int strip = first + q * stride;
    if (c == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
    }
    if constexpr (PRO == 2) {
      // BatchNorm backward on the fragment: A a + B y + D in fp32, rounded once (the input gradient as the
      // separate data-gradient pass would have stored it)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kb = c * KC + 16 * s + 8 * h;
        V8 v = __builtin_bit_cast(V8, a[s]);
        const V8 yy = __builtin_bit_cast(V8, yv[s]);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = from_f<T>(fmaf(to_f<T>(v[j]), ss[kb + j], fmaf(to_f<T>(yy[j]), ss[K + kb + j], ss[2 * K + kb + j])));
        a[s] = __builtin_bit_cast(i4v, v);
      }
    }
    if constexpr (PRO == 1) {
      // BatchNorm + ReLU of the producing layer, on the fragment (channels 16 s + 8 h .. + 7)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kb = c * KC + 16 * s + 8 * h;
        const float4 c0 = *reinterpret_cast<const float4*>(ss + kb);
        const float4 c1 = *reinterpret_cast<const float4*>(ss + kb + 4);
        const float4 d0 = *reinterpret_cast<const float4*>(ss + K + kb);
        const float4 d1 = *reinterpret_cast<const float4*>(ss + K + kb + 4);
        const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sh[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        V8 v = __builtin_bit_cast(V8, a[s]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = from_f<T>(fmaxf(fmaf(to_f<T>(v[j]), sc[j], sh[j]), 0.f));
        a[s] = __builtin_bit_cast(i4v, v);
      }
    }
    T xh[kHoist ? NT : 1][16];
    if constexpr (kHoist) {
      if (c + 1 == nch) {
        const T* src = RES ? Rp : Yp;
        const int64_t rh = (int64_t)strip * 32 + 4 * h;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int v = 0; v < 16; ++v) xh[t][v] = src[(rh + 8 * (v >> 2) + (v & 3)) * N + col0 + 32 * t + r];
      }
    }
    int boff = r * RS + 16 * h + c * KC * 2;
    asm volatile("" : "+v"(boff));  // opaque: keeps the B fragment reads in the loop, not in VGPRs
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const i4v bf = *reinterpret_cast<const i4v*>(bl + boff + t * 32 * RS + 32 * s);
        acc[t] = Mf<T>::run(a[s], bf, acc[t]);
      }
    if (c + 1 < nch) return;
    // ---- epilogue ----
    const int64_t row0 = (int64_t)strip * 32 + 4 * h;
    // output rows of this lane: the scatter maps them once per strip (shared by every column tile);
    // otherwise row v is row0 + 8 (v >> 2) + (v & 3)
    int64_t orow[S2 == 2 ? 16 : 1];
    auto out_row = [&](int v) -> int64_t {
      if constexpr (S2 == 2) return orow[v];
      else return row0 + 8 * (v >> 2) + (v & 3);
    };
#pragma unroll
    for (int v = 0; v < (S2 == 2 ? 16 : 0); ++v) {
      const int64_t m = row0 + 8 * (v >> 2) + (v & 3);
      const int Wo = p.s2_W >> 1, HWo = (p.s2_H >> 1) * Wo;
      const int64_t n = m / HWo;
      const int rem = (int)(m - n * HWo), yo = rem / Wo, xo = rem - yo * Wo;
      orow[v] = (n * p.s2_H + 2 * yo) * p.s2_W + 2 * xo;
    }
    unsigned int held[4];  // the even tile's rows 16-31 (see the staging note above)
    int held_row[4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = col0 + 32 * t + r;
      unsigned int o_prev = 0;
      float xr[16];
      if constexpr (kHoist) {
#pragma unroll
        for (int v = 0; v < 16; ++v) xr[v] = to_f<T>(xh[t][v]);
      } else if constexpr (RES || EPI == kC1x1Bwd) {
        const T* src = RES ? Rp : Yp;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[4 * j + i] = to_f<T>(src[out_row(4 * j + i) * N + col]);
      }
      float bsc = 0.f, bsh = 0.f, bmn = 0.f;
      if constexpr (EPI == kC1x1Bwd || EPI == kC1x1Affine) {
        bsc = se[32 * t + r];
        bsh = se[NC + 32 * t + r];
      }
      if constexpr (EPI == kC1x1Bwd) bmn = se[2 * NC + 32 * t + r];
      uint32_t mw[EPI == kC1x1Mask ? 16 : 1];  // kMask: the 32 mask bits of this tile's columns, per row
      if constexpr (EPI == kC1x1Mask) {
        const uint32_t* mp = reinterpret_cast<const uint32_t*>(p.mbits);
        const int wcol = (col0 + 32 * t) >> 5;
#pragma unroll
        for (int v = 0; v < 16; ++v) mw[v] = mp[out_row(v) * (N >> 5) + wcol];
      }
      float yv[16];
      if constexpr (RES && EPI == kC1x1Bwd) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) yv[4 * j + i] = to_f<T>(Yp[out_row(4 * j + i) * N + col]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int v = 4 * j + i;
          float x = acc[t][v];
          if constexpr (EPI == kC1x1Affine) {
            // conv + bias / frozen BatchNorm (+ residual) (+ ReLU) (x mask): one pass
            x = fmaf(x, bsc, bsh);
            if constexpr (RES) {
              if (!p.r_mul) x += xr[v];
            }
            if (p.relu) x = fmaxf(x, 0.f);
            if constexpr (RES) {
              if (p.r_mul) x *= xr[v];
            }
          } else if constexpr (RES) {
            x += xr[v];
          }
          if constexpr (EPI == kC1x1Mask) x = ((mw[v] >> r) & 1u) ? x : 0.f;
          const T o = from_f<T>(x);
          if constexpr (S2 == 2) {
            Cp[out_row(v) * N + col] = o;
          } else {
            const unsigned int ou = __builtin_bit_cast(unsigned short, o);
            if (v & 1) {
              int row;
              const unsigned int w = pair_word(v, o_prev, ou, &row);
              if (v < 8) {
                put(row, t & 1, w);
              } else if (!(t & 1)) {
                held[(v - 8) >> 1] = w;
                held_row[(v - 8) >> 1] = row;
              } else {
                put(row, 1, w);
              }
              if ((t & 1) && v == 7) {  // rows 0-15 of the pair complete: out, then the held rows in
                flush(strip, t >> 1, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k) put(held_row[k], 0, held[k]);
              }
              if ((t & 1) && v == 15) flush(strip, t >> 1, 1);
            } else {
              o_prev = ou;
            }
          }
          const float f = to_f<T>(o);  // statistics of the value as stored
          if constexpr (EPI == kC1x1Stats) {
            const float d = f - e0[t];
            s1[t] += d;
            s2[t] = fmaf(d, d, s2[t]);
          } else if constexpr (EPI == kC1x1Bwd) {
            const float y = RES ? yv[v] : xr[v];
            const float dz = (!p.brelu || fmaf(y, bsc, bsh) > 0.f) ? f : 0.f;
            s1[t] += dz;
            s2[t] = fmaf(dz, y - bmn, s2[t]);
          } else if constexpr (EPI == kC1x1Mask) {
            s1[t] += f;
          }
        }
      // one tile's residual / input loads at a time: hoisting every tile's 16-32 loads to the top
      // of the epilogue spills at NC >= 128
      if constexpr (RES || EPI == kC1x1Bwd || EPI == kC1x1Mask) __builtin_amdgcn_sched_barrier(0);
    }
  };
  // prefetches are unconditional (clamped to the last strip: re-read, never used), so the compiler's
  // vmcnt bookkeeping stays exact across iterations; behind `if (i + 1 < total)` it merged the paths
  // into a full vmcnt(0) drain before each strip's A rows (profiles/conv_pmc_r6.md)
  if (total > 0) {
    const int last = total - 1;
    load(0, a0, y0);
    for (int i = 0; i < total; i += 2) {
      load(min(i + 1, last), a1, y1);
      process(i, a0, y0);
      load(min(i + 2, last), a0, y0);
      if (i + 1 < total) process(i + 1, a1, y1);
    }
  }

  if constexpr (EPI == kC1x1Stats || EPI == kC1x1Bwd || EPI == kC1x1Mask) {
    float* red = reinterpret_cast<float*>(smem + g.red_off);  // [waves][2][NC], aliases the staging tiles
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      s1[t] += __shfl_xor(s1[t], 32);
      s2[t] += __shfl_xor(s2[t], 32);
      if (h == 0) {
        red[(wave * 2) * NC + 32 * t + r] = s1[t];
        red[(wave * 2 + 1) * NC + 32 * t + r] = s2[t];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += kThreads) {
      float u = 0.f, w = 0.f;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) {
        u += red[(q * 2) * NC + c];
        w += red[(q * 2 + 1) * NC + c];
      }
      p.part[(int64_t)grp * N + col0 + c] = u;
      p.part[((int64_t)g.G + grp) * N + col0 + c] = w;
    }
  }
}

constexpr int kSumRows = 16;  // partial rows summed in parallel per column

// (optional) the BatchNorm's parameter gradients from the same sums: gb = sum dy (statistic 0), gw = sum
// dy x_hat = (statistic 1) * invstd -- the two tiny elementwise launches per BatchNorm they replace
__global__ __launch_bounds__(64 * kSumRows) void k_sum_parts(int G, int N, const float* __restrict__ part,
                                                             float* __restrict__ sums, float count,
                                                             const float* __restrict__ invstd, float* __restrict__ gw,
                                                             float* __restrict__ gb) {
  // block = 64 columns x kSumRows row groups of one statistic (blockIdx.y); coalesced 256-byte rows,
  // a fixed order (strided per group, then the groups in order): deterministic
  // the rows in the bn_part_segments order (one segment after the other here; bn_merge_parts sums
  // large-G segments in parallel with the same bits)
  __shared__ float sh[kSumRows][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, which = blockIdx.y;
  const int SG = bn_part_segments(G), R = (G + SG - 1) / SG;
  float t = 0.f;
  for (int s = 0; s < SG; ++s) {
    const int g1 = min(G, (s + 1) * R);
    float acc = 0.f;
    if (c < N) {
      const float* src = part + (int64_t)which * G * N + c;
      int g = s * R + rg;
      // 8 rows of loads in flight per lane; the adds stay in row order
      for (; g + 7 * kSumRows < g1; g += 8 * kSumRows) {
        float u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = src[(int64_t)(g + j * kSumRows) * N];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += u[j];
      }
      for (; g < g1; g += kSumRows) acc += src[(int64_t)g * N];
    }
    if (s > 0) __syncthreads();  // the previous segment's reads of sh are done
    sh[rg][cl] = acc;
    __syncthreads();
    float st = 0.f;
#pragma unroll
    for (int q = 0; q < kSumRows; ++q) st += sh[q][cl];
    t += st;
  }
  if (rg == 0 && c < N) {
    sums[(int64_t)which * N + c] = t;
    if (which == 0 && gb) gb[c] = t;
    if (which == 1 && gw) gw[c] = t * invstd[c];
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && count >= 0.f) sums[2 * N] = count;
}

// ---------------------------------------------------------------------------- host side
struct Plan {
  int NC, KC, lds, occ;
  Geo g;
};

int ss_bytes(int NC, int K, int pro, bool bwd, bool aff) {
  // prologue constants per k (1: scale, shift; 2: A, B, D), then the epilogue's per column
  return (pro == 1 ? 8 * K : (pro == 2 ? 12 * K : 0)) + (bwd ? 12 * NC : (aff ? 8 * NC : 0));
}

int lds_bytes(int NC, int K, int pro, bool bwd, bool aff, bool stats, bool scatter) {
  // the statistics reduction buffer (used after the strip loop) aliases the output staging tiles
  return NC * (2 * K + 16) + ss_bytes(NC, K, pro, bwd, aff) +
         std::max(stats ? kWaves * 2 * NC * 4 : 0, scatter ? 0 : kWaves * kStageBytes);
}

bool make_plan(const C1x1Args& a, Plan* pl) {
  if (a.K <= 0 || a.N <= 0 || a.M <= 0 || a.K % 64 != 0 || a.N % 64 != 0 || a.M % 32 != 0) return false;
  if (a.M / 32 >= (1ll << 31)) return false;
  const int pro = a.bnb ? 2 : (a.pro_scale != nullptr ? 1 : 0);
  const bool stats = a.epi == kC1x1Stats || a.epi == kC1x1Bwd || a.epi == kC1x1Mask,
             bwd = a.epi == kC1x1Bwd, aff = a.epi == kC1x1Affine, scatter = a.s2_H > 0 && a.s2_scatter;
  // register budget: the backward epilogue (input loads + statistics) fits 4 column tiles per wave
  // (the mask epilogue's per-row mask words spill at wider slices)
  int max_nc = a.epi == kC1x1Mask ? 64 : (bwd ? (a.R ? 64 : 128) : 256);
  if (a.bnb) max_nc = std::min(max_nc, scatter ? 64 : 128);  // (the second fragment stream's registers)
  int NC = 0, occ = 0;
  // the widest column slice (A read once per slice) that still leaves two workgroups per CU; else one
  // (a higher resident-workgroup target measured no better: profiles/c1x1_occupancy_ab.txt)
  constexpr int occ_max = 2;
  for (int want_occ = occ_max; want_occ >= 1 && !NC; --want_occ)
    for (int nc : {256, 128, 64})
      if (nc <= max_nc && a.N % nc == 0 &&
          lds_bytes(nc, a.K, pro, bwd, aff, stats, scatter) <= 160 * 1024 / want_occ) {
        NC = nc;
        occ = want_occ;
        break;
      }
  if (!NC) return false;
  // registers: two A chunks of KC / 4 VGPRs each next to NC / 2 accumulators
  // (the BatchNorm-backward prologue's second fragment stream leaves room for 64-deep chunks only)
  const int KC = (NC <= 128 && a.K % 128 == 0 && !(bwd && NC == 128) && pro != 2) ? 128 : 64;
  Geo g{};
  g.nslices = a.N / NC;
  g.strips = (int)(a.M / 32);
  const int want = (g.strips + kWaves - 1) / kWaves;         // one strip per wave
  const int cap = std::max(1, occ * 256 / g.nslices);        // resident workgroups per slice
  g.G = (std::min(want, cap) + 7) / 8 * 8;
  g.ss_off = NC * (2 * a.K + 16);
  g.red_off = g.ss_off + ss_bytes(NC, a.K, pro, bwd, aff);
  g.stage_off = g.red_off;
  pl->NC = NC;
  pl->KC = KC;
  pl->lds = lds_bytes(NC, a.K, pro, bwd, aff, stats, scatter);
  pl->occ = occ;
  pl->g = g;
  return true;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <typename T> struct Tag { using type = T; };

}  // namespace

bool c1x1_supported(const C1x1Args& a) {
  Plan pl;
  if (!make_plan(a, &pl)) return false;
  if (!al16(a.A) || !al16(a.B) || !al16(a.C) || (a.R && !al16(a.R))) return false;
  if (a.epi == kC1x1Bwd && (!a.by || !a.bscale || !a.bshift || !a.bmean)) return false;
  if (a.epi == kC1x1Affine && (!a.a_scale || !a.a_shift || a.pro_scale || a.s2_scatter)) return false;
  if ((a.epi == kC1x1Stats || a.epi == kC1x1Bwd || a.epi == kC1x1Mask) && !a.part) return false;
  if (a.epi == kC1x1Mask &&
      (!a.mbits || (reinterpret_cast<uintptr_t>(a.mbits) & 3) || a.N % 32 || a.pro_scale || a.bnb || a.s2_H > 0))
    return false;
  if (a.s2_H > 0) {
    if (a.s2_H % 2 || a.s2_W % 2 || a.M % ((int64_t)(a.s2_H / 2) * (a.s2_W / 2))) return false;
    if (a.pro_scale || a.epi == kC1x1Bwd) return false;  // combinations not instantiated
    if (a.bnb && a.lda) return false;
    // (bnb scatter: 64-column slices re-read A and its y stream per slice; past 256 channels that leaves L2)
    if (a.bnb && a.K > 256) return false;
    // gather: no residual (the affine epilogue excepted); scatter: plain epilogue accumulating into the
    // full-resolution C (R == C)
    if (a.s2_scatter ? (a.epi != kC1x1Plain || a.R != a.C) : (a.R != nullptr && a.epi != kC1x1Affine)) return false;
  } else if (a.s2_scatter) {
    return false;
  }
  if (a.pro_scale && (a.R || a.epi != kC1x1Stats)) return false;
  // BatchNorm-backward prologue: a second [M, K] stream; plain or backward-sums epilogue, no residual / stride 2
  if (a.bnb && (!a.bnb_y || !al16(a.bnb_y) || a.pro_scale || (a.s2_H > 0 && !a.s2_scatter) ||
                (a.epi != kC1x1Plain && a.epi != kC1x1Bwd)))
    return false;
  if (a.lda && (a.lda < a.K || a.lda % 8 || a.s2_H > 0)) return false;
  return true;
}

int c1x1_parts(const C1x1Args& a) {
  Plan pl;
  return make_plan(a, &pl) ? pl.g.G : 0;
}

void c1x1_run(int dt, const C1x1Args& a_in, hipStream_t st) {
  if (!c1x1_supported(a_in)) throw std::runtime_error("c1x1: unsupported shape / arguments");
  C1x1Args a = a_in;
  if (a.a_load < 0) a.a_load = 0;
  Plan pl;
  make_plan(a, &pl);
  const dim3 grid(pl.g.nslices * pl.g.G), block(kThreads);
  const bool pro = a.pro_scale != nullptr, s2 = a.s2_H > 0, res = a.R != nullptr, bnb = a.bnb != nullptr;
  // instantiated flag combinations: (epi, pro, s2, res)
  auto go = [&](auto tt, auto kc, auto nc) {
    using T = typename decltype(tt)::type;
    constexpr int KC = decltype(kc)::value, NC = decltype(nc)::value;
    auto L = [&](auto kern) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, pl.lds);
      hipLaunchKernelGGL(kern, grid, block, pl.lds, st, a, pl.g);
    };
    if (bnb) {  // BatchNorm-backward prologue (KC 64 only, see make_plan)
      if constexpr (KC == 64 && NC <= 64) {
        if (a.epi == kC1x1Bwd && res) L(k_c1x1<T, KC, NC, kC1x1Bwd, 2, 0, true>);
      }
      if constexpr (KC == 64 && NC <= 64) {  // the downsample's data gradient scattered onto conv1's
        if (s2 && a.s2_scatter) L(k_c1x1<T, KC, NC, kC1x1Plain, 2, 2, true>);
      }
      if constexpr (KC == 64 && NC <= 128) {
        if (a.epi == kC1x1Bwd && !res) L(k_c1x1<T, KC, NC, kC1x1Bwd, 2, 0, false>);
        else if (a.epi != kC1x1Bwd && !res) L(k_c1x1<T, KC, NC, kC1x1Plain, 2, 0, false>);
        else if (a.epi != kC1x1Bwd && !s2) L(k_c1x1<T, KC, NC, kC1x1Plain, 2, 0, true>);
      }
    } else if (a.epi == kC1x1Mask) {
      if constexpr (NC == 64) {
        if (res) L(k_c1x1<T, KC, NC, kC1x1Mask, 0, 0, true>);
        else L(k_c1x1<T, KC, NC, kC1x1Mask, 0, 0, false>);
      }
    } else if (a.epi == kC1x1Stats) {
      if (pro) L(k_c1x1<T, KC, NC, kC1x1Stats, 1, 0, false>);
      else if (s2) L(k_c1x1<T, KC, NC, kC1x1Stats, 0, 1, false>);
      else L(k_c1x1<T, KC, NC, kC1x1Stats, 0, 0, false>);
    } else if (a.epi == kC1x1Bwd) {
      if constexpr (NC <= 64) {
        if (res) L(k_c1x1<T, KC, NC, kC1x1Bwd, 0, 0, true>);
      }
      if constexpr (NC <= 128) {
        if (!res) L(k_c1x1<T, KC, NC, kC1x1Bwd, 0, 0, false>);
      }
    } else if (a.epi == kC1x1Affine) {
      if (s2) {
        if (res) L(k_c1x1<T, KC, NC, kC1x1Affine, 0, 1, true>);
        else L(k_c1x1<T, KC, NC, kC1x1Affine, 0, 1, false>);
      } else {
        if (res) L(k_c1x1<T, KC, NC, kC1x1Affine, 0, 0, true>);
        else L(k_c1x1<T, KC, NC, kC1x1Affine, 0, 0, false>);
      }
    } else {
      if (s2 && a.s2_scatter) L(k_c1x1<T, KC, NC, kC1x1Plain, 0, 2, true>);
      else if (s2) L(k_c1x1<T, KC, NC, kC1x1Plain, 0, 1, false>);
      else if (res) L(k_c1x1<T, KC, NC, kC1x1Plain, 0, 0, true>);
      else L(k_c1x1<T, KC, NC, kC1x1Plain, 0, 0, false>);
    }
  };
  auto by_nc = [&](auto tt, auto kc) {
    switch (pl.NC) {
      case 64: go(tt, kc, std::integral_constant<int, 64>{}); break;
      case 128: go(tt, kc, std::integral_constant<int, 128>{}); break;
      default:
        if constexpr (decltype(kc)::value == 64) go(tt, kc, std::integral_constant<int, 256>{});
        else throw std::runtime_error("c1x1: KC 128 with NC 256 is not instantiated");
    }
  };
  auto by_kc = [&](auto tt) {
    if (pl.KC == 64) by_nc(tt, std::integral_constant<int, 64>{});
    else by_nc(tt, std::integral_constant<int, 128>{});
  };
  switch (dt) {
    case kF16: by_kc(Tag<f16>{}); break;
    case kBF16: by_kc(Tag<bf16>{}); break;
    default: throw std::runtime_error("c1x1: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("c1x1: ") + hipGetErrorString(e));
}

void c1x1_sum_parts(int G, int N, const float* part, float* sums, float count, hipStream_t st, const float* invstd,
                    float* gw, float* gb) {
  hipLaunchKernelGGL(k_sum_parts, dim3((N + 63) / 64, 2), dim3(64 * kSumRows), 0, st, G, N, part, sums, count, invstd,
                     gw, gb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("c1x1_sum_parts: ") + hipGetErrorString(e));
}

// ---- stride-2 pixel gather / scatter-add for the 1x1 stride-2 convolutions (NHWC, 16-bit) ----------------
// out[n, yo, xo, :] = x[n, 2 yo, 2 xo, :] and full[n, 2 yo, 2 xo, :] += q[n, yo, xo, :]: one thread per 16-byte
// channel chunk of a quarter-resolution pixel, so every access is a whole 16-byte vector (torch's strided
// copy / add_ over the same views moved ~1.3 TB/s)
namespace {
template <typename T, bool ADD>
__global__ __launch_bounds__(256) void k_s2_pixels(T* __restrict__ full, T* __restrict__ quarter, int64_t npix_q,
                                                   int Ho, int Wo, int C8) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix_q * C8) return;
  const int64_t pq = i / C8;
  const int c8 = (int)(i - pq * C8);
  const int64_t n = pq / ((int64_t)Ho * Wo);
  const int rem = (int)(pq - n * Ho * Wo), yo = rem / Wo, xo = rem - yo * Wo;
  const int64_t pf = (n * (2 * Ho) + 2 * yo) * (int64_t)(2 * Wo) + 2 * xo;
  typedef T t8 __attribute__((ext_vector_type(8)));
  t8* fp = reinterpret_cast<t8*>(full + pf * C8 * 8) + c8;
  t8* qp = reinterpret_cast<t8*>(quarter + pq * C8 * 8) + c8;
  if constexpr (ADD) {
    t8 a = *fp;
    const t8 b = *qp;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = from_f<T>(to_f<T>(a[j]) + to_f<T>(b[j]));
    *fp = a;
  } else {
    *qp = *fp;
  }
}
}  // namespace

void s2_pixels(int dt, void* full, void* quarter, int64_t n, int ho, int wo, int c, bool add, hipStream_t st) {
  if (c % 8) throw std::runtime_error("s2_pixels: channels must be a multiple of 8");
  const int64_t npix = n * ho * wo, work = npix * (c / 8);
  if (work == 0) return;
  const dim3 grid((unsigned)((work + 255) / 256));
  switch (dt) {
    case kF16:
      if (add) hipLaunchKernelGGL((k_s2_pixels<f16, true>), grid, dim3(256), 0, st, (f16*)full, (f16*)quarter, npix, ho, wo, c / 8);
      else hipLaunchKernelGGL((k_s2_pixels<f16, false>), grid, dim3(256), 0, st, (f16*)full, (f16*)quarter, npix, ho, wo, c / 8);
      break;
    case kBF16:
      if (add) hipLaunchKernelGGL((k_s2_pixels<bf16, true>), grid, dim3(256), 0, st, (bf16*)full, (bf16*)quarter, npix, ho, wo, c / 8);
      else hipLaunchKernelGGL((k_s2_pixels<bf16, false>), grid, dim3(256), 0, st, (bf16*)full, (bf16*)quarter, npix, ho, wo, c / 8);
      break;
    default: throw std::runtime_error("s2_pixels: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("s2_pixels: ") + hipGetErrorString(e));
}

// global-average-pool backward: out[n, y, x, :] = g[n, :] * scale for a channels_last [n, c, h, w] output, one
// 16-byte chunk per thread (torch's expand + contiguous copy from the stride-0 view ran ~1.4 TB/s)
namespace {
template <typename T>
__global__ __launch_bounds__(256) void k_pool_bcast(const T* __restrict__ g, T* __restrict__ out, int64_t hw, int C8,
                                                    int64_t total, float scale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t p = i / C8;
  const int c8 = (int)(i - p * C8);
  const int64_t n = p / hw;
  typedef T t8 __attribute__((ext_vector_type(8)));
  t8 v = *(reinterpret_cast<const t8*>(g + n * C8 * 8) + c8);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = from_f<T>(to_f<T>(v[j]) * scale);
  *(reinterpret_cast<t8*>(out) + i) = v;
}
}  // namespace

void pool_bcast(int dt, const void* g, void* out, int64_t n, int64_t hw, int c, float scale, hipStream_t st) {
  if (c % 8) throw std::runtime_error("pool_bcast: channels must be a multiple of 8");
  const int64_t total = n * hw * (c / 8);
  if (total == 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  switch (dt) {
    case kF16: hipLaunchKernelGGL(k_pool_bcast<f16>, grid, dim3(256), 0, st, (const f16*)g, (f16*)out, hw, c / 8, total, scale); break;
    case kBF16: hipLaunchKernelGGL(k_pool_bcast<bf16>, grid, dim3(256), 0, st, (const bf16*)g, (bf16*)out, hw, c / 8, total, scale); break;
    default: throw std::runtime_error("pool_bcast: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("pool_bcast: ") + hipGetErrorString(e));
}

}  // namespace bh
