// Implicit-GEMM NHWC convolution on MFMA 32x32x16 (gfx950): see bh/igemm_api.h.
//
// GEMM view: rows = output pixels of the grid, columns = output channels, reduction = (tap, input
// channel). A workgroup (4 waves) owns a tile of 4 * MW pixels x NC output channels; each k-step is one
// tap x 64 input channels. The A operand (pixels x channels) never touches LDS: lane (r, h) of a wave
// loads channels 16 ks + 8 h .. + 7 of its pixel r straight into its MFMA fragment (16-byte buffer
// loads through a whole-tensor resource: a tap that falls outside the image gets an out-of-range
// offset and reads zeros -- the convolution's padding -- with no select in front of the MFMAs). The
// stride-2 gather is only address math: the re-reads of an input pixel by its <= 4 taps hit L2. The
// B operand (the [NC x 64] weight slice of the k-step) is staged in LDS, double buffered, rows padded
// by 16 bytes (the 16-lane phases of a ds_read_b128 hit distinct banks); its next slice and the next
// A fragments are in flight during the current k-step's MFMAs. Each lane keeps MW / 32 x NC / 32
// accumulator tiles (the B fragment read from LDS is reused MW / 32 times).
//
// Epilogue: acc[m][t][v] is output pixel 32 m + 8 (v >> 2) + 4 h + (v & 3) of the wave's rows,
// channel 32 t + r: 2-byte stores, 32 lanes = 64 contiguous bytes of one pixel. The statistics of
// the stored values (the next BatchNorm) are reduced per workgroup in a fixed order (lane halves,
// then waves through LDS) into one partial row per pixel tile: deterministic, no atomics.
#include "bh/api.h"
#include "bh/device.h"
#include "bh/igemm_api.h"
#include "bh/knobs.h"

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

template <typename T> struct Mfi;
template <> struct Mfi<f16> {
  typedef h8v v8;
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfi<bf16> {
  typedef b8v v8;
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kCK = 64;            // input channels per k-step
constexpr int kRS = kCK * 2 + 16;  // LDS bytes per staged weight row
constexpr int kMaxProC = 512;
constexpr int kOutOfRange = 0x7ff00000;  // a byte offset past every tensor the kernel reads

// output + statistics epilogue shared by both kernels: acc[m][t][v] is output pixel 32 m + 8 (v >> 2) + 4 h +
// (v & 3) of the wave's MW rows, channel 32 t + r; red: >= 8 NC floats of LDS no wave still reads
template <typename T, int NC, int MW, bool STATS>
BH_DEVICE void igemm_epilogue(const IgemmArgs& a, const IgemmPhase& ph, f16v (&acc)[MW / 32][NC / 32], int mt,
                              int o0, int tiles_m, float* red) {
  constexpr int NT = NC / 32, MT = MW / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int HWg = a.Hg * a.Wg;
  const int64_t P = (int64_t)a.N * HWg;
  // stores through a buffer resource: 32-bit byte offsets (igemm_supported keeps the output below kOutOfRange)
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      a.y, (short)0, (int)((int64_t)a.N * a.Hy * a.Wy * a.Nout * 2), 0x00020000);
  float s1[NT], s2[NT], e0[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    s1[t] = s2[t] = 0.f;
    e0[t] = (STATS && a.kshift) ? a.kshift[o0 + 32 * t + r] : 0.f;
  }
  // pixel -> (image, row, column) by two divisions per strip, then stepping: the 16 pixels of a lane are
  // pb + 0..3, 8..11, 16..19, 24..27 (grid < 2^31 pixels, igemm_supported); a 64-bit division per pixel
  // cost ~2 VALU per MFMA
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int pb = mt * (kWaves * MW) + wave * MW + 32 * m + 4 * h;
    const int n0 = pb / HWg, rem0 = pb - n0 * HWg, i0 = rem0 / a.Wg, j0 = rem0 - i0 * a.Wg;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int d = 8 * (v >> 2) + (v & 3);
      if ((int64_t)pb + d >= P) continue;
      int n = n0, i = i0, j = j0 + d;
      while (j >= a.Wg) {
        j -= a.Wg;
        if (++i == a.Hg) {
          i = 0;
          ++n;
        }
      }
      const int off = ((n * a.Hy + i * a.so + ph.py) * a.Wy + j * a.so + ph.px) * a.Nout + o0 + r;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const T o = from_f<T>(acc[m][t][v]);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, o), rsY, (off + 32 * t) * 2, 0, 0);
        if constexpr (STATS) {
          const float dd = to_f<T>(o) - e0[t];
          s1[t] += dd;
          s2[t] = fmaf(dd, dd, s2[t]);
        }
      }
    }
  }
  if constexpr (STATS) {
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
    for (int c = tid; c < 2 * NC; c += kThreads) {
      const int stat = c / NC, col = c - stat * NC;
      float u = 0.f;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) u += red[(q * 2 + stat) * NC + col];
      a.part[((int64_t)stat * tiles_m + mt) * a.Nout + o0 + col] = u;
    }
  }
}

template <typename T, int NC, int MW, bool PRO, bool STATS>
__global__ __launch_bounds__(kThreads, 2) void k_igemm(IgemmArgs a, int tiles_m) {
  constexpr int NT = NC / 32, MT = MW / 32, NB = NC / 32;  // NB: 16-byte weight pieces per thread per k-step
  using V8 = typename Mfi<T>::v8;
  __shared__ __attribute__((aligned(16))) char smem[2 * NC * kRS + (PRO ? 8 * kMaxProC : 0)];
  const int mt = blockIdx.x;
  if (mt >= tiles_m) return;  // (whole workgroup, before any barrier)
  const IgemmPhase& ph = a.ph[blockIdx.z];
  const int o0 = blockIdx.y * NC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int Ha = a.Ha, Wa = a.Wa, Ca = a.Ca;
  const int HWg = a.Hg * a.Wg;
  const int64_t P = (int64_t)a.N * HWg;
  float* ss = reinterpret_cast<float*>(smem + 2 * NC * kRS);
  if constexpr (PRO) {
    for (int c = tid; c < Ca; c += kThreads) {
      ss[c] = a.pro_scale[c];
      ss[kMaxProC + c] = a.pro_shift[c];
    }
  }
  // this lane's A pixel of each 32-row sub-strip: byte offset of its tap-grid origin (lane half included)
  // and that origin's (row, column) packed 16:16 (a pixel past the grid: a row no tap brings inside)
  int pbase[MT], pyx[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int64_t p = (int64_t)mt * (kWaves * MW) + wave * MW + 32 * m + r;
    const int pp = p < P ? (int)p : 0;
    const int pn = pp / HWg, rem = pp - pn * HWg, pi = rem / a.Wg, pj = rem - pi * a.Wg;
    pbase[m] = ((pn * Ha + pi * a.sa) * Wa + pj * a.sa) * Ca * 2 + 16 * h;
    pyx[m] = p < P ? ((pi * a.sa) << 16) | (pj * a.sa) : 0x40004000;
  }
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.a), 0, (int)((int64_t)a.N * Ha * Wa * Ca * 2), 0x00020000);
  // weights through a buffer resource too: the per-thread part of each piece's offset is fixed for the
  // kernel, the (tap, chunk) part rides in soffset (no 64-bit address math per k-step)
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.b), 0, (int)((int64_t)a.Nout * a.taps_total * Ca * 2), 0x00020000);
  int bvoff[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = tid + i * kThreads, row = q >> 3, ch = q & 7;
    bvoff[i] = ((o0 + row) * a.taps_total * Ca + ch * 8) * 2;
  }
  const int nch = Ca / kCK, steps = ph.ntaps * nch;

  // A fragments of k-step s: ar[m][ks] = channels 16 ks + 8 h .. + 7 of the tap's input pixel
  auto a_load = [&](int s, i4v(&ar)[MT][4], uint32_t& msk) __attribute__((always_inline)) {
    const int t = s / nch, c = s - t * nch;
    const int oy = ph.oy[t], ox = ph.ox[t];
    const int del = ((oy * Wa + ox) * Ca + c * kCK) * 2;  // (uniform)
    msk = 0;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int yi = (pyx[m] >> 16) + oy, xi = (pyx[m] & 0xffff) + ox;
      const bool ok = yi >= 0 && yi < Ha && xi >= 0 && xi < Wa;
      const int off = ok ? pbase[m] + del : kOutOfRange;
      msk |= (ok ? 1u : 0u) << m;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) ar[m][ks] = __builtin_amdgcn_raw_buffer_load_b128(rsA, off + 32 * ks, 0, 0);
    }
  };
  // weight slice of k-step s: rows o0 .. o0 + NC - 1, channels c * 64 .. + 63 of tap tap[t]
  auto b_load = [&](int s, i4v(&br)[NB]) __attribute__((always_inline)) {
    const int t = s / nch, c = s - t * nch;
    const int so = (ph.tap[t] * Ca + c * kCK) * 2;
#pragma unroll
    for (int i = 0; i < NB; ++i) br[i] = __builtin_amdgcn_raw_buffer_load_b128(rsB, bvoff[i], so, 0);
  };
  auto b_store = [&](char* buf, const i4v(&br)[NB]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + i * kThreads;
      *reinterpret_cast<i4v*>(buf + (q >> 3) * kRS + (q & 7) * 16) = br[i];
    }
  };

  f16v acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;

  auto compute = [&](const char* buf, i4v(&ar)[MT][4], uint32_t msk, int s) __attribute__((always_inline)) {
    if constexpr (PRO) {
      const int c = s - (s / nch) * nch;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int cb = c * kCK + 16 * ks + 8 * h;
        const float4 c0 = *reinterpret_cast<const float4*>(ss + cb);
        const float4 c1 = *reinterpret_cast<const float4*>(ss + cb + 4);
        const float4 d0 = *reinterpret_cast<const float4*>(ss + kMaxProC + cb);
        const float4 d1 = *reinterpret_cast<const float4*>(ss + kMaxProC + cb + 4);
        const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sh[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (!((msk >> m) & 1u)) continue;  // padding pads the normalised activation: stays zero
          V8 v = __builtin_bit_cast(V8, ar[m][ks]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = from_f<T>(fmaxf(fmaf(to_f<T>(v[j]), sc[j], sh[j]), 0.f));
          ar[m][ks] = __builtin_bit_cast(i4v, v);
        }
      }
    }
    (void)msk;
    (void)s;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const i4v bf = *reinterpret_cast<const i4v*>(buf + (32 * t + r) * kRS + 32 * ks + 16 * h);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = Mfi<T>::run(ar[m][ks], bf, acc[m][t]);
      }
  };

  char* buf0 = smem;
  char* buf1 = smem + NC * kRS;
  i4v a0[MT][4], a1[MT][4], br[NB];
  uint32_t m0 = 0, m1 = 0;
  a_load(0, a0, m0);
  b_load(0, br);
  b_store(buf0, br);
  __syncthreads();  // weight slice 0 (and the prologue constants) visible
  // Every prefetch is unconditional (past the last k-step it re-reads the last one, never used): with the
  // loads behind `if (s + 1 < steps)` the compiler's vmcnt bookkeeping merged the two paths and waited
  // for EVERYTHING (vmcnt(0)) ahead of each weight store, including the A fragments just requested for
  // the next k-step (profiles/conv_pmc_r6.md). (The compute of the odd tail step stays conditional: it
  // issues no global load.)
  const int last = steps - 1;
  for (int s = 0; s < steps; s += 2) {
    a_load(min(s + 1, last), a1, m1);
    b_load(min(s + 1, last), br);
    compute(buf0, a0, m0, s);
    b_store(buf1, br);
    __syncthreads();
    a_load(min(s + 2, last), a0, m0);
    b_load(min(s + 2, last), br);
    if (s + 1 < steps) compute(buf1, a1, m1, s + 1);
    b_store(buf0, br);
    __syncthreads();
  }

  // ---- epilogue ---- (the weight buffers are free: every wave passed the loop's last barrier)
  igemm_epilogue<T, NC, MW, STATS>(a, ph, acc, mt, o0, tiles_m, reinterpret_cast<float*>(smem));
}


// ---- LDS-staged variant (Config.igemm_lds) ----
// Both operands of a k-step arrive by LDS-DMA (buffer_load ... lds: 16 B per lane through whole-tensor
// resources; a tap outside the image gets an out-of-range offset and lands as zeros) in 144-byte pixel /
// weight-row slots (conflict-free ds_read_b128 fragments), double buffered with ONE barrier per k-step.
// No operand passes through VGPRs on its way in, and the A fragments come from LDS instead of
// fragment-shaped global loads (16 B of each of 32 pixels per instruction), which keep the waves of the
// register-staged kernel waiting on memory (MFMA ~20 %, profiles/conv_pmc_r6.md). 128 output pixels x NC
// channels per workgroup, 32 pixels x NC per wave, as k_igemm<NC, 32>. Measured SLOWER (data gradient
// 1.1-1.2x, forward with the prologue 1.05-1.18x the time; -0.5 % per ResNet-50 step,
// profiles/igemm_lds_ab_r6.txt): the double-buffered stages cost the third workgroup per CU (LDS) and
// every 16-MFMA k-step waits for its DMA at a barrier; so it stays behind Config.igemm_lds (default off).
constexpr int kSlot = 144;
constexpr int kTileP = kWaves * 32;
constexpr unsigned kRsrcWord3 = 0x00020000u;
typedef int i4s __attribute__((ext_vector_type(4)));

// one LDS-DMA instruction (lane-linear 16 B at LDS byte address lds) through resource rs: inline asm, so the
// compiler does not order its LDS write against reads of the other buffer (it would put a vmcnt(0) in
// front of every ds_read); the kernel orders them (vmcnt + barrier at the k-step boundary)
BH_DEVICE void dma16(i4s rs, int voff, unsigned lds) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %2, 0 offen lds" ::"v"(voff),
      "s"(lds), "s"(rs)
      : "memory", "m0");
}
BH_DEVICE i4s rsrc(const void* base, int64_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  return i4s{(int)(uint32_t)b, (int)((b >> 32) & 0xffff), (int)(uint32_t)bytes, (int)kRsrcWord3};
}
BH_DEVICE unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
template <int N> BH_DEVICE void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
BH_DEVICE void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T, int NC, bool PRO, bool STATS>
__global__ __launch_bounds__(kThreads, 2) void k_igemm_lds(IgemmArgs a, int tiles_m) {
  constexpr int NT = NC / 32;
  constexpr int PA = kTileP * kSlot / 1024, PB = NC * kSlot / 1024;  // 1-KiB DMA pieces (18, 18 / 9)
  static_assert(kTileP * kSlot % 1024 == 0 && NC * kSlot % 1024 == 0, "slot images are whole pieces");
  // A pieces wave + 4 i (i < NPA) and B pieces wave + 4 j (j < NPB) of a stage per wave
  constexpr int STAGE = (PA + PB) * 1024, NPA = (PA + kWaves - 1) / kWaves, NPB = (PB + kWaves - 1) / kWaves;
  constexpr int NPW = NPA + NPB;
  using V8 = typename Mfi<T>::v8;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + (PRO ? 8 * kMaxProC : 0)];
  const int mt = blockIdx.x;
  if (mt >= tiles_m) return;  // (whole workgroup, before any barrier)
  const IgemmPhase& ph = a.ph[blockIdx.z];
  const int o0 = blockIdx.y * NC;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ha = a.Ha, Wa = a.Wa, Ca = a.Ca;
  const int HWg = a.Hg * a.Wg;
  const int64_t P = (int64_t)a.N * HWg;
  float* ss = reinterpret_cast<float*>(smem + 2 * STAGE);
  if constexpr (PRO) {
    for (int c = tid; c < Ca; c += kThreads) {
      ss[c] = a.pro_scale[c];
      ss[kMaxProC + c] = a.pro_shift[c];
    }
  }
  const i4s rsA = rsrc(a.a, (int64_t)a.N * Ha * Wa * Ca * 2);
  const i4s rsB = rsrc(a.b, (int64_t)a.Nout * a.taps_total * Ca * 2);
  constexpr int kBadYX = 0x40004000;  // a (y, x) base no tap brings inside the image
  // pixel (row / column base of the tap grid, packed 16:16) and source offset of a tile pixel
  auto pixel = [&](int slot, int& yx, int& off) __attribute__((always_inline)) {
    const int64_t p = (int64_t)mt * kTileP + slot;
    if (p >= P) {
      yx = kBadYX;
      off = 0;
      return;
    }
    const int pn = (int)(p / HWg), rem = (int)(p - (int64_t)pn * HWg), pi = rem / a.Wg, pj = rem - pi * a.Wg;
    yx = ((pi * a.sa) << 16) | (pj * a.sa);
    off = ((pn * Ha + pi * a.sa) * Wa + pj * a.sa) * Ca * 2;
  };
  // this lane's part of its pieces: piece pc of an image fills bytes [1024 pc + 16 lane, +16) of it, i.e.
  // chunk ch of slot sl (ch 8 = the slot's pad: stays an out-of-range read)
  int pyx[NPA], poff[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const bool isa = i < NPA;
    const int pc = wave + kWaves * (isa ? i : i - NPA);
    const int byte = pc * 1024 + 16 * lane, sl = byte / kSlot, ch = (byte - sl * kSlot) >> 4;
    poff[i] = -1;
    if (isa) {
      pyx[i] = kBadYX;
      if (pc < PA && ch < 8) {
        pixel(sl, pyx[i], poff[i]);
        poff[i] += ch * 16;
      }
    } else if (pc < PB && ch < 8) {
      poff[i] = (o0 + sl) * a.taps_total * Ca * 2 + ch * 16;
    }
  }
  // the compute pixel of this lane (PRO: padding taps stay zero, in-image ones get the BatchNorm)
  int cyx = kBadYX, coff = 0;
  if constexpr (PRO) pixel(wave * 32 + r, cyx, coff);
  (void)coff;
  const int nch = Ca / kCK, steps = ph.ntaps * nch;
  auto in_image = [&](int yx, int oy, int ox) __attribute__((always_inline)) {
    const int yi = (yx >> 16) + oy, xi = (yx & 0xffff) + ox;
    return yi >= 0 && yi < Ha && xi >= 0 && xi < Wa;
  };
  auto issue = [&](int s, char* stage) __attribute__((always_inline)) {
    const int t = s / nch, c = s - t * nch;
    const int oy = ph.oy[t], ox = ph.ox[t], tap = ph.tap[t];
    const int adel = ((oy * Wa + ox) * Ca + c * kCK) * 2, bdel = (tap * Ca + c * kCK) * 2;
#pragma unroll
    for (int i = 0; i < NPA; ++i) {
      const int pc = wave + kWaves * i;
      if (pc < PA)  // (wave-uniform; only the last i can fail)
        dma16(rsA, in_image(pyx[i], oy, ox) ? poff[i] + adel : kOutOfRange,
              __builtin_amdgcn_readfirstlane(lds_u32(stage + pc * 1024)));
    }
#pragma unroll
    for (int j = 0; j < NPB; ++j) {
      const int pc = wave + kWaves * j;
      if (pc < PB)
        dma16(rsB, poff[NPA + j] >= 0 ? poff[NPA + j] + bdel : kOutOfRange,
              __builtin_amdgcn_readfirstlane(lds_u32(stage + (PA + pc) * 1024)));
    }
  };

  f16v acc[1][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[0][t][i] = 0.f;

  auto compute = [&](const char* stage, int s) __attribute__((always_inline)) {
    const char* as = stage + (wave * 32 + r) * kSlot + 16 * h;
    const char* bs = stage + PA * 1024 + r * kSlot + 16 * h;
    bool ok = true;
    int cb = 0;
    if constexpr (PRO) {
      const int t = s / nch, c = s - t * nch;
      ok = in_image(cyx, ph.oy[t], ph.ox[t]);
      cb = c * kCK + 8 * h;
    }
    // every fragment of the step first (4 A + 4 NT B reads in flight), then the MFMAs
    i4v av[4], bv[4][NT];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      av[ks] = *reinterpret_cast<const i4v*>(as + 32 * ks);
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[ks][t] = *reinterpret_cast<const i4v*>(bs + 32 * t * kSlot + 32 * ks);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if constexpr (PRO) {
        if (ok) {
          const float* sc = ss + cb + 16 * ks;
          V8 v = __builtin_bit_cast(V8, av[ks]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = from_f<T>(fmaxf(fmaf(to_f<T>(v[j]), sc[j], sc[kMaxProC + j]), 0.f));
          av[ks] = __builtin_bit_cast(i4v, v);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[0][t] = Mfi<T>::run(av[ks], bv[ks][t], acc[0][t]);
    }
  };

  // k-step s computes from stage s & 1 while the DMA of step s + 1 fills the other stage; every issue is
  // unconditional (past the last step it re-reads the last one into the free stage, never used)
  const int last = steps - 1;
  issue(0, smem);
  for (int s = 0; s < steps; ++s) {
    wait_vm<0>();   // this wave's pieces of step s have landed ...
    lds_barrier();  // ... and everyone's; everyone is done reading the other stage (step s - 1)
    issue(min(s + 1, last), smem + ((s + 1) & 1) * STAGE);
    compute(smem + (s & 1) * STAGE, s);
  }
  wait_vm<0>();  // no DMA may land in LDS after the workgroup has ended
  __syncthreads();  // every wave done with the stages (the statistics reduction reuses them)
  igemm_epilogue<T, NC, 32, STATS>(a, ph, acc, mt, o0, tiles_m, reinterpret_cast<float*>(smem));
}

struct Plan {
  int NC, MW, tiles_m;
};

Plan make_plan(const IgemmArgs& a) {
  Plan p;
  // (64-channel tiles everywhere measured slower: profiles/igemm_nc64_ab.txt)
  p.NC = a.Nout % 128 == 0 ? 128 : 64;
  const int64_t P = (int64_t)a.N * a.Hg * a.Wg;
  const int64_t slices = a.Nout / p.NC;
  // 128-channel tiles: 32 pixel rows per wave (64 x 128 spills at two waves per SIMD). 64-channel
  // tiles without the prologue: 64 pixel rows per wave (each weight fragment read from LDS feeds two
  // MFMAs) while that still leaves >= 2 workgroups per CU
  p.MW = (p.NC == 64 && !a.pro_scale && ((P + 255) / 256) * slices * a.nphase >= 512) ? 64 : 32;
  // (64 x 128 wave tiles at one workgroup per CU -- 512 registers, each weight fragment feeding two
  // MFMAs -- measured 0.69-0.99x of this at the three ResNet-50 shapes: profiles/conv3x3_s2_vs_miopen.jsonl)
  p.tiles_m = (int)((P + 4 * p.MW - 1) / (4 * p.MW));
  return p;
}

template <typename T> struct Tag { using type = T; };

}  // namespace

bool igemm_supported(const IgemmArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (a.N <= 0 || a.Ha <= 0 || a.Wa <= 0 || a.Hg <= 0 || a.Wg <= 0 || a.Ca <= 0 || a.Nout <= 0) return false;
  if (a.Ca % kCK || a.Nout % 64 || !al(a.a) || !al(a.b) || !al(a.y)) return false;
  if (a.nphase < 1 || a.nphase > 4 || a.taps_total < 1 || a.taps_total > 255) return false;
  for (int z = 0; z < a.nphase; ++z) {
    if (a.ph[z].ntaps < 1 || a.ph[z].ntaps > 9) return false;
    for (int t = 0; t < a.ph[z].ntaps; ++t)
      if (a.ph[z].tap[t] >= a.taps_total) return false;
  }
  // 32-bit buffer offsets for a (the out-of-range sentinel sits past it), 32-bit pixel indices
  if ((int64_t)a.N * a.Ha * a.Wa * a.Ca * 2 + 128 >= kOutOfRange) return false;
  if ((int64_t)a.Nout * a.taps_total * a.Ca * 2 >= kOutOfRange) return false;  // 32-bit weight offsets
  if ((int64_t)a.N * a.Hy * a.Wy * a.Nout * 2 >= kOutOfRange) return false;     // 32-bit output offsets
  if ((int64_t)a.N * a.Hg * a.Wg >= (1ll << 31)) return false;
  if (a.pro_scale && (!a.pro_shift || a.Ca > kMaxProC)) return false;
  if (a.part && a.nphase != 1) return false;
  return true;
}

int igemm_parts(const IgemmArgs& a) { return make_plan(a).tiles_m; }

void igemm_run(int dt, const IgemmArgs& a, hipStream_t st) {
  if (!igemm_supported(a)) throw std::runtime_error("igemm: unsupported shape / arguments");
  const Plan pl = make_plan(a);
  const dim3 grid((unsigned)pl.tiles_m, (unsigned)(a.Nout / pl.NC), (unsigned)a.nphase);
  const bool pro = a.pro_scale != nullptr, stats = a.part != nullptr;
  const bool lds = knob("igemm_lds", 0) != 0;  // Config.igemm_lds: the LDS-staged kernel (NC = 128 plans)
  auto go = [&](auto tt, auto nc, auto mw) {
    using T = typename decltype(tt)::type;
    constexpr int NC = decltype(nc)::value, MW = decltype(mw)::value;
    auto L = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(kThreads), 0, st, a, pl.tiles_m); };
    if constexpr (MW == 32 && NC == 128) {
      if (lds) {
        if (pro && stats) L(k_igemm_lds<T, NC, true, true>);
        else if (pro) L(k_igemm_lds<T, NC, true, false>);
        else if (stats) L(k_igemm_lds<T, NC, false, true>);
        else L(k_igemm_lds<T, NC, false, false>);
        return;
      }
    }
    if constexpr (MW == 32) {
      if (pro && stats) L(k_igemm<T, NC, MW, true, true>);
      else if (pro) L(k_igemm<T, NC, MW, true, false>);
      else if (stats) L(k_igemm<T, NC, MW, false, true>);
      else L(k_igemm<T, NC, MW, false, false>);
    } else {  // 64 x 64 wave tiles, no prologue (it spills at 64 rows per wave)
      if (stats) L(k_igemm<T, NC, MW, false, true>);
      else L(k_igemm<T, NC, MW, false, false>);
    }
  };
  auto by_mw = [&](auto tt, auto nc) {
    if constexpr (decltype(nc)::value == 64) {
      if (pl.MW == 64) return go(tt, nc, std::integral_constant<int, 64>{});
    }
    go(tt, nc, std::integral_constant<int, 32>{});
  };
  auto by_nc = [&](auto tt) {
    if (pl.NC == 128) by_mw(tt, std::integral_constant<int, 128>{});
    else by_mw(tt, std::integral_constant<int, 64>{});
  };
  switch (dt) {
    case kF16: by_nc(Tag<f16>{}); break;
    case kBF16: by_nc(Tag<bf16>{}); break;
    default: throw std::runtime_error("igemm: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("igemm: ") + hipGetErrorString(e));
}

IgemmArgs igemm_conv3x3_s2_fwd(const void* x, const void* w, void* y, int N, int H, int W, int C, int K) {
  IgemmArgs a;
  a.a = x;
  a.b = w;
  a.y = y;
  a.N = N;
  a.Ha = H;
  a.Wa = W;
  a.Ca = C;
  a.Nout = K;
  a.taps_total = 9;
  a.Hg = a.Hy = (H + 1) / 2;
  a.Wg = a.Wy = (W + 1) / 2;
  a.sa = 2;
  a.so = 1;
  a.nphase = 1;
  IgemmPhase& p = a.ph[0];
  p.ntaps = 9;
  for (int t = 0; t < 9; ++t) {
    p.oy[t] = t / 3 - 1;
    p.ox[t] = t % 3 - 1;
    p.tap[t] = t;
  }
  return a;
}

IgemmArgs igemm_conv3x3_s2_dgrad(const void* dy, const void* wt, void* dx, int N, int H, int W, int C, int K) {
  // dx[2i + py, 2j + px] = sum over taps (r, s) with 2 yo + r - 1 = 2i + py (and likewise columns) of
  // dy[yo, xo] . w[r, s]: an even output row takes r = 1 (yo = i), an odd one r = 0 (yo = i + 1) and
  // r = 2 (yo = i); four phases of 1, 2, 2 and 4 taps over the (H/2) x (W/2) grid
  IgemmArgs a;
  a.a = dy;
  a.b = wt;
  a.y = dx;
  a.N = N;
  a.Ha = H / 2;
  a.Wa = W / 2;
  a.Ca = K;
  a.Nout = C;
  a.taps_total = 9;
  a.Hg = H / 2;
  a.Wg = W / 2;
  a.sa = 1;
  a.Hy = H;
  a.Wy = W;
  a.so = 2;
  a.nphase = 4;
  for (int z = 0; z < 4; ++z) {
    const int py = z >> 1, px = z & 1;
    IgemmPhase& p = a.ph[z];
    p.py = py;
    p.px = px;
    p.ntaps = 0;
    for (int rr = 0; rr < 3; ++rr) {
      if ((rr & 1) == py) continue;  // parity: 2 yo + rr - 1 == 2 i + py needs rr odd for py = 0, even for 1
      for (int sc = 0; sc < 3; ++sc) {
        if ((sc & 1) == px) continue;
        p.oy[p.ntaps] = (py + 1 - rr) / 2;
        p.ox[p.ntaps] = (px + 1 - sc) / 2;
        p.tap[p.ntaps] = rr * 3 + sc;
        ++p.ntaps;
      }
    }
  }
  return a;
}

}  // namespace bh
