// ResNet stem convolution forward: 7x7 / stride 2 / pad 3, 3 -> 64 channels, 224x224 NHWC fp16 / bf16
// input (see bh/conv_api.h), on MFMA 16x16x32 (gfx950).
//
// Three input channels make the reduction awkward for a generic implicit GEMM (MIOpen's kernel for
// this shape runs at ~150 TFLOP/s). Here the reduction index of kernel row r is j = 3 s + c, and for
// output pixel p the 21 values j = 0 .. 20 are CONTIGUOUS in the staged input row (input columns
// 2p - 3 .. 2p + 3, three channels each). One k-step of 32 = one kernel row, padded 21 -> 32 with
// zero weights, so a B fragment (8 consecutive j of one pixel) is 8 contiguous halves of an LDS row.
// The weights (64 x 7 x 32 halves, staged once per persistent workgroup) stay in registers; each wave computes the
// transposed tile C^T[channel][pixel] (weights as the first operand) for 16 pixels x 64 channels per
// item, and writes it through an LDS transpose so every pixel's 64 channels leave as one 128-byte row.
// A workgroup owns four output rows of one image: 13 staged input rows (zero outside the image),
// 28 items (4 rows x 7 tiles of 16 pixels) over 4 waves.
#include "bh/api.h"
#include "bh/conv_api.h"
#include "bh/device.h"

#include <stdexcept>
#include <string>
#include <type_traits>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma16;
template <> struct Mfma16<f16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma16<bf16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kH = 224, kW = 224, kOH = 112, kOW = 112, kK = 64, kR = 7;
constexpr int kRowsOut = 4;                    // output rows per workgroup
constexpr int kRowsIn = 2 * kRowsOut + 5;      // 13 staged input rows
constexpr int kRowHalves = 720;                // staged row: 9 pad halves, 672 data, pad to 720
constexpr int kLead = 9;                       // input column -3 (3 channels) = staged half 0
constexpr int kTileStride = 72;                // epilogue LDS: halves per pixel row (64 + 8 pad)

// STATS: also the BatchNorm statistics of the output (part [2][gridDim.x][64]: per-workgroup sums of
// y - kshift and (y - kshift)^2 over the stored values), so the stem's BatchNorm needs no statistics
// pass. Each lane accumulates its 16 (channel) values over every item the wave computes.
template <typename T, bool STATS = false>
__global__ __launch_bounds__(256) void k_stem_fwd(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y,
                                                  int N, const float* __restrict__ kshift = nullptr,
                                                  float* __restrict__ part = nullptr) {
  __shared__ __attribute__((aligned(16))) uint16_t rows[kRowsIn * kRowHalves];
  __shared__ __attribute__((aligned(16))) uint16_t tile[4][16 * kTileStride];
  __shared__ __attribute__((aligned(16))) uint16_t wl[kK * kR * 32];  // [channel][r][j], j >= 21 zero
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint16_t* xs = reinterpret_cast<const uint16_t*>(x);

  // ---- weights, once per (persistent) workgroup: coalesced 16-byte loads of the [64][147] tensor,
  // scattered into the padded [64][7][32] LDS image, then every lane's 28 A fragments (8 halves of j
  // for channel 16 mt + (lane & 15), j = 8 (lane >> 4) ..) read into registers ----
  for (int i = tid; i < kK * kR * 32 / 8; i += 256) reinterpret_cast<i4v*>(wl)[i] = i4v{0, 0, 0, 0};
  __syncthreads();
  {
    const uint16_t* ws = reinterpret_cast<const uint16_t*>(w);
    for (int i = tid; i < kK * kR * 21 / 8; i += 256) {  // 9408 halves = 1176 chunks
      const i4v v = reinterpret_cast<const i4v*>(ws)[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = i * 8 + e, cr = f / 21, j = f - cr * 21;  // cr = channel * 7 + r
        wl[cr * 32 + j] = (uint16_t)((uint32_t)v[e >> 1] >> (16 * (e & 1)));
      }
    }
  }
  __syncthreads();
  i4v wa[4][kR];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < kR; ++r)
      wa[mt][r] = *reinterpret_cast<const i4v*>(wl + ((16 * mt + (lane & 15)) * kR + r) * 32 + 8 * (lane >> 4));

  // the 9 leading and 39 trailing halves of every staged row stay zero (image padding)
  for (int i = tid; i < kRowsIn * (kRowHalves - 672); i += 256) {
    const int row = i / (kRowHalves - 672), e = i - row * (kRowHalves - 672);
    rows[row * kRowHalves + (e < kLead ? e : e + 672)] = 0;
  }
  uint16_t* tw = tile[wave];
  // STATS: lane holds channels 16 mt + 4 (lane >> 4) + i (i < 4) of its pixel in acc[mt][i]
  float s1[4][4] = {}, s2[4][4] = {}, ks[4][4] = {};
  if constexpr (STATS) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) ks[mt][i] = kshift ? kshift[16 * mt + 4 * (lane >> 4) + i] : 0.f;
  }
  const int nblk = N * (kOH / kRowsOut);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int n = blk / (kOH / kRowsOut), yb = blk - n * (kOH / kRowsOut);
    const int iy0 = 2 * kRowsOut * yb - 3;  // input row of staged row 0
    // ---- stage 13 input rows: 672 data halves per row (16-byte global loads), zero elsewhere ----
    __syncthreads();  // the previous block's items are done with `rows`
    for (int i = tid; i < kRowsIn * 84; i += 256) {  // 84 chunks of 8 halves per image row
      const int row = i / 84, c8 = i - row * 84, iy = iy0 + row;
      const i4v v = (iy >= 0 && iy < kH)
                        ? *reinterpret_cast<const i4v*>(xs + ((int64_t)n * kH + iy) * (kW * 3) + c8 * 8)
                        : i4v{0, 0, 0, 0};
      uint16_t* dst = rows + row * kRowHalves + kLead + c8 * 8;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dst[2 * e] = (uint16_t)(v[e] & 0xffff);
        dst[2 * e + 1] = (uint16_t)((uint32_t)v[e] >> 16);
      }
    }
    __syncthreads();

    // ---- 28 items (output row yl, pixel tile pt) over 4 waves ----
    for (int item = wave; item < kRowsOut * 7; item += 4) {
      const int yl = item / 7, pt = item - yl * 7;
      const int p = pt * 16 + (lane & 15);
      const int j0 = 8 * (lane >> 4);
      f4v acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        // B fragment: halves 6 p + j0 .. + 7 of staged row 2 yl + r (4-byte aligned: four 32-bit reads)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(rows + (2 * yl + r) * kRowHalves + 6 * p + j0);
        const i4v b = i4v{(int)src[0], (int)src[1], (int)src[2], (int)src[3]};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = Mfma16<T>::run(wa[mt][r], b, acc[mt]);
      }
      // lane holds channels 16 mt + 4 (lane >> 4) + i of pixel p: transpose through LDS, then each
      // pixel's 64 channels leave as one 128-byte row
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        T o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = from_f<T>(acc[mt][i]);
        if constexpr (STATS) {  // every item is 16 whole pixels of a real output row
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = to_f<T>(o[i]) - ks[mt][i];
            s1[mt][i] += d;
            s2[mt][i] = fmaf(d, d, s2[mt][i]);
          }
        }
        *reinterpret_cast<uint2*>(tw + (lane & 15) * kTileStride + 16 * mt + 4 * (lane >> 4)) =
            *reinterpret_cast<const uint2*>(o);
      }
      __builtin_amdgcn_wave_barrier();
      const int oy = kRowsOut * yb + yl;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = lane + 64 * h, px = q >> 3, c8 = q & 7;
        const i4v v = *reinterpret_cast<const i4v*>(tw + px * kTileStride + c8 * 8);
        *reinterpret_cast<i4v*>(reinterpret_cast<uint16_t*>(y) +
                                (((int64_t)n * kOH + oy) * kOW + pt * 16 + px) * kK + c8 * 8) = v;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if constexpr (STATS) {
    // over the 16 pixel lanes of each channel group, then the 4 waves through LDS (the row stage is
    // free); one partial row per workgroup, fixed order: deterministic
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          s1[mt][i] += __shfl_xor(s1[mt][i], m);
          s2[mt][i] += __shfl_xor(s2[mt][i], m);
        }
    float* red = reinterpret_cast<float*>(rows);  // [4 waves][2][64]
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * mt + 4 * (lane >> 4) + i;
          red[(wave * 2) * 64 + c] = s1[mt][i];
          red[(wave * 2 + 1) * 64 + c] = s2[mt][i];
        }
    }
    __syncthreads();
    if (tid < 128) {
      const int stat = tid >> 6, c = tid & 63;
      const float v = red[(0 * 2 + stat) * 64 + c] + red[(1 * 2 + stat) * 64 + c] + red[(2 * 2 + stat) * 64 + c] +
                      red[(3 * 2 + stat) * 64 + c];
      part[((int64_t)stat * gridDim.x + blockIdx.x) * 64 + c] = v;
    }
  }
}

// ---- weight gradient: dW[k][r][j] = sum over output pixels p of dY[p][k] * X_r[p][j] ----
// MFMA 32x32x16 with the output channel on the row (A = dY^T) and j on the column (B = X^T), the
// reduction over 16 pixels per k-step. Both operands come from LDS through ds_read_b64_tr_b16: dY rows
// (one 128-byte pixel each, 192-byte stride: conflict free) and the staged input rows, where pixel p's
// 21 values start at half 6p. A transposed read needs 8-byte-aligned rows, which 12p bytes is only for
// even p, so every input row is staged twice: as is, and shifted by two halves for the odd pixels.
// j = 21 .. 31 read the next pixels' values (finite) and are dropped. Persistent workgroups walk output
// rows; wave (mt = wave & 1) owns 32 channels and the kernel rows r = (wave >> 1) + 2 i; each
// workgroup writes one fp32 partial [64][7][21], summed in a fixed order by k_stem_wgrad_reduce.
typedef short s4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;

template <typename T> struct Mfma32s;
template <> struct Mfma32s<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32s<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kDyStride = 96;      // halves per staged dY pixel (64 + 32 pad: 48-dword stride)
constexpr int kXRow = 736;         // halves per staged input-row copy (720 + 16)

template <typename T>
__global__ __launch_bounds__(256) void k_stem_wgrad(const T* __restrict__ x, const T* __restrict__ dy,
                                                    float* __restrict__ part, int N) {
  __shared__ __attribute__((aligned(16))) uint16_t dys[kOW * kDyStride];
  __shared__ __attribute__((aligned(16))) uint16_t xr[kR][2][kXRow];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mt = wave & 1, rbase = wave >> 1;
  const uint16_t* xs = reinterpret_cast<const uint16_t*>(x);
  const uint16_t* ds = reinterpret_cast<const uint16_t*>(dy);
  // zero padding of the input-row copies (never overwritten: data goes to [kLead, kLead + 672))
  for (int i = tid; i < kR * 2 * kXRow; i += 256) (&xr[0][0][0])[i] = 0;

  f16v acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // transposed-read lane roles (16-lane groups): lane 4q + pc names row q, columns 4pc .. 4pc + 3
  const int g16 = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3, h = lane >> 5;
  const int nrows = N * kOH;
  // the next row's dY (896 chunks of 16 B) and input rows (588 chunks) are prefetched into registers
  // while the current row computes, and stored to LDS after the barrier
  constexpr int kDC = kOW * 8, kXC = kR * 84;
  i4v pd[(kDC + 255) / 256], px[(kXC + 255) / 256];
  auto load_row = [&](int row) {
    const int n = row / kOH, oy = row - n * kOH;
#pragma unroll
    for (int i = 0; i < (kDC + 255) / 256; ++i) {
      const int c = tid + 256 * i, pxl = c >> 3, c8 = c & 7;
      if (c < kDC) pd[i] = *reinterpret_cast<const i4v*>(ds + (((int64_t)n * kOH + oy) * kOW + pxl) * kK + c8 * 8);
    }
#pragma unroll
    for (int i = 0; i < (kXC + 255) / 256; ++i) {
      const int c = tid + 256 * i, r = c / 84, c8 = c - r * 84, iy = 2 * oy - 3 + r;
      px[i] = (c < kXC && iy >= 0 && iy < kH)
                  ? *reinterpret_cast<const i4v*>(xs + ((int64_t)n * kH + iy) * (kW * 3) + c8 * 8)
                  : i4v{0, 0, 0, 0};
    }
  };
  auto store_row = [&]() {
#pragma unroll
    for (int i = 0; i < (kDC + 255) / 256; ++i) {
      const int c = tid + 256 * i;
      if (c < kDC) *reinterpret_cast<i4v*>(dys + (c >> 3) * kDyStride + (c & 7) * 8) = pd[i];
    }
#pragma unroll
    for (int i = 0; i < (kXC + 255) / 256; ++i) {
      const int c = tid + 256 * i;
      if (c >= kXC) continue;
      const int r = c / 84, c8 = c - r * 84;
      uint16_t* d0 = &xr[r][0][kLead + c8 * 8];
      uint16_t* d1 = &xr[r][1][kLead + c8 * 8 + 2];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t lo = (uint16_t)(px[i][e] & 0xffff), hi = (uint16_t)((uint32_t)px[i][e] >> 16);
        d0[2 * e] = lo;
        d0[2 * e + 1] = hi;
        d1[2 * e] = lo;
        d1[2 * e + 1] = hi;
      }
    }
  };
  // (prefetches unconditional, clamped to the last row -- re-read, never used -- so the compiler's vmcnt
  // bookkeeping stays exact instead of merging the paths into vmcnt(0))
  if (nrows <= 0) return;
  load_row(min((int)blockIdx.x, nrows - 1));
  __syncthreads();  // zero padding written
  store_row();
  __syncthreads();
  for (int row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int next = row + gridDim.x;
    load_row(min(next, nrows - 1));
#pragma unroll
    for (int ks = 0; ks < kOW / 16; ++ks) {
      // A = dY^T: lane (channel 32 mt + (lane & 31), half h) gets pixels 16 ks + 8 h .. + 7
      const int col = 32 * mt + 16 * (g16 & 1) + 4 * pc;
      const int pA = 16 * ks + 8 * h + q;
      const s4v a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(dys + pA * kDyStride + col));
      const s4v a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(dys + (pA + 4) * kDyStride + col));
      const i2v la = __builtin_bit_cast(i2v, a0), ha = __builtin_bit_cast(i2v, a1);
      const i4v fa = i4v{la[0], la[1], ha[0], ha[1]};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = rbase + 2 * t;
        if (r >= kR) break;  // wave-uniform
        // B = X_r^T: lane (j = (lane & 31), half h) gets pixels 16 ks + 8 h .. + 7; row p starts at
        // half 6p of copy 0 (even p) or at half 6p + 2 of copy 1 (odd p)
        const int j = 16 * (g16 & 1) + 4 * pc;
        auto xaddr = [&](int p) {
          return (p & 1) ? &xr[r][1][6 * p + 2 + j] : &xr[r][0][6 * p + j];
        };
        const s4v b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)xaddr(pA));
        const s4v b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)xaddr(pA + 4));
        const i2v lb = __builtin_bit_cast(i2v, b0), hb = __builtin_bit_cast(i2v, b1);
        acc[t] = Mfma32s<T>::run(fa, i4v{lb[0], lb[1], hb[0], hb[1]}, acc[t]);
      }
    }
    __syncthreads();  // everyone is done with this row's tiles
    if (next < nrows) {
      store_row();
      __syncthreads();
    }
  }
  // lane holds j = lane & 31 and channels 32 mt + 8 i + 4 h + e (acc[t][4 i + e]) of kernel row r
  const int jj = lane & 31;
  if (jj < 21) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = rbase + 2 * t;
      if (r >= kR) break;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = 32 * mt + 8 * i + 4 * h + e;
          part[(int64_t)blockIdx.x * (kK * kR * 21) + (ch * kR + r) * 21 + jj] = acc[t][4 * i + e];
        }
    }
  }
}

// out[i] = sum over the workgroups' partials in a fixed order: a block owns 64 outputs (16 float4
// quads) x 16 partial groups (group g sums partials g, g + 16, ...), the groups added in order in LDS
template <typename T>
__global__ __launch_bounds__(256) void k_stem_wgrad_reduce(const float* __restrict__ part, int parts, T* __restrict__ out) {
  constexpr int kN = kK * kR * 21;  // 9408 = 147 blocks x 64
  __shared__ float4 red[16][16];
  const int tq = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int i = (blockIdx.x * 16 + tq) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = sg; b < parts; b += 16) {
    const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)b * kN + i);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  red[sg][tq] = acc;
  __syncthreads();
  if (sg == 0) {
    float4 t = red[0][tq];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      t.x += red[k][tq].x;
      t.y += red[k][tq].y;
      t.z += red[k][tq].z;
      t.w += red[k][tq].w;
    }
    out[i] = from_f<T>(t.x);
    out[i + 1] = from_f<T>(t.y);
    out[i + 2] = from_f<T>(t.z);
    out[i + 3] = from_f<T>(t.w);
  }
}

}  // namespace

bool conv_stem_supported(int N, int C, int H, int W, int K) {
  return N > 0 && C == 3 && H == kH && W == kW && K == kK;
}

int conv_stem_parts(int N) {
  const int nblk = N * (kOH / kRowsOut);
  return nblk < 512 ? nblk : 512;
}

void conv_stem_forward(int dt, const void* x, const void* w, void* y, int N, hipStream_t st, const float* kshift,
                       float* part) {
  // persistent: two workgroups per CU (57 KB of LDS each), each walks row blocks blockIdx.x + k * grid
  const dim3 grid((unsigned)conv_stem_parts(N));
  switch (dt) {
    case kF16:
      if (part) hipLaunchKernelGGL((k_stem_fwd<f16, true>), grid, dim3(256), 0, st, (const f16*)x, (const f16*)w,
                                   (f16*)y, N, kshift, part);
      else hipLaunchKernelGGL((k_stem_fwd<f16, false>), grid, dim3(256), 0, st, (const f16*)x, (const f16*)w, (f16*)y,
                              N, nullptr, nullptr);
      break;
    case kBF16:
      if (part) hipLaunchKernelGGL((k_stem_fwd<bf16, true>), grid, dim3(256), 0, st, (const bf16*)x, (const bf16*)w,
                                   (bf16*)y, N, kshift, part);
      else hipLaunchKernelGGL((k_stem_fwd<bf16, false>), grid, dim3(256), 0, st, (const bf16*)x, (const bf16*)w,
                              (bf16*)y, N, nullptr, nullptr);
      break;
    default: throw std::runtime_error("conv_stem_forward: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv_stem_forward: ") + hipGetErrorString(e));
}

}  // namespace bh

namespace bh {
int conv_stem_wgrad_parts(int N) { return N * kOH < 512 ? N * kOH : 512; }

void conv_stem_wgrad(int dt, const void* x, const void* dy, void* out, float* ws, int N, hipStream_t st) {
  const int parts = conv_stem_wgrad_parts(N);
  auto run = [&](auto tt) {
    using T = typename decltype(tt)::type;
    hipLaunchKernelGGL(k_stem_wgrad<T>, dim3(parts), dim3(256), 0, st, (const T*)x, (const T*)dy, ws, N);
    hipLaunchKernelGGL(k_stem_wgrad_reduce<T>, dim3(kK * kR * 21 / 64), dim3(256), 0, st, ws, parts, (T*)out);
  };
  switch (dt) {
    case kF16: run(std::common_type<f16>{}); break;
    case kBF16: run(std::common_type<bf16>{}); break;
    default: throw std::runtime_error("conv_stem_wgrad: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv_stem_wgrad: ") + hipGetErrorString(e));
}
}  // namespace bh
