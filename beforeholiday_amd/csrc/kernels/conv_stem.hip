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

template <typename T>
__global__ __launch_bounds__(256) void k_stem_fwd(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y,
                                                  int N) {
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
}

}  // namespace

bool conv_stem_supported(int N, int C, int H, int W, int K) {
  return N > 0 && C == 3 && H == kH && W == kW && K == kK;
}

void conv_stem_forward(int dt, const void* x, const void* w, void* y, int N, hipStream_t st) {
  // persistent: two workgroups per CU (57 KB of LDS each), each walks row blocks blockIdx.x + k * grid
  const int nblk = N * (kOH / kRowsOut);
  const dim3 grid((unsigned)(nblk < 512 ? nblk : 512));
  switch (dt) {
    case kF16:
      hipLaunchKernelGGL(k_stem_fwd<f16>, grid, dim3(256), 0, st, (const f16*)x, (const f16*)w, (f16*)y, N);
      break;
    case kBF16:
      hipLaunchKernelGGL(k_stem_fwd<bf16>, grid, dim3(256), 0, st, (const bf16*)x, (const bf16*)w, (bf16*)y, N);
      break;
    default: throw std::runtime_error("conv_stem_forward: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv_stem_forward: ") + hipGetErrorString(e));
}

}  // namespace bh
