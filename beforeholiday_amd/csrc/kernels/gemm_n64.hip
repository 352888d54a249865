// Skinny GEMM for the 64-channel side of ResNet-50's 56x56 1x1 convolutions:
//   C[M, 64] = A[M, K] . B[64, K]^T (+ R[M, 64]),  K in {64, 128, 256}, fp32 accumulation.
// A is an NHWC activation viewed as [pixels, channels] (M = N*H*W = 802816 at batch 256), so the op
// is HBM bound (K = 256: 512 + 128 bytes per row), and hipBLASLt / MIOpen tile it as a general GEMM
// (0.13-0.17 ms for 64 <-> 256 at 56x56 vs a 0.09 ms streaming floor,
// profiles/resnet50_conv_paths_miopen_vs_gemm.jsonl). Here a wave owns whole 32-row strips with
// all 64 output columns: both MFMA operands are 16-byte row-contiguous global loads
// (v_mfma_f32_32x32x16: lane l supplies row l % 32, k = 8 (l / 32) .. +7), the weights stay in
// registers (K = 64) or LDS (K >= 128) for the life of the persistent workgroup, and the next
// strip's rows are loaded while the current strip's MFMAs and stores run. R (optional) is added in
// the epilogue -- the residual-branch gradient of the bottleneck's data gradient, so that sum costs
// no extra pass. Measured at 3.5-3.8 TB/s (profiles/gemm_n64_vs_hipblaslt_miopen.jsonl): ahead of
// hipBLASLt at every shape and of MIOpen at K = 64, behind MIOpen's 256 -> 64 forward; the model
// times it against MIOpen per shape.
#include "bh/api.h"
#include "bh/dense_api.h"
#include "bh/device.h"

#include <algorithm>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma32;
template <> struct Mfma32<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 256;  // 4 waves, each a stream of 32-row strips

template <typename T, int KD>
__global__ __launch_bounds__(kThreads) void k_gemm_n64(const T* __restrict__ A, const T* __restrict__ B,
                                                       const T* __restrict__ R, T* __restrict__ C, int strips) {
  constexpr int KS = KD / 16;  // k-steps
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  // weights, both 32-column halves, every k-step: in registers for K = 64; for K >= 128 (64 KD-wide
  // rows would take 128 VGPRs and one wave per SIMD) staged once in LDS with 16-byte padded rows
  // (row stride 4 banks apart: the 16-lane phases of a ds_read_b128 hit 64 distinct banks)
  constexpr bool kLds = KD >= 128;
  constexpr int RS = KD * 2 + 16;
  __shared__ __attribute__((aligned(16))) char bl[kLds ? 64 * RS : 16];
  i4v b[2][kLds ? 1 : KS];
  if constexpr (kLds) {
    for (int c = threadIdx.x; c < 64 * KD / 8; c += kThreads) {
      const int row = c / (KD / 8), c8 = c - row * (KD / 8);
      *reinterpret_cast<i4v*>(bl + row * RS + c8 * 16) = *reinterpret_cast<const i4v*>(B + (int64_t)row * KD + c8 * 8);
    }
    __syncthreads();
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s)
        b[t][s] = *reinterpret_cast<const i4v*>(B + (int64_t)(32 * t + r) * KD + 16 * s + 8 * h);
  }
  const int stride = gridDim.x * (kThreads / 64);
  int strip = blockIdx.x * (kThreads / 64) + wave;
  i4v a[KS];
  auto load = [&](int sp) {
    const T* src = A + ((int64_t)sp * 32 + r) * KD + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(src + 16 * s));
  };
  // prefetches are unconditional (clamped to the last strip: re-read, never used) so the compiler's
  // vmcnt bookkeeping stays exact: the wait for a[] then leaves the previous strip's stores in flight
  // instead of draining them (a conditional load merged into vmcnt(0), profiles/conv_pmc_r6.md)
  if (strips <= 0) return;
  load(min(strip, strips - 1));
  for (; strip < strips; strip += stride) {
    f16v acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
    if constexpr (kLds) {
      int boff = r * RS + 16 * h;
      asm volatile("" : "+v"(boff));  // opaque per strip: keeps the LDS reads in the loop (not hoisted into VGPRs)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const i4v b0 = *reinterpret_cast<const i4v*>(bl + boff + 32 * s);
        const i4v b1 = *reinterpret_cast<const i4v*>(bl + boff + 32 * RS + 32 * s);
        acc[0] = Mfma32<T>::run(a[s], b0, acc[0]);
        acc[1] = Mfma32<T>::run(a[s], b1, acc[1]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc[0] = Mfma32<T>::run(a[s], b[0][s], acc[0]);
        acc[1] = Mfma32<T>::run(a[s], b[1][s], acc[1]);
      }
    }
    const int next = strip + stride;
    load(min(next, strips - 1));  // the a[] registers are free once the MFMAs above have read them
    // lane holds C[8 j + 4 h + i][32 t + r] in acc[t][4 j + i]: per store, lanes 0-31 write one
    // 64-byte row segment. (Swapping the operands so each lane holds four consecutive columns, one
    // 8-byte store per row, measured slower: 0.072 vs 0.055 ms at K = 64 -- 32 rows per store.)
    const int64_t row0 = (int64_t)strip * 32 + 4 * h;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t o = (row0 + 8 * j + i) * 64 + r;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float v = acc[t][4 * j + i];
          if (R) v += to_f(R[o + 32 * t]);
          C[o + 32 * t] = from_f<T>(v);
        }
      }
  }
}

}  // namespace

bool gemm_n64_supported(int64_t M, int K, int N) {
  return N == 64 && (K == 64 || K == 128 || K == 256) && M > 0 && M % 32 == 0 && M / 32 < (1ll << 31);
}

void gemm_n64(int dt, const void* a, const void* b, const void* resid, void* c, int64_t M, int K, hipStream_t st) {
  if (!gemm_n64_supported(M, K, 64)) throw std::runtime_error("gemm_n64: M % 32 == 0, K in {64, 128, 256}");
  const int strips = (int)(M / 32);
  // persistent workgroups, as many as are resident at once (K = 256: 108 VGPRs + 32 AGPRs, three
  // per CU; otherwise four) so no late workgroup runs a tail alone
  const int grid = std::min((strips + 3) / 4, 256 * (K == 256 ? 3 : 4));
  auto run = [&](auto tt) {
    using T = typename decltype(tt)::type;
    switch (K) {
      case 64:
        hipLaunchKernelGGL((k_gemm_n64<T, 64>), dim3(grid), dim3(kThreads), 0, st, (const T*)a, (const T*)b,
                           (const T*)resid, (T*)c, strips);
        break;
      case 128:
        hipLaunchKernelGGL((k_gemm_n64<T, 128>), dim3(grid), dim3(kThreads), 0, st, (const T*)a, (const T*)b,
                           (const T*)resid, (T*)c, strips);
        break;
      default:
        hipLaunchKernelGGL((k_gemm_n64<T, 256>), dim3(grid), dim3(kThreads), 0, st, (const T*)a, (const T*)b,
                           (const T*)resid, (T*)c, strips);
    }
  };
  switch (dt) {
    case kF16: run(std::common_type<f16>{}); break;
    case kBF16: run(std::common_type<bf16>{}); break;
    default: throw std::runtime_error("gemm_n64: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("gemm_n64: ") + hipGetErrorString(e));
}

}  // namespace bh
