// 2:4 structured-sparsity channel-permutation search (gfx950).
//
// Reference behaviour: apex/contrib/sparsity/permutation_search_kernels/CUDA_kernels/
// permutation_search_kernels.cu:48,85 (sum_after_2_to_4, build_permute_map: magnitude kept by 2:4
// pruning for candidate column groupings) driven by exhaustive_search.py (stripe groups of 8
// columns, best regrouping per group) and call_permutation_search_kernels.py.
//
// MI355X design:
//  * the search primitive is "evaluate every pair of stripes": one workgroup per stripe pair, its
//    256 lanes stride over rows, each lane keeps 35 split accumulators in VGPRs (top-2 of 4 is a
//    6-op compare network), then a wave64 shuffle + LDS reduction per split. All pairs of a
//    [R, C] matrix are scored in one launch; the host greedily applies disjoint improving pairs.
//  * the kept-magnitude sum is a grid-stride partial sum + deterministic second pass.
#include "bh/api.h"
#include "bh/device.h"
#include "bh/sparsity_api.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

BH_DEVICE float top2(float a, float b, float c, float d) {
  const float m1 = fmaxf(a, b), n1 = fminf(a, b), m2 = fmaxf(c, d), n2 = fminf(c, d);
  return fmaxf(m1, m2) + fmaxf(fminf(m1, m2), fmaxf(n1, n2));
}

// bit k set => column k of the 8 goes to the first stripe; column 0 always does (unordered splits).
// Index 0 is the identity split {0,1,2,3 | 4,5,6,7}. Compile-time so every split's gather folds.
constexpr uint8_t kSplit[kStripeSplits] = {
    0x0F, 0x17, 0x1B, 0x1D, 0x27, 0x2B, 0x2D, 0x33, 0x35, 0x39, 0x47, 0x4B, 0x4D, 0x53, 0x55, 0x59, 0x63, 0x65,
    0x69, 0x71, 0x87, 0x8B, 0x8D, 0x93, 0x95, 0x99, 0xA3, 0xA5, 0xA9, 0xB1, 0xC3, 0xC5, 0xC9, 0xD1, 0xE1};

template <uint8_t M>
BH_DEVICE float split_value(const float (&a)[8]) {
  float g0[4], g1[4];
  int i0 = 0, i1 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (M & (1u << k)) g0[i0++] = a[k];
    else g1[i1++] = a[k];
  }
  return top2(g0[0], g0[1], g0[2], g0[3]) + top2(g1[0], g1[1], g1[2], g1[3]);
}

template <int S>
BH_DEVICE void accumulate_splits(const float (&a)[8], float (&acc)[kStripeSplits]) {
  acc[S] += split_value<kSplit[S]>(a);
  if constexpr (S + 1 < kStripeSplits) accumulate_splits<S + 1>(a, acc);
}

__global__ __launch_bounds__(kBlock) void k_pair_gains(const float* __restrict__ m, int64_t R, int64_t C,
                                                       const int32_t* __restrict__ pairs, float* __restrict__ gain,
                                                       int32_t* __restrict__ split) {
  __shared__ float red[kWaves][kStripeSplits];
  const int64_t p = blockIdx.x;
  const int si = pairs[2 * p], sj = pairs[2 * p + 1];
  float acc[kStripeSplits];
#pragma unroll
  for (int s = 0; s < kStripeSplits; ++s) acc[s] = 0.f;
  for (int64_t r = threadIdx.x; r < R; r += kBlock) {
    const float4 x = *reinterpret_cast<const float4*>(m + r * C + 4 * (int64_t)si);
    const float4 y = *reinterpret_cast<const float4*>(m + r * C + 4 * (int64_t)sj);
    const float a[8] = {fabsf(x.x), fabsf(x.y), fabsf(x.z), fabsf(x.w), fabsf(y.x), fabsf(y.y), fabsf(y.z), fabsf(y.w)};
    accumulate_splits<0>(a, acc);
  }
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
#pragma unroll
  for (int s = 0; s < kStripeSplits; ++s) {
    const float v = wave_sum(acc[s]);
    if (lane == 0) red[w][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < kStripeSplits) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) v += red[k][threadIdx.x];
    red[0][threadIdx.x] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float base = red[0][0];
    float best = 0.f;
    int bi = 0;
    for (int s = 1; s < kStripeSplits; ++s) {
      const float g = red[0][s] - base;
      if (g > best) { best = g; bi = s; }
    }
    gain[p] = best;
    split[p] = bi;
  }
}

__global__ __launch_bounds__(kBlock) void k_sum24_part(const float* __restrict__ m, int64_t groups,
                                                       float* __restrict__ part) {
  __shared__ float smem[kWaves];
  float acc = 0.f;
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += (int64_t)gridDim.x * kBlock) {
    const float4 x = *reinterpret_cast<const float4*>(m + 4 * g);
    acc += top2(fabsf(x.x), fabsf(x.y), fabsf(x.z), fabsf(x.w));
  }
  acc = block_sum(acc, smem);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_sum24_final(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float smem[kWaves];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += kBlock) acc += part[i];
  acc = block_sum(acc, smem);
  if (threadIdx.x == 0) out[0] = acc;
}

}  // namespace

int perm_sum_parts(int64_t R, int64_t C) {
  const int64_t groups = R * (C / 4);
  int64_t b = (groups + kBlock - 1) / kBlock;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 1024));
}

void perm_sum_after_2to4(const float* m, int64_t R, int64_t C, float* part, float* out, hipStream_t st) {
  if (C % 4 != 0) throw std::runtime_error("perm_sum_after_2to4: C must be a multiple of 4");
  const int parts = perm_sum_parts(R, C);
  hipLaunchKernelGGL(k_sum24_part, dim3(parts), dim3(kBlock), 0, st, m, R * (C / 4), part);
  hipLaunchKernelGGL(k_sum24_final, dim3(1), dim3(kBlock), 0, st, part, parts, out);
  check_launch("perm_sum_after_2to4");
}

void perm_stripe_pair_gains(const float* m, int64_t R, int64_t C, const int32_t* pairs, int64_t npairs, float* gain,
                            int32_t* split, hipStream_t st) {
  if (C % 4 != 0) throw std::runtime_error("perm_stripe_pair_gains: C must be a multiple of 4");
  if (npairs == 0) return;
  hipLaunchKernelGGL(k_pair_gains, dim3((unsigned)npairs), dim3(kBlock), 0, st, m, R, C, pairs, gain, split);
  check_launch("perm_stripe_pair_gains");
}

}  // namespace bh
