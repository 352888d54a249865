// Multi-head-attention softmax block (gfx950): mask -> softmax -> dropout, forward and backward.
//
// Reference behaviour: apex/contrib/csrc/multihead_attn/softmax.cuh (dispatch_masked_softmax /
// dispatch_additive_masked_softmax, masked_softmax_dropout_backward) and the python default path
// apex/contrib/multihead_attn/self_multihead_attn_func.py:90-140 (time mask [sq, sk] or key padding
// mask [b, sk] filled with -inf, or an additive [b, sk] mask; dropout after softmax).
//
// MI355X design:
//  * one wave64 per attention row with the row in registers (8 columns per lane per vector,
//    sk <= 4096); reductions are wave shuffles, the scores are read once.
//  * dropout is counter-based (Philox4x32-10 keyed by (seed, row, column/4)), so the keep mask is
//    REGENERATED in backward instead of being stored: the reference keeps a byte mask of the full
//    [b*h, sq, sk] probability tensor.
//  * forward writes the softmax (needed by backward) and the dropped probabilities (input of the
//    P·V GEMM); backward fuses dropout-backward with the softmax backward in one pass.
//  * a fully masked row produces zeros (the reference produces NaN).
#include "bh/api.h"
#include "bh/device.h"
#include "bh/mha_api.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;
constexpr int kRowsPerBlock = kBlock / kWave;

#define MHA_DISPATCH(code, T, ...)                                         \
  switch (code) {                                                          \
    case kF32: { using T = float; __VA_ARGS__; } break;                    \
    case kF16: { using T = f16; __VA_ARGS__; } break;                      \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("mha: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
BH_DEVICE void ld8m(const T* p, int col, int n, bool vec, float (&r)[8], float fill) {
  if (vec && col + 8 <= n) {
    VecIO<T>::load(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = (col + k < n) ? to_f<T>(p[col + k]) : fill;
  }
}
template <typename T>
BH_DEVICE void st8m(T* p, int col, int n, bool vec, const float (&r)[8]) {
  if (vec && col + 8 <= n) {
    VecIO<T>::store(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (col + k < n) p[col + k] = from_f<T>(r[k]);
  }
}

// keep flags for columns col..col+7 of `row` (col % 8 == 0)
BH_DEVICE void keep8(uint64_t seed, uint64_t offset, int64_t row, int col, float p_keep, float (&keep)[8]) {
  Philox ph(seed, (uint64_t)row, offset + (uint64_t)(col >> 2));
  const float4 a = ph.uniform4();
  const float4 b = ph.uniform4();
  keep[0] = a.x <= p_keep; keep[1] = a.y <= p_keep; keep[2] = a.z <= p_keep; keep[3] = a.w <= p_keep;
  keep[4] = b.x <= p_keep; keep[5] = b.y <= p_keep; keep[6] = b.z <= p_keep; keep[7] = b.w <= p_keep;
}

// mask_mode: 0 none, 1 key padding bool [B, sk], 2 additive [B, sk] (dtype Tm), 3 time bool [sq, sk]
template <typename T, typename Tm, int V>
__global__ __launch_bounds__(kBlock) void k_mha_fwd(const T* __restrict__ x, const void* __restrict__ mask,
                                                    T* __restrict__ sm, T* __restrict__ dropped, int64_t rows,
                                                    int sq, int sk, int heads, int mask_mode, float p_drop,
                                                    uint64_t seed, uint64_t offset, bool vec) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
  if (row >= rows) return;
  const int q = (int)(row % sq);
  const int64_t b = row / ((int64_t)sq * heads);
  const uint8_t* bm = nullptr;
  const Tm* am = nullptr;
  if (mask_mode == 1) bm = reinterpret_cast<const uint8_t*>(mask) + b * sk;
  else if (mask_mode == 3) bm = reinterpret_cast<const uint8_t*>(mask) + (int64_t)q * sk;
  else if (mask_mode == 2) am = reinterpret_cast<const Tm*>(mask) + b * sk;
  const T* xr = x + row * sk;
  float v[V][8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * kWave + lane) * 8;
    ld8m(xr, col, sk, vec, v[j], -INFINITY);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = col + k;
      float e = v[j][k];
      if (c < sk) {
        if (bm && bm[c]) e = -INFINITY;
        if (am) e += to_f<Tm>(am[c]);
      }
      v[j][k] = e;
      mx = fmaxf(mx, e);
    }
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float e = (v[j][k] == -INFINITY) ? 0.f : __expf(v[j][k] - mx);
      v[j][k] = e;
      s += e;
    }
  s = wave_sum(s);
  const float inv = (s > 0.f) ? 1.f / s : 0.f;
  const float p_keep = 1.f - p_drop;
  const float kscale = p_keep > 0.f ? 1.f / p_keep : 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * kWave + lane) * 8;
    if (col >= sk) break;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = v[j][k] * inv;
    st8m(sm + row * sk, col, sk, vec, o);
    if (dropped) {
      float keep[8];
      keep8(seed, offset, row, col, p_keep, keep);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] *= keep[k] * kscale;
      st8m(dropped + row * sk, col, sk, vec, o);
    }
  }
}

// dx = y * (g - sum(g * y)),  g = dy * keep / (1 - p)   (dropout regenerated from the seed)
template <typename T, int V>
__global__ __launch_bounds__(kBlock) void k_mha_bwd(const T* __restrict__ dy, const T* __restrict__ sm,
                                                    T* __restrict__ dx, int64_t rows, int sk, float p_drop,
                                                    uint64_t seed, uint64_t offset, bool use_dropout, bool vec) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
  if (row >= rows) return;
  const float p_keep = 1.f - p_drop;
  const float kscale = p_keep > 0.f ? 1.f / p_keep : 0.f;
  float g[V][8], y[V][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * kWave + lane) * 8;
    ld8m(dy + row * sk, col, sk, vec, g[j], 0.f);
    ld8m(sm + row * sk, col, sk, vec, y[j], 0.f);
    if (use_dropout && col < sk) {
      float keep[8];
      keep8(seed, offset, row, col, p_keep, keep);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[j][k] *= keep[k] * kscale;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s = fmaf(g[j][k], y[j][k], s);
  }
  s = wave_sum(s);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * kWave + lane) * 8;
    if (col >= sk) break;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = y[j][k] * (g[j][k] - s);
    st8m(dx + row * sk, col, sk, vec, o);
  }
}

#define MHA_V_DISPATCH(sk, V, ...)                                               \
  if (sk <= 512) { constexpr int V = 1; __VA_ARGS__; }                           \
  else if (sk <= 1024) { constexpr int V = 2; __VA_ARGS__; }                     \
  else if (sk <= 2048) { constexpr int V = 4; __VA_ARGS__; }                     \
  else if (sk <= 4096) { constexpr int V = 8; __VA_ARGS__; }                     \
  else { throw std::runtime_error("mha softmax: sk > 4096 is not supported by the fused kernel"); }

}  // namespace

int mha_max_sk() { return 4096; }

void mha_softmax_dropout_forward(int dt, const void* x, int mask_mode, int dt_mask, const void* mask, void* sm,
                                 void* dropped, int64_t rows, int sq, int sk, int heads, float p_drop, uint64_t seed,
                                 uint64_t offset, bool vec, hipStream_t st) {
  if (rows == 0 || sk == 0) return;
  const unsigned grid = (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  MHA_DISPATCH(dt, T, MHA_V_DISPATCH(sk, V,
      if (mask_mode == 2) {
        MHA_DISPATCH(dt_mask, Tm, hipLaunchKernelGGL((k_mha_fwd<T, Tm, V>), dim3(grid), dim3(kBlock), 0, st,
                                                     (const T*)x, mask, (T*)sm, (T*)dropped, rows, sq, sk, heads,
                                                     mask_mode, p_drop, seed, offset, vec));
      } else {
        hipLaunchKernelGGL((k_mha_fwd<T, float, V>), dim3(grid), dim3(kBlock), 0, st, (const T*)x, mask, (T*)sm,
                           (T*)dropped, rows, sq, sk, heads, mask_mode, p_drop, seed, offset, vec);
      }));
  check_launch("mha_softmax_dropout_forward");
}

void mha_softmax_dropout_backward(int dt, const void* dy, const void* sm, void* dx, int64_t rows, int sk, float p_drop,
                                  uint64_t seed, uint64_t offset, bool use_dropout, bool vec, hipStream_t st) {
  if (rows == 0 || sk == 0) return;
  const unsigned grid = (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  MHA_DISPATCH(dt, T, MHA_V_DISPATCH(sk, V,
      hipLaunchKernelGGL((k_mha_bwd<T, V>), dim3(grid), dim3(kBlock), 0, st, (const T*)dy, (const T*)sm, (T*)dx,
                         rows, sk, p_drop, seed, offset, use_dropout, vec)));
  check_launch("mha_softmax_dropout_backward");
}

}  // namespace bh
