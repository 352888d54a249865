// Scaled (masked) softmax for attention + softmax cross-entropy, gfx950.
//
// Reference behaviour: csrc/megatron/scaled_masked_softmax.h (forward :211, fully-masked rows -> 0
// :275-303, backward :340), scaled_upper_triang_masked_softmax.h (:114/:233),
// generic_scaled_masked_softmax.h (:66/:190), and apex/contrib/csrc/xentropy/xentropy_kernel.cu.
//
// MI355X design:
//  * one wave64 per row with the row in registers (8 elements / lane / vector) for sk <= 4096:
//    the max and sum reductions are wave reductions, the row is read once and written once.
//  * sk > 4096 (up to any length that fits 256 threads x 8 x 16 registers = 32768): one 256-thread
//    workgroup per row, still register-resident, block reductions through LDS. The reference caps
//    masked rows at sk 4096 and causal at 16384; there is no such cap here.
//  * causal rows only touch columns <= row (the masked tail is written as zeros, never read).
//  * backward dx = scale * y * (dy - sum(dy * y)) in the same layout, in place on dy like the
//    reference (the caller decides whether dx aliases dy).
//  * cross-entropy: one workgroup per row (vocab-sized rows), fp32 log-sum-exp, label smoothing,
//    gradient recomputed from the saved log-sum-exp (no softmax tensor is stored).
#include "bh/api.h"
#include "bh/device.h"
#include "bh/softmax_api.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;
constexpr float kMaskedValue = -10000.f;

#define SM_DISPATCH(code, T, ...)                                         \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    default: throw std::runtime_error("softmax: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
BH_DEVICE void ld8(const T* p, int col, int n, bool vec, float (&r)[8], float fill) {
  if (vec && col + 8 <= n) {
    VecIO<T>::load(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = (col + k < n) ? to_f<T>(p[col + k]) : fill;
  }
}
template <typename T>
BH_DEVICE void st8(T* p, int col, int n, bool vec, const float (&r)[8]) {
  if (vec && col + 8 <= n) {
    VecIO<T>::store(p + col, r);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (col + k < n) p[col + k] = from_f<T>(r[k]);
  }
}

// row geometry: mode 0 none, 1 padding mask [mb, 1, sq, sk] (uint8, 1 = masked), 2 causal
struct RowInfo {
  int valid;          // columns that take part (causal: q+1)
  const uint8_t* m;   // mask row or null
};
BH_DEVICE RowInfo row_info(int64_t row, int mode, int sq, int sk, int heads, int mask_batches, const uint8_t* mask) {
  RowInfo ri{sk, nullptr};
  if (mode == 2) {
    const int q = (int)(row % sq);
    ri.valid = min(q + 1, sk);
  } else if (mode == 1) {
    const int64_t q = row % sq;
    const int64_t b = row / ((int64_t)sq * heads);
    const int64_t mb = mask_batches == 1 ? 0 : b;
    ri.m = mask + (mb * sq + q) * (int64_t)sk;
  }
  return ri;
}

// groups = lanes cooperating on a row: 64 (wave) or 256 (block)
template <int G> BH_DEVICE float grp_max(float v, float* red) {
  if constexpr (G == kWave) return wave_max(v);
  else return block_max(v, red);
}
template <int G> BH_DEVICE float grp_sum(float v, float* red) {
  if constexpr (G == kWave) return wave_sum(v);
  else return block_sum(v, red);
}

// forward: G threads per row, V vectors of 8 per thread
template <typename T, int G, int V>
__global__ __launch_bounds__(kBlock) void k_softmax_fwd(const T* __restrict__ x, const uint8_t* __restrict__ mask,
                                                        T* __restrict__ y, int64_t rows, int sq, int sk, int heads,
                                                        int mask_batches, int mode, float scale, bool vec) {
  __shared__ float red[kBlock / kWave];
  const int t = threadIdx.x % G;
  const int64_t row = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G;
  if (row >= rows) return;  // G == kBlock: grid == rows, never taken for a whole block
  const RowInfo ri = row_info(row, mode, sq, sk, heads, mask_batches, mask);
  const T* xr = x + row * sk;
  float v[V][8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * G + t) * 8;
    ld8(xr, col, ri.valid, vec && ri.valid == sk, v[j], 0.f);
    float mk[8];
    if (ri.m) {
      if (vec && col + 8 <= sk) {
        const uint2 mm = *reinterpret_cast<const uint2*>(ri.m + col);
        const uint32_t w[2] = {mm.x, mm.y};
#pragma unroll
        for (int k = 0; k < 8; ++k) mk[k] = ((w[k >> 2] >> (8 * (k & 3))) & 0xff) ? 1.f : 0.f;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) mk[k] = (col + k < sk) ? (ri.m[col + k] ? 1.f : 0.f) : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float e = v[j][k] * scale;
      if (ri.m && mk[k] != 0.f) e = kMaskedValue;
      if (col + k >= ri.valid) e = -INFINITY;
      v[j][k] = e;
      mx = fmaxf(mx, e);
    }
  }
  mx = grp_max<G>(mx, red);
  // padding mask: a fully-masked row (max == -10000) produces zeros (reference :275-303)
  const bool dead = (ri.m != nullptr) && (mx == kMaskedValue);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float e = (v[j][k] == -INFINITY) ? 0.f : __expf(v[j][k] - mx);
      v[j][k] = e;
      s += e;
    }
  s = grp_sum<G>(s, red);
  const float inv = dead ? 0.f : 1.f / s;
  T* yr = y + row * sk;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * G + t) * 8;
    if (col >= sk) break;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = v[j][k] * inv;
    st8(yr, col, sk, vec, o);
  }
}

// backward: dx = scale * y * (dy - sum(dy*y)); causal rows only reduce over valid columns
template <typename T, int G, int V>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd(const T* __restrict__ dy, const T* __restrict__ y,
                                                        T* __restrict__ dx, int64_t rows, int sq, int sk, int mode,
                                                        float scale, bool vec) {
  __shared__ float red[kBlock / kWave];
  const int t = threadIdx.x % G;
  const int64_t row = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G;
  if (row >= rows) return;
  const int valid = (mode == 2) ? min((int)(row % sq) + 1, sk) : sk;
  float g[V][8], p[V][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * G + t) * 8;
    ld8(dy + row * sk, col, valid, vec && valid == sk, g[j], 0.f);
    ld8(y + row * sk, col, valid, vec && valid == sk, p[j], 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s = fmaf(g[j][k], p[j][k], s);
  }
  s = grp_sum<G>(s, red);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int col = (j * G + t) * 8;
    if (col >= sk) break;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (col + k < valid) ? scale * p[j][k] * (g[j][k] - s) : 0.f;
    st8(dx + row * sk, col, sk, vec, o);
  }
}

// ------------------------------------------------------------------------------------------
// softmax cross entropy with label smoothing (row per block, any vocabulary size)
//   loss = lse - (1-eps) * x[y] - eps * mean(x)
//   dx   = g * (exp(x - lse) - (1-eps) * [j == y] - eps / V)
// ------------------------------------------------------------------------------------------
template <typename T, typename To>
__global__ __launch_bounds__(kBlock) void k_xent_fwd(const T* __restrict__ x, const int64_t* __restrict__ labels,
                                                     To* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                     float smoothing, bool vec) {
  __shared__ float red[kBlock / kWave];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * V;
  float mx = -INFINITY, sx = 0.f;
  for (int col = threadIdx.x * 8; col < V; col += kBlock * 8) {
    float v[8];
    ld8(xr, col, V, vec, v, -INFINITY);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mx = fmaxf(mx, v[k]);
      if (col + k < V) sx += v[k];
    }
  }
  mx = block_max(mx, red);
  sx = block_sum(sx, red);
  float se = 0.f;
  for (int col = threadIdx.x * 8; col < V; col += kBlock * 8) {
    float v[8];
    ld8(xr, col, V, vec, v, -INFINITY);
#pragma unroll
    for (int k = 0; k < 8; ++k) se += __expf(v[k] - mx);
  }
  se = block_sum(se, red);
  if (threadIdx.x == 0) {
    const float lse = mx + __logf(se);
    const int64_t lab = labels[row];
    const float xy = (lab >= 0 && lab < V) ? to_f<T>(xr[lab]) : 0.f;
    loss[row] = from_f<To>(lse - (1.f - smoothing) * xy - smoothing * sx / (float)V);
    lse_out[row] = lse;
  }
}

template <typename T, typename Tg>
__global__ __launch_bounds__(kBlock) void k_xent_bwd(const Tg* __restrict__ gloss, const T* __restrict__ x,
                                                     const float* __restrict__ lse, const int64_t* __restrict__ labels,
                                                     T* __restrict__ dx, int V, float smoothing, bool vec) {
  const int64_t row = blockIdx.x;
  const float g = to_f<Tg>(gloss[row]);
  const float l = lse[row];
  const int64_t lab = labels[row];
  const float u = smoothing / (float)V;
  for (int col = threadIdx.x * 8; col < V; col += kBlock * 8) {
    float v[8];
    ld8(x + row * V, col, V, vec, v, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float tgt = (col + k == lab) ? (1.f - smoothing) : 0.f;
      v[k] = g * (__expf(v[k] - l) - tgt - u);
    }
    st8(dx + row * V, col, V, vec, v);
  }
}


// ------------------------------------------------------------------------------------------
// vocab-parallel cross-entropy partials: ONE pass over this rank's vocab shard per row with an
// online (max, sum-exp) pair, plus the target logit when the target falls in [start, start+V).
// stats[row] = {max, sum exp(x - max), target logit or 0, 0}. Ranks exchange these 16 bytes per row
// with a single all-gather (instead of three full-row all-reduces) and combine them in k_vp_combine.
// ------------------------------------------------------------------------------------------
BH_DEVICE void ms_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_vp_stats(const T* __restrict__ x, const int64_t* __restrict__ target,
                                                     float4* __restrict__ stats, int V, int64_t start, bool vec) {
  __shared__ float red[2 * (kBlock / kWave)];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * V;
  float m = -INFINITY, s = 0.f;
  for (int col = threadIdx.x * 8; col < V; col += kBlock * 8) {
    float v[8];
    ld8(xr, col, V, vec, v, -INFINITY);
    float cm = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) cm = fmaxf(cm, v[k]);
    float cs = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) cs += __expf(v[k] - cm);
    ms_merge(m, s, cm, cs);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, kWave);
    const float s2 = __shfl_xor(s, o, kWave);
    ms_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) {
    red[2 * wid] = m;
    red[2 * wid + 1] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[0], S = red[1];
    for (int w = 1; w < kBlock / kWave; ++w) ms_merge(M, S, red[2 * w], red[2 * w + 1]);
    const int64_t t = target[row] - start;
    const float xt = (t >= 0 && t < V) ? to_f<T>(xr[t]) : 0.f;
    stats[row] = make_float4(M, S, xt, 0.f);
  }
}

// gathered stats [world][rows] -> loss[row] = log(sum_r S_r e^{M_r - M}) + M - sum_r t_r, lse[row]
template <typename To>
__global__ void k_vp_combine(const float4* __restrict__ stats, int world, int64_t rows, To* __restrict__ loss,
                             float* __restrict__ lse) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float M = -INFINITY, S = 0.f, xt = 0.f;
  for (int r = 0; r < world; ++r) {
    const float4 st = stats[(int64_t)r * rows + row];
    ms_merge(M, S, st.x, st.y);
    xt += st.z;
  }
  const float l = M + __logf(S);
  lse[row] = l;
  loss[row] = from_f<To>(l - xt);
}

#define SM_SHAPE_DISPATCH(sk, G, V, ...)                                               \
  if (sk <= 512) { constexpr int G = kWave; constexpr int V = 1; __VA_ARGS__; }        \
  else if (sk <= 1024) { constexpr int G = kWave; constexpr int V = 2; __VA_ARGS__; }  \
  else if (sk <= 2048) { constexpr int G = kWave; constexpr int V = 4; __VA_ARGS__; }  \
  else if (sk <= 4096) { constexpr int G = kWave; constexpr int V = 8; __VA_ARGS__; }  \
  else if (sk <= 8192) { constexpr int G = kBlock; constexpr int V = 4; __VA_ARGS__; } \
  else if (sk <= 16384) { constexpr int G = kBlock; constexpr int V = 8; __VA_ARGS__; } \
  else { constexpr int G = kBlock; constexpr int V = 16; __VA_ARGS__; }

}  // namespace

int softmax_max_sk() { return kBlock * 8 * 16; }

void softmax_forward(int dt, const void* x, const uint8_t* mask, void* y, int64_t rows, int sq, int sk, int heads,
                     int mask_batches, int mode, float scale, bool vec, hipStream_t st) {
  if (rows == 0 || sk == 0) return;
  if (sk > softmax_max_sk()) throw std::runtime_error("softmax: sk too large");
  SM_DISPATCH(dt, T, SM_SHAPE_DISPATCH(sk, G, V,
      const int64_t grid = (rows + (kBlock / G) - 1) / (kBlock / G);
      hipLaunchKernelGGL((k_softmax_fwd<T, G, V>), dim3((unsigned)grid), dim3(kBlock), 0, st, (const T*)x, mask, (T*)y,
                         rows, sq, sk, heads, mask_batches, mode, scale, vec)));
  check_launch("softmax_forward");
}

void softmax_backward(int dt, const void* dy, const void* y, void* dx, int64_t rows, int sq, int sk, int mode,
                      float scale, bool vec, hipStream_t st) {
  if (rows == 0 || sk == 0) return;
  if (sk > softmax_max_sk()) throw std::runtime_error("softmax: sk too large");
  SM_DISPATCH(dt, T, SM_SHAPE_DISPATCH(sk, G, V,
      const int64_t grid = (rows + (kBlock / G) - 1) / (kBlock / G);
      hipLaunchKernelGGL((k_softmax_bwd<T, G, V>), dim3((unsigned)grid), dim3(kBlock), 0, st, (const T*)dy,
                         (const T*)y, (T*)dx, rows, sq, sk, mode, scale, vec)));
  check_launch("softmax_backward");
}

void xentropy_forward(int dt, const void* x, const int64_t* labels, int dt_loss, void* loss, float* lse, int64_t rows,
                      int V, float smoothing, bool vec, hipStream_t st) {
  if (rows == 0) return;
  SM_DISPATCH(dt, T, SM_DISPATCH(dt_loss, To,
      hipLaunchKernelGGL((k_xent_fwd<T, To>), dim3((unsigned)rows), dim3(kBlock), 0, st, (const T*)x, labels, (To*)loss,
                         lse, V, smoothing, vec)));
  check_launch("xentropy_forward");
}

void xentropy_backward(int dt, const void* x, int dt_g, const void* gloss, const float* lse, const int64_t* labels,
                       void* dx, int64_t rows, int V, float smoothing, bool vec, hipStream_t st) {
  if (rows == 0) return;
  SM_DISPATCH(dt, T, SM_DISPATCH(dt_g, Tg,
      hipLaunchKernelGGL((k_xent_bwd<T, Tg>), dim3((unsigned)rows), dim3(kBlock), 0, st, (const Tg*)gloss, (const T*)x,
                         lse, labels, (T*)dx, V, smoothing, vec)));
  check_launch("xentropy_backward");
}

void vocab_xent_stats(int dt, const void* x, const int64_t* target, float* stats, int64_t rows, int V, int64_t start,
                      bool vec, hipStream_t st) {
  if (rows == 0) return;
  SM_DISPATCH(dt, T, hipLaunchKernelGGL((k_vp_stats<T>), dim3((unsigned)rows), dim3(kBlock), 0, st, (const T*)x, target,
                                        (float4*)stats, V, start, vec));
  check_launch("vocab_xent_stats");
}

void vocab_xent_combine(const float* stats, int world, int64_t rows, int dt_loss, void* loss, float* lse,
                        hipStream_t st) {
  if (rows == 0) return;
  const unsigned grid = (unsigned)((rows + kBlock - 1) / kBlock);
  SM_DISPATCH(dt_loss, To, hipLaunchKernelGGL((k_vp_combine<To>), dim3(grid), dim3(kBlock), 0, st,
                                              (const float4*)stats, world, rows, (To*)loss, lse));
  check_launch("vocab_xent_combine");
}

}  // namespace bh
