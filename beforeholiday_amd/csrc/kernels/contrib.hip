// contrib kernels (gfx950): sigmoid focal loss, index_mul_2d.
//
// Reference behaviour: apex/contrib/csrc/focal_loss/focal_loss_cuda_kernel.cu (loss + cached partial
// gradient, rows labelled -2 ignored, classes >= num_real_classes padding, label smoothing) and
// apex/contrib/csrc/index_mul_2d/index_mul_2d_cuda_kernel.cu (out = in1[idx] * in2 with scatter-add
// gradients and a double-backward).
//
// MI355X design:
//  * focal loss: one pass writes the partial gradient and a per-workgroup loss partial; a second
//    one-workgroup kernel sums the partials in a fixed order (deterministic: the reference
//    atomically adds block sums into the loss). Backward scales the cached gradient in place.
//  * index_mul_2d: rows are independent; one thread per element, grid-stride, 4 elements in flight
//    per thread. The scatter-add into in1's gradient uses hardware fp32 atomics (fp16 gradients are
//    accumulated in an fp32 buffer and converted once).
#include "bh/api.h"
#include "bh/contrib_api.h"
#include "bh/device.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

#define CT_DISPATCH(code, T, ...)                                          \
  switch (code) {                                                          \
    case kF32: { using T = float; __VA_ARGS__; } break;                    \
    case kF16: { using T = f16; __VA_ARGS__; } break;                      \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("contrib: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline unsigned grid_for(int64_t n, int per_thread = 1, int cap = 16384) {
  int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ------------------------------------------------------------------------------------------
// focal loss
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_focal_fwd(const T* __restrict__ x, const int64_t* __restrict__ y,
                                                      T* __restrict__ pgrad, float* __restrict__ part,
                                                      int64_t rows, int C, int real_C, float alpha, float gamma,
                                                      float smoothing) {
  __shared__ float red[kBlock / kWave];
  const float nn_n = 1.f - smoothing * 0.5f, np_n = smoothing * 0.5f;
  const float pn_n = smoothing - smoothing * 0.5f, pp_n = 1.f - smoothing + smoothing * 0.5f;
  const int64_t total = rows * (int64_t)C;
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / C;
    const int c = (int)(i - r * C);
    const int64_t lab = y[r];
    if (lab == -2 || c >= real_C) {
      pgrad[i] = from_f<T>(0.f);
      continue;
    }
    const float p = to_f<T>(x[i]);
    const float sigma = 1.f / (1.f + __expf(-p));
    const float off_a = fmaxf(-p, 0.f) + log1pf(__expf(-fabsf(p)));  // softplus(-p) = -log(sigmoid(p))
    float base, off_b, f1, f2, b1, b2;
    if (lab >= 0 && c == lab) {
      base = smoothing > 0.f ? pn_n * p : 0.f;
      off_b = (smoothing > 0.f ? pp_n : 1.f) - sigma;
      f1 = alpha; f2 = 1.f - sigma; b1 = -gamma; b2 = sigma;
    } else {
      base = smoothing > 0.f ? nn_n * p : p;
      off_b = (smoothing > 0.f ? np_n : 0.f) - sigma;
      f1 = 1.f - alpha; f2 = sigma; b1 = gamma; b2 = 1.f - sigma;
    }
    const float cf = f1 * powf(f2, gamma);
    const float t = base + off_a;
    acc += cf * t;
    pgrad[i] = from_f<T>(cf * (b1 * b2 * t - off_b));
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_focal_finalize(const float* __restrict__ part, int n,
                                                           const float* __restrict__ num_pos,
                                                           float* __restrict__ loss) {
  __shared__ float red[kBlock / kWave];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += kBlock) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) loss[0] = s / num_pos[0];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_focal_bwd(T* __restrict__ g, const float* __restrict__ gout,
                                                      const float* __restrict__ num_pos, int64_t n) {
  const float s = gout[0] / num_pos[0];
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    g[i] = from_f<T>(to_f<T>(g[i]) * s);
}

// ------------------------------------------------------------------------------------------
// index_mul_2d: out[i, f] = in1[idx[i], f] * in2[i, f]
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_imul_fwd(T* __restrict__ out, const T* __restrict__ in1,
                                                     const T* __restrict__ in2, const int64_t* __restrict__ idx,
                                                     int64_t n, int F) {
  const int64_t total = n * (int64_t)F;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / F;
    const int f = (int)(i - r * F);
    out[i] = from_f<T>(to_f<T>(in1[idx[r] * F + f]) * to_f<T>(in2[i]));
  }
}

// grad_in1 (fp32 accumulation buffer) += scatter(g * in2); grad_in2 = g * in1[idx]
template <typename T>
__global__ __launch_bounds__(kBlock) void k_imul_bwd(float* __restrict__ acc1, T* __restrict__ gin2,
                                                     const T* __restrict__ gout, const T* __restrict__ in1,
                                                     const T* __restrict__ in2, const int64_t* __restrict__ idx,
                                                     int64_t n, int F) {
  const int64_t total = n * (int64_t)F;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / F;
    const int f = (int)(i - r * F);
    const int64_t j = idx[r] * F + f;
    const float g = to_f<T>(gout[i]);
    atomicAdd(acc1 + j, g * to_f<T>(in2[i]));
    gin2[i] = from_f<T>(g * to_f<T>(in1[j]));
  }
}

// double backward: ggo = gg1[idx] * in2 + gg2 * in1[idx]; gin1 += scatter(gg2 * g); gin2 = gg1[idx] * g
template <typename T>
__global__ __launch_bounds__(kBlock) void k_imul_bwd_bwd(T* __restrict__ ggo, float* __restrict__ acc1,
                                                         T* __restrict__ gin2, const T* __restrict__ gout,
                                                         const T* __restrict__ gg1, const T* __restrict__ gg2,
                                                         const T* __restrict__ in1, const T* __restrict__ in2,
                                                         const int64_t* __restrict__ idx, int64_t n, int F) {
  const int64_t total = n * (int64_t)F;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / F;
    const int f = (int)(i - r * F);
    const int64_t j = idx[r] * F + f;
    const float g = to_f<T>(gout[i]);
    const float a = to_f<T>(gg1[j]);
    const float b = to_f<T>(gg2[i]);
    ggo[i] = from_f<T>(a * to_f<T>(in2[i]) + b * to_f<T>(in1[j]));
    atomicAdd(acc1 + j, b * g);
    gin2[i] = from_f<T>(a * g);
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_cast_from_f32(const float* __restrict__ src, T* __restrict__ dst,
                                                          int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    dst[i] = from_f<T>(src[i]);
}

}  // namespace

int focal_loss_parts(int64_t numel) { return (int)grid_for(numel, 4, 2048); }

void focal_loss_forward(int dt, const void* x, const int64_t* y, void* pgrad, float* part, int nparts,
                        const float* num_pos, float* loss, int64_t rows, int C, int real_C, float alpha, float gamma,
                        float smoothing, hipStream_t st) {
  CT_DISPATCH(dt, T, hipLaunchKernelGGL((k_focal_fwd<T>), dim3(nparts), dim3(kBlock), 0, st, (const T*)x, y, (T*)pgrad,
                                        part, rows, C, real_C, alpha, gamma, smoothing));
  check_launch("focal_loss_forward");
  hipLaunchKernelGGL(k_focal_finalize, dim3(1), dim3(kBlock), 0, st, part, nparts, num_pos, loss);
  check_launch("focal_loss_finalize");
}

void focal_loss_backward(int dt, void* g, const float* gout, const float* num_pos, int64_t n, hipStream_t st) {
  if (n == 0) return;
  CT_DISPATCH(dt, T, hipLaunchKernelGGL((k_focal_bwd<T>), dim3(grid_for(n, 4)), dim3(kBlock), 0, st, (T*)g, gout,
                                        num_pos, n));
  check_launch("focal_loss_backward");
}

void index_mul_2d_forward(int dt, void* out, const void* in1, const void* in2, const int64_t* idx, int64_t n, int F,
                          hipStream_t st) {
  if (n * (int64_t)F == 0) return;
  CT_DISPATCH(dt, T, hipLaunchKernelGGL((k_imul_fwd<T>), dim3(grid_for(n * (int64_t)F, 4)), dim3(kBlock), 0, st,
                                        (T*)out, (const T*)in1, (const T*)in2, idx, n, F));
  check_launch("index_mul_2d_forward");
}

void index_mul_2d_backward(int dt, float* acc1, void* gin1, int64_t n1, void* gin2, const void* gout, const void* in1,
                           const void* in2, const int64_t* idx, int64_t n, int F, hipStream_t st) {
  CT_DISPATCH(dt, T,
      if (n * (int64_t)F > 0) {
        hipLaunchKernelGGL((k_imul_bwd<T>), dim3(grid_for(n * (int64_t)F, 4)), dim3(kBlock), 0, st, acc1, (T*)gin2,
                           (const T*)gout, (const T*)in1, (const T*)in2, idx, n, F);
        check_launch("index_mul_2d_backward");
      }
      if (gin1 && n1 * (int64_t)F > 0) {
        hipLaunchKernelGGL((k_cast_from_f32<T>), dim3(grid_for(n1 * (int64_t)F, 4)), dim3(kBlock), 0, st, acc1,
                           (T*)gin1, n1 * (int64_t)F);
        check_launch("index_mul_2d_cast");
      });
}

void index_mul_2d_backward_backward(int dt, void* ggo, float* acc1, void* gin1, int64_t n1, void* gin2,
                                    const void* gout, const void* gg1, const void* gg2, const void* in1,
                                    const void* in2, const int64_t* idx, int64_t n, int F, hipStream_t st) {
  CT_DISPATCH(dt, T,
      if (n * (int64_t)F > 0) {
        hipLaunchKernelGGL((k_imul_bwd_bwd<T>), dim3(grid_for(n * (int64_t)F, 4)), dim3(kBlock), 0, st, (T*)ggo, acc1,
                           (T*)gin2, (const T*)gout, (const T*)gg1, (const T*)gg2, (const T*)in1, (const T*)in2, idx,
                           n, F);
        check_launch("index_mul_2d_backward_backward");
      }
      if (gin1 && n1 * (int64_t)F > 0) {
        hipLaunchKernelGGL((k_cast_from_f32<T>), dim3(grid_for(n1 * (int64_t)F, 4)), dim3(kBlock), 0, st, acc1,
                           (T*)gin1, n1 * (int64_t)F);
        check_launch("index_mul_2d_cast");
      });
}

}  // namespace bh
