// Max pooling for NHWC (channels_last) activations, optionally fused with the preceding batch-norm
// affine + ReLU (ResNet stem: conv1 -> bn1 -> relu -> maxpool 3x3/2).
//
// Reference behaviour: torch.nn.MaxPool2d (first maximum of the window in row-major order wins,
// NaN propagates), and apex's fused BN+ReLU (csrc/welford.cu batchnorm_forward_c_last :633).
//
// MI355X design:
//  * a thread owns 8 consecutive channels of one output pixel: 16-byte loads of fp16/bf16, the window
//    is read straight from HBM/L2 (each input pixel is shared by <= 4 windows, so the cache absorbs
//    the overlap) -- no LDS staging needed for a 3x3 window.
//  * fused with BN: y = max(relu(x*scale + shift)) is computed in fp32 from the conv output, so the
//    normalised [N,H,W,C] activation is never written (the backward recomputes the ReLU mask from x).
//  * the argmax is stored as a uint8 window offset per (pixel, channel): 1 byte instead of torch's
//    int64 index, i.e. 1/8 of the index traffic.
//  * backward is a gather (one thread per input pixel x 8 channels walks the <= ceil(k/s)^2 windows
//    that contain it): deterministic, no atomics, no zero-fill pass.
#include "bh/api.h"
#include "bh/device.h"
#include "bh/pool_api.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// I: index type -- uint32_t when every element offset of the launch fits (the ResNet stem: 205 M
// elements), which turns the per-thread 64-bit divisions of the pixel decomposition into 32-bit ones
template <typename T, typename I>
__global__ __launch_bounds__(kBlock) void k_maxpool_fwd_nhwc(PoolArgs a, const T* __restrict__ x,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, T* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int64_t* counter) {
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) *counter += 1;
  const I cv = (I)(a.C / 8);
  const I total = (I)a.N * a.OH * a.OW * cv;
  const I t = (I)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  I p = t / cv;
  const int ow = (int)(p % (I)a.OW);
  p /= (I)a.OW;
  const int oh = (int)(p % (I)a.OH);
  const int n = (int)(p / (I)a.OH);
  float sc[8], sh[8];
  const bool bn = scale != nullptr;
  if (bn) {
    VecIO<float>::load(scale + c0, sc);
    VecIO<float>::load(shift + c0, sh);
  }
  float best[8];
  int bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    best[j] = -INFINITY;
    bi[j] = 0;
  }
  const int hs = oh * a.stride - a.pad, ws = ow * a.stride - a.pad;
  for (int kh = 0; kh < a.k; ++kh) {
    const int ih = hs + kh;
    if (ih < 0 || ih >= a.H) continue;
    for (int kw = 0; kw < a.k; ++kw) {
      const int iw = ws + kw;
      if (iw < 0 || iw >= a.W) continue;
      float v[8];
      VecIO<T>::load(x + (((I)n * a.H + ih) * a.W + iw) * a.C + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float u = v[j];
        if (bn) u = fmaf(u, sc[j], sh[j]);
        if (a.relu) u = fmaxf(u, 0.f);
        if (u > best[j] || isnan(u)) {
          best[j] = u;
          bi[j] = kh * a.k + kw;
        }
      }
    }
  }
  const I o = (((I)n * a.OH + oh) * a.OW + ow) * a.C + c0;
  VecIO<T>::store(y + o, best);
  if (idx) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo |= (uint32_t)bi[j] << (8 * j);
      hi |= (uint32_t)bi[4 + j] << (8 * j);
    }
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
  }
}

template <typename T, typename I>
__global__ __launch_bounds__(kBlock) void k_maxpool_bwd_nhwc(PoolArgs a, const T* __restrict__ gy,
                                                             const uint8_t* __restrict__ idx, T* __restrict__ gx) {
  const I cv = (I)(a.C / 8);
  const I total = (I)a.N * a.H * a.W * cv;
  const I t = (I)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  I p = t / cv;
  const int iw = (int)(p % (I)a.W);
  p /= (I)a.W;
  const int ih = (int)(p % (I)a.H);
  const int n = (int)(p / (I)a.H);
  // windows containing ih: oh*s - pad <= ih <= oh*s - pad + k - 1
  const int oh0 = max(0, (ih + a.pad - a.k + a.stride) / a.stride);
  const int oh1 = min(a.OH - 1, (ih + a.pad) / a.stride);
  const int ow0 = max(0, (iw + a.pad - a.k + a.stride) / a.stride);
  const int ow1 = min(a.OW - 1, (iw + a.pad) / a.stride);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int oh = oh0; oh <= oh1; ++oh) {
    const int kh = ih - (oh * a.stride - a.pad);
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int want = kh * a.k + iw - (ow * a.stride - a.pad);
      const I o = (((I)n * a.OH + oh) * a.OW + ow) * a.C + c0;
      const uint2 id = *reinterpret_cast<const uint2*>(idx + o);
      float g[8];
      VecIO<T>::load(gy + o, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = j < 4 ? id.x : id.y;
        if ((int)((w >> (8 * (j & 3))) & 0xffu) == want) acc[j] += g[j];
      }
    }
  }
  VecIO<T>::store(gx + (((I)n * a.H + ih) * a.W + iw) * a.C + c0, acc);
}

#define POOL_DISPATCH(code, T, ...)                                        \
  switch (code) {                                                          \
    case kF32: { using T = float; __VA_ARGS__; } break;                    \
    case kF16: { using T = f16; __VA_ARGS__; } break;                      \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("maxpool: unsupported dtype " + std::to_string(code)); \
  }

int blocks_for(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

void maxpool_forward_nhwc(const PoolArgs& a, int dt, const void* x, const float* scale, const float* shift, void* y,
                          uint8_t* idx, int64_t* counter, hipStream_t st) {
  if (a.C % 8 != 0 || a.k * a.k > 255) throw std::runtime_error("maxpool_forward_nhwc: needs C % 8 == 0, k*k <= 255");
  const int64_t total = (int64_t)a.N * a.OH * a.OW * (a.C / 8);
  if (total == 0) return;
  const bool i32 = (int64_t)a.N * a.H * a.W * a.C < (1ll << 31);  // input is the larger tensor
  POOL_DISPATCH(dt, T,
      if (i32) hipLaunchKernelGGL((k_maxpool_fwd_nhwc<T, uint32_t>), dim3(blocks_for(total)), dim3(kBlock), 0, st, a,
                                  (const T*)x, scale, shift, (T*)y, idx, counter);
      else hipLaunchKernelGGL((k_maxpool_fwd_nhwc<T, int64_t>), dim3(blocks_for(total)), dim3(kBlock), 0, st, a,
                              (const T*)x, scale, shift, (T*)y, idx, counter));
  check_launch("maxpool_forward_nhwc");
}

void maxpool_backward_nhwc(const PoolArgs& a, int dt, const void* gy, const uint8_t* idx, void* gx, hipStream_t st) {
  if (a.C % 8 != 0) throw std::runtime_error("maxpool_backward_nhwc: needs C % 8 == 0");
  const int64_t total = (int64_t)a.N * a.H * a.W * (a.C / 8);
  if (total == 0) return;
  const bool i32 = (int64_t)a.N * a.H * a.W * a.C < (1ll << 31);
  POOL_DISPATCH(dt, T,
      if (i32) hipLaunchKernelGGL((k_maxpool_bwd_nhwc<T, uint32_t>), dim3(blocks_for(total)), dim3(kBlock), 0, st, a,
                                  (const T*)gy, idx, (T*)gx);
      else hipLaunchKernelGGL((k_maxpool_bwd_nhwc<T, int64_t>), dim3(blocks_for(total)), dim3(kBlock), 0, st, a,
                              (const T*)gy, idx, (T*)gx));
  check_launch("maxpool_backward_nhwc");
}

}  // namespace bh
