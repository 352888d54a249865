// NHWC max pooling (kernels/pool.hip), optionally fused with a preceding per-channel affine
// (batch-norm scale/shift) and ReLU. Window argmax is kept as a uint8 offset kh*k + kw.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

struct PoolArgs {
  int N = 0, H = 0, W = 0, C = 0, OH = 0, OW = 0;
  int k = 3, stride = 2, pad = 1;
  bool relu = false;
};

// y[N,OH,OW,C] = max over the window of (relu)(x*scale + shift) (scale/shift may be null);
// idx (may be null) gets the argmax offsets; counter (may be null) is incremented once.
void maxpool_forward_nhwc(const PoolArgs& a, int dt, const void* x, const float* scale, const float* shift, void* y,
                          uint8_t* idx, int64_t* counter, hipStream_t st);
// gx[N,H,W,C] = sum over windows whose argmax is this pixel of gy
void maxpool_backward_nhwc(const PoolArgs& a, int dt, const void* gy, const uint8_t* idx, void* gx, hipStream_t st);

}  // namespace bh
