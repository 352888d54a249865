// Direct 3x3 / stride 1 / pad 1 convolution for NHWC fp16 / bf16 (kernels/conv.hip): the ResNet-50
// bottleneck's middle conv. Implicit GEMM on MFMA 32x32x16: a workgroup owns an 8-row x 32-column
// window of output pixels (several images side by side when W is small) and 64 output channels; per
// 64-channel input chunk the (8+2)-row halo of the window is staged in LDS once and read at all nine
// (r, s) offsets, while the 64x64 weight slice of each offset streams through a double buffer.
// The data gradient of the same conv is this kernel on dY with the flipped, transposed weights, read
// in place from the forward's weight tensor (transposed LDS reads), so no weight copy is made.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

struct Conv3x3Args {
  const void* x = nullptr;  // [N, H, W, C]
  const void* w = nullptr;  // [K, 3, 3, C]
  void* y = nullptr;        // [N, H, W, K]
  int N = 0, H = 0, W = 0, C = 0, K = 0;
};

// true when the kernel covers the shape (C % 64 == 0, K % 64 == 0, 16-byte aligned tensors)
bool conv3x3_supported(const Conv3x3Args& a);
void conv3x3_forward(int dt, const Conv3x3Args& a, hipStream_t st);
// data gradient: a.x = dY [N, H, W, K_w], a.w = the forward weights [K_w, 3, 3, C_w] as they are,
// a.y = dX [N, H, W, C_w]; a.C = K_w (channels read), a.K = C_w (channels written)
void conv3x3_dgrad(int dt, const Conv3x3Args& a, hipStream_t st);

}  // namespace bh
