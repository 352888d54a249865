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

enum ConvEpi { kConvEpiPlain = 0, kConvEpiStats = 1, kConvEpiBwd = 2, kConvEpiAffine = 3 };

struct Conv3x3Args {
  const void* x = nullptr;  // [N, H, W, C]
  const void* w = nullptr;  // [K, 3, 3, C]
  void* y = nullptr;        // [N, H, W, K]
  int N = 0, H = 0, W = 0, C = 0, K = 0;
  // forward only: BatchNorm + ReLU of the producing layer applied to x as it is staged (C <= 512)
  const float* pro_scale = nullptr;
  const float* pro_shift = nullptr;
  // per-workgroup partial statistics per output channel, part [2][G][K], G = conv3x3_parts():
  //   kConvEpiStats (forward): sums of (y - kshift) and (y - kshift)^2 of y as stored;
  //   kConvEpiBwd (data gradient): with yb = by (the previous BatchNorm's raw input, [N, H, W, K]),
  //     dz = y * (yb * bscale + bshift > 0): sums of dz and dz * (yb - bmean)
  int epi = kConvEpiPlain;
  float* part = nullptr;
  const float* kshift = nullptr;
  const void* by = nullptr;
  const float* bscale = nullptr;
  const float* bshift = nullptr;
  const float* bmean = nullptr;
  bool brelu = true;
  // forward kConvEpiAffine: y = relu?(acc * a_scale[k] + a_shift[k] (+ r)) (* r when r_mul), r [N, H, W, K]
  const float* a_scale = nullptr;
  const float* a_shift = nullptr;
  const void* r = nullptr;
  bool relu = false;
  bool r_mul = false;
};

// true when the kernel covers the shape (C % 64 == 0, K % 64 == 0, 16-byte aligned tensors)
bool conv3x3_supported(const Conv3x3Args& a);
void conv3x3_forward(int dt, const Conv3x3Args& a, hipStream_t st);
// data gradient: a.x = dY [N, H, W, K_w], a.w = the forward weights [K_w, 3, 3, C_w] as they are,
// a.y = dX [N, H, W, C_w]; a.C = K_w (channels read), a.K = C_w (channels written)
void conv3x3_dgrad(int dt, const Conv3x3Args& a, hipStream_t st);
// partial rows G of the statistics epilogues for this shape
int conv3x3_parts(const Conv3x3Args& a);

// Weight gradient of a stride-1 "same" R x R convolution (R = 1 or 3, pad (R-1)/2), kernels/conv_wgrad.hip:
// out[k][r][s][c] = sum over pixels of dy[n, y, x, k] * x[n, y + r - P, x + s - P, c].
struct ConvWgradArgs {
  const void* x = nullptr;   // [N, stride H, stride W, C]
  const void* dy = nullptr;  // [N, H, W, K]
  void* out = nullptr;       // [K, R, R, C]
  int N = 0, H = 0, W = 0, C = 0, K = 0, R = 3;
  int stride = 1;            // 2: 1x1 / stride-2 convolution (R = 1; dY pixel (y, x) reads x pixel (2y, 2x))
  int wout = 0;              // set by the launcher: the real output width of a flattened 1x1 problem
  // optional BatchNorm + ReLU prologue on x (fp32 [C] each, stride 1 only): the weight gradient of a
  // convolution whose input relu(x * pro_scale + pro_shift) was never materialised
  const float* pro_scale = nullptr;
  const float* pro_shift = nullptr;
};
struct ConvWgradGeo {
  int G4 = 0, TH = 0, ksteps = 0, wpi = 0, nwin = 0, ctiles = 0, tiles = 0, wpw = 0, splits = 0, grid = 0, kt = 1, ct = 1, parts = 0;
  bool wide = false;  // 1x1: 256 x 128 tiles, 64-pixel windows
  // set by the caller after conv_wgrad_plan: every split (even a single one) writes fp32 partials to ws,
  // never the 16-bit `out` (the BatchNorm fold combines the raw fp32 product, bh/bn_fold_api.h)
  bool f32 = false;
};
// false when the kernel does not cover the shape (C, K % 64, 16-byte alignment, window fits in LDS)
bool conv_wgrad_plan(const ConvWgradArgs& a, ConvWgradGeo* geo);
// fp32 elements of split partials the launch needs (0: the kernel writes `out` directly)
int64_t conv_wgrad_workspace(const ConvWgradGeo& g, const ConvWgradArgs& a);
// reduce = false: only the partials kernel; conv_wgrad_reduce then sums the g.parts split partials
// of ws into a.out (possibly on another stream: the weight gradient is off the critical path)
void conv_wgrad(int dt, const ConvWgradArgs& a, const ConvWgradGeo& g, float* ws, hipStream_t st, bool reduce = true);
void conv_wgrad_reduce(int dt, const float* ws, void* out, int64_t n, int parts, hipStream_t st);

// ResNet stem forward (kernels/conv_stem.hip): 7x7 / stride 2 / pad 3, C = 3 -> K = 64, 224x224 NHWC
// x [N, 224, 224, 3], w [64, 7, 7, 3], y [N, 112, 112, 64]
bool conv_stem_supported(int N, int C, int H, int W, int K);
// part (optional, fp32 [2][conv_stem_parts(N)][64]): BatchNorm statistics partials of the output about
// kshift (fp32 [64] or null), see kernels/conv_stem.hip
int conv_stem_parts(int N);
void conv_stem_forward(int dt, const void* x, const void* w, void* y, int N, hipStream_t st,
                       const float* kshift = nullptr, float* part = nullptr);
// its weight gradient: out [64, 7, 7, 3] from x and dy [N, 112, 112, 64]; ws holds
// conv_stem_wgrad_parts(N) * 9408 fp32 partials
int conv_stem_wgrad_parts(int N);
void conv_stem_wgrad(int dt, const void* x, const void* dy, void* out, float* ws, int N, hipStream_t st);

}  // namespace bh
