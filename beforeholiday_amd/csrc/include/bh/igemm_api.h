// Implicit-GEMM NHWC convolution (kernels/conv_igemm.hip) for the ResNet-50 convolutions the direct
// stride-1 kernel (kernels/conv.hip) does not cover: the stride-2 3x3 convolutions of the three
// downsampling blocks -- forward, and data gradient as four stride-1 "phase" convolutions.
//
// One launch computes, for every phase z < nphase and every pixel (n, i, j) of the Hg x Wg grid,
//   y[n, i so + py_z, j so + px_z, o] = sum_{t < ntaps_z} sum_c a[n, i sa + oy_zt, j sa + ox_zt, c] *
//                                        b[o, tap_zt, c]
// with a pixels outside the Ha x Wa image read as zero (the convolution's padding). b is a KRSC weight
// tensor [Nout][taps_total][Ca]. Optional: a BatchNorm + ReLU prologue on a (relu(a * scale + shift)
// of in-image pixels; the padding stays zero) and the next BatchNorm's statistics partials in the
// epilogue (phase 0 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// (int tables: the kernel indexes them with a uniform runtime tap, which the compiler turns into
// scalar s_load_dword from the kernel arguments; byte tables became vector global_load_ubyte + a
// vmcnt wait on every k-step)
struct IgemmPhase {
  int ntaps = 0, py = 0, px = 0;
  int oy[9] = {}, ox[9] = {};
  int tap[9] = {};
};

struct IgemmArgs {
  const void* a = nullptr;  // [N, Ha, Wa, Ca]
  const void* b = nullptr;  // [Nout, taps_total, Ca]
  void* y = nullptr;        // [N, Hy, Wy, Nout]
  int N = 0, Ha = 0, Wa = 0, Ca = 0, Nout = 0, taps_total = 9;
  int Hg = 0, Wg = 0, sa = 1;   // output grid and its stride into a
  int Hy = 0, Wy = 0, so = 1;   // written image and the grid's stride into it
  int nphase = 1;
  IgemmPhase ph[4];
  const float* pro_scale = nullptr;  // [Ca] (Ca <= 512)
  const float* pro_shift = nullptr;
  // statistics epilogue (nphase == 1): part [2][igemm_parts()][Nout] sums of (y - kshift), (y - kshift)^2
  float* part = nullptr;
  const float* kshift = nullptr;
};

bool igemm_supported(const IgemmArgs& a);
int igemm_parts(const IgemmArgs& a);
void igemm_run(int dt, const IgemmArgs& a, hipStream_t st);

// the two ResNet uses, as argument builders
// forward of conv2d(x, w, stride 2, padding 1), x [N, H, W, C] (H, W even), w [K, 3, 3, C], y [N, H/2, W/2, K]
IgemmArgs igemm_conv3x3_s2_fwd(const void* x, const void* w, void* y, int N, int H, int W, int C, int K);
// its data gradient: dy [N, H/2, W/2, K], wt = the weights as [C, 3, 3, K] (w transposed in/out),
// dx [N, H, W, C]
IgemmArgs igemm_conv3x3_s2_dgrad(const void* dy, const void* wt, void* dx, int N, int H, int W, int C, int K);

}  // namespace bh
