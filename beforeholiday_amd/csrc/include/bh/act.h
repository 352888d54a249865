// Activation functions and their derivatives shared by the dense epilogue kernels
// (kernels/dense.hip) and the MFMA GEMM epilogues (kernels/gemm.hip).
#pragma once

#include "bh/dense_api.h"
#include "bh/device.h"

namespace bh {

BH_DEVICE float act_f(float v, int act) {
  switch (act) {
    case kActRelu: return fmaxf(v, 0.f);
    case kActSigmoid: return 1.f / (1.f + __expf(-v));
    case kActGelu: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    case kActGeluTanh: {
      const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      return 0.5f * v * (1.f + tanhf(u));
    }
    default: return v;
  }
}

// derivative given aux: ReLU/sigmoid take the activation OUTPUT, GELU the pre-activation
BH_DEVICE float act_d(float a, int act) {
  switch (act) {
    case kActRelu: return a > 0.f ? 1.f : 0.f;
    case kActSigmoid: return a * (1.f - a);
    case kActGelu: {
      const float cdf = 0.5f * (1.f + erff(a * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * a * a);
      return cdf + a * pdf;
    }
    case kActGeluTanh: {
      const float k = 0.7978845608028654f;
      const float u = k * (a + 0.044715f * a * a * a);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * a * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * a * a);
    }
    default: return 1.f;
  }
}

}  // namespace bh
