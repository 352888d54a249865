// Activation functions and their derivatives shared by the dense epilogue kernels
// (kernels/dense.hip) and the MFMA GEMM epilogues (kernels/gemm.hip).
#pragma once

#include "bh/dense_api.h"
#include "bh/device.h"

namespace bh {

// erf(x) given ex2 = exp(-x * x) (Abramowitz & Stegun 7.1.26, |error| < 1.5e-7): one reciprocal,
// one exponential and a degree-5 polynomial instead of ocml's branchy erff - the GELU epilogues run
// it once per output element. GELU's derivative reuses the same exponential for its pdf term.
BH_DEVICE float erf_given_exp(float x, float ex2) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(x), 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  return copysignf(fmaf(-poly, ex2, 1.f), x);
}
BH_DEVICE float gelu_erf(float v) {
  const float x = v * 0.70710678118654752f;
  return 0.5f * v * (1.f + erf_given_exp(x, __expf(-x * x)));
}
BH_DEVICE float dgelu_erf(float a) {
  const float x = a * 0.70710678118654752f;
  const float e = __expf(-x * x);  // = exp(-a^2 / 2)
  return 0.5f * (1.f + erf_given_exp(x, e)) + a * 0.3989422804014327f * e;
}

BH_DEVICE float act_f(float v, int act) {
  switch (act) {
    case kActRelu: return fmaxf(v, 0.f);
    case kActSigmoid: return 1.f / (1.f + __expf(-v));
    case kActGelu: return gelu_erf(v);
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
    case kActGelu: return dgelu_erf(a);
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
