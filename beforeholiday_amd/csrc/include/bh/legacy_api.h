// Launchers of the deprecated `fused_adam_cuda` extension (kernels/legacy_optim.hip).
// Reference API: apex/contrib/csrc/optimizers/fused_adam_cuda.cpp:79-85.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bh/api.h"

namespace bh {

// copy dtype codes: -1 = no copy, kF32 / kF16 / kBF16, kU8 = e5m2 byte (upper byte of an fp16,
// round-to-nearest), as produced for DistributedFusedAdam / DistributedFusedLAMB's compressed
// parameter all-gather.
struct LegacyAdamArgs {
  float beta1, beta2, eps, grad_scale, step_size, decay;
  int mode;  // 0: eps inside the sqrt, 1: eps outside
};

// p -= step_size * (m/denom + decay*p) with m/v updated from g/grad_scale; optional p_copy = p.
void legacy_adam(int64_t n, int dt_p, void* p, int dt_copy, void* p_copy, void* m, void* v, int dt_g,
                 const void* g, const LegacyAdamArgs& a, hipStream_t s);
// same on a multi-tensor plan, lists p, m, v, g [, p_copy] (the reference's order)
void legacy_adam_mt(const MTAView& view, int dt_g, int dt_p, int dt_copy, const LegacyAdamArgs& a, hipStream_t s);
// Adam that leaves (p, m, v) of elements with a non-finite scaled gradient untouched; if any was
// seen and p_copy is given, p_copy[0] = +inf (so the reduced copy carries the overflow). `scratch`:
// one device int (zeroed by the caller).
void legacy_reversible_adam(int64_t n, int dt_p, void* p, int dt_copy, void* p_copy, void* m, void* v,
                            int dt_g, const void* g, const LegacyAdamArgs& a, int* scratch, hipStream_t s);
// exact inverse of one legacy_adam step, applied only when *overflow != 0
void legacy_adam_undo(int64_t n, const int* overflow, int dt_p, void* p, void* m, void* v, int dt_g,
                      const void* g, const LegacyAdamArgs& a, hipStream_t s);
// *flag = 1 if any x[j*stride] is non-finite (u8 decoded as e5m2); clear_first zeroes it first
void strided_check_finite(int64_t n, int* flag, int dt, const void* x, int stride, bool clear_first,
                          hipStream_t s);
// out = cast(in) (f32 / f16 / u8-e5m2 in any combination) unless *overflow != 0
void maybe_cast(int64_t n, const int* overflow, int dt_in, const void* in, int dt_out, void* out,
                hipStream_t s);
void maybe_cast_mt(const MTAView& view, const int* overflow, int dt_in, int dt_out, hipStream_t s);

}  // namespace bh

namespace bh {

// distributed_lamb_cuda (reference: apex/contrib/csrc/optimizers/multi_tensor_distopt_lamb.cpp):
// device-resident hyper-parameters, skipped entirely when *noop != 0 (no host synchronisation).
struct DistLambStage1Args {
  const float *beta1, *beta2, *beta3, *eps, *decay;  // per tensor
  const int* bias_correction;                          // per tensor
  const int* step;                                     // device scalar
  const float* global_scale;                           // device scalar: gradients are divided by it
  const float* global_grad_norm;                       // device scalar (norm of the raw gradients)
  float max_grad_norm;                                 // <= 0: no clipping
  int mode;                                            // 0: L2, 1: decoupled weight decay
};
// lists g, p, m, v, u (u fp32)
void distopt_lamb_stage1(const MTAView& view, int dt_g, int dt_p, const DistLambStage1Args& a, const int* noop,
                         hipStream_t s);
struct DistLambStage2Args {
  const float* param_norm;    // per tensor
  const float* update_norm;   // indexed through update_norm_offset
  const int64_t* update_norm_offset;
  const float* lr;            // device scalar
  const float* decay;         // per tensor
  bool use_nvlamb;
};
// lists p, u [, p_copy] (copy fp16 / bf16 / fp32 / u8-e5m2)
void distopt_lamb_stage2(const MTAView& view, int dt_p, int dt_copy, const DistLambStage2Args& a, const int* noop,
                         hipStream_t s);

}  // namespace bh

namespace bh {

// distributed_adam_cuda.multi_tensor_fused_adam (reference: multi_tensor_distopt_adam_kernel.cu:32-228):
// lists p, m, v, g [, p_copy]; per-tensor beta1 / beta2 / bias_correction / eps / weight_decay;
// denom from the bias-corrected v (eps inside the sqrt for mode 0); p -= lr*(m_hat/denom + wd*p).
struct DistAdamArgs {
  const float *beta1, *beta2, *eps, *decay;
  const int* bias_correction;
  float lr, grad_scale;
  int step, mode;
};
void distopt_adam(const MTAView& view, int dt_p, int dt_g, int dt_copy, const DistAdamArgs& a, hipStream_t s);

}  // namespace bh

