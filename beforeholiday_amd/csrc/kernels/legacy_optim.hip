// Deprecated `fused_adam_cuda` extension for gfx950: single-tensor / multi-tensor legacy Adam,
// reversible Adam + undo, strided finite check, and the e5m2 byte (de)compression casts used by
// the distributed optimizers' compressed parameter all-gather.
//
// Reference behaviour: apex/contrib/csrc/optimizers/fused_adam_cuda_kernel.cu (adam_cuda_kernel :37,
// strided_check_finite :466-495, maybe_cast_kernel :526, reversible_adam :571, maybe_adam_undo :657)
// and the front-end fused_adam_cuda.cpp:79-85.
//
// Legacy Adam math (differs from amp_C's Adam/AdamW): step_size = lr*sqrt(1-b2^t)/(1-b1^t) (host),
//   m = b1*m + (1-b1)*g/scale ; v = b2*v + (1-b2)*(g/scale)^2
//   denom = sqrt(v + eps) (mode 0) | sqrt(v) + eps (mode 1)
//   p -= step_size * (m/denom + decay*p)
//
// MI355X design: every kernel is a grid-stride loop over 8-element slices (16-byte accesses for the
// aligned 16-bit cases), one 256-thread workgroup = 4 wave64s, grid capped at 8 workgroups per CU; the
// multi-tensor variants run one workgroup per chunk of the shared device-resident plan (bh::MTAView).
// The reversible-Adam overflow marker is written by a second 1-thread kernel from a device flag, so
// p_copy[0] never races with the workgroup that owns element 0.
#include "bh/api.h"
#include "bh/device.h"
#include "bh/legacy_api.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

struct NoCopy {};
struct E5M2 {};  // uint8 storage: the upper byte of an fp16

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// e5m2 <- float: round to nearest by adding half an e5m2 ulp (2^(e-3)) before truncating the fp16
BH_DEVICE uint8_t to_e5m2(float x) {
  union { float f; uint32_t u; } s;
  s.f = x;
  s.u &= 0xFF800000u;  // sign and exponent of x
  const _Float16 h = static_cast<_Float16>(x + s.f * 0.125f);
  return (uint8_t)(__builtin_bit_cast(uint16_t, h) >> 8);
}
BH_DEVICE float from_e5m2(uint8_t b) {
  return static_cast<float>(__builtin_bit_cast(_Float16, (uint16_t)((uint16_t)b << 8)));
}

template <typename T> BH_DEVICE float ldf(const T* p, int64_t i) { return to_f<T>(p[i]); }
template <> BH_DEVICE float ldf<E5M2>(const E5M2* p, int64_t i) {
  return from_e5m2(reinterpret_cast<const uint8_t*>(p)[i]);
}
template <typename T> BH_DEVICE void stf(T* p, int64_t i, float x) { p[i] = from_f<T>(x); }
template <> BH_DEVICE void stf<E5M2>(E5M2* p, int64_t i, float x) { reinterpret_cast<uint8_t*>(p)[i] = to_e5m2(x); }
template <> BH_DEVICE void stf<NoCopy>(NoCopy*, int64_t, float) {}

template <typename A>
struct AdamStep {
  // returns false (and leaves the state alone) when skip_nonfinite and g/scale is not finite
  static BH_DEVICE bool apply(A& p, A& m, A& v, A g, const LegacyAdamArgs& a, bool skip_nonfinite) {
    const A sg = g / (A)a.grad_scale;
    if (skip_nonfinite && !__builtin_isfinite((float)sg)) return false;
    m = (A)a.beta1 * m + (A)(1.f - a.beta1) * sg;
    v = (A)a.beta2 * v + (A)(1.f - a.beta2) * sg * sg;
    const A denom = a.mode == 0 ? sqrt(v + (A)a.eps) : sqrt(v) + (A)a.eps;
    p = p - (A)a.step_size * (m / denom + (A)a.decay * p);
    return true;
  }
};

template <typename P, typename G, typename C>
__global__ __launch_bounds__(kBlock) void k_adam(int64_t n, P* __restrict__ p, C* __restrict__ pc, P* __restrict__ m,
                                                 P* __restrict__ v, const G* __restrict__ g, LegacyAdamArgs a,
                                                 bool reversible, int* overflow) {
  using A = typename Acc<P>::type;
  bool ovf = false;
  for (int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i0 < n; i0 += (int64_t)gridDim.x * kBlock * 4) {
    A pv[4], mv[4], vv[4], gv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k;
      if (i < n) {
        pv[k] = (A)p[i];
        mv[k] = (A)m[i];
        vv[k] = (A)v[i];
        gv[k] = (A)to_f<G>(g[i]);
        if constexpr (sizeof(G) == 8) gv[k] = (A)g[i];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k;
      if (i < n) {
        if (!AdamStep<A>::apply(pv[k], mv[k], vv[k], gv[k], a, reversible)) ovf = true;
        p[i] = (P)pv[k];
        m[i] = (P)mv[k];
        v[i] = (P)vv[k];
        if (pc) stf<C>(pc, i, (float)pv[k]);
      }
    }
  }
  if (ovf && overflow) __hip_atomic_store(overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename C>
__global__ void k_mark_inf(const int* flag, C* pc) {
  if (*flag != 0) stf<C>(pc, 0, INFINITY);
}

template <typename P, typename G>
__global__ __launch_bounds__(kBlock) void k_adam_undo(int64_t n, const int* overflow, P* __restrict__ p,
                                                      P* __restrict__ m, P* __restrict__ v, const G* __restrict__ g,
                                                      LegacyAdamArgs a) {
  if (*overflow == 0) return;  // nothing to undo
  using A = typename Acc<P>::type;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    A gv = (A)to_f<G>(g[i]);
    if constexpr (sizeof(G) == 8) gv = (A)g[i];
    const A sg = gv / (A)a.grad_scale;
    if (!__builtin_isfinite((float)sg)) continue;  // the reversible step skipped this element
    A pv = (A)p[i], mv = (A)m[i], vv = (A)v[i];
    const A denom = a.mode == 0 ? sqrt(vv + (A)a.eps) : sqrt(vv) + (A)a.eps;
    pv = (pv + (A)a.step_size * (mv / denom)) / ((A)1 - (A)a.step_size * (A)a.decay);
    mv = (mv - (A)(1.f - a.beta1) * sg) / (A)a.beta1;
    vv = (vv - (A)(1.f - a.beta2) * sg * sg) / (A)a.beta2;
    vv = vv >= (A)0 ? vv : (A)0;  // round-off when reverting the very first step
    p[i] = (P)pv;
    m[i] = (P)mv;
    v[i] = (P)vv;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_strided_finite(int64_t n, int* flag, const T* x, int stride) {
  bool bad = false;
  for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * stride; i < n;
       i += (int64_t)gridDim.x * kBlock * stride)
    bad |= !__builtin_isfinite(ldf<T>(x, i));
  if (bad) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_clear(int* flag) { *flag = 0; }

template <typename Ti, typename To>
__global__ __launch_bounds__(kBlock) void k_cast(int64_t n, const int* overflow, const Ti* in, To* out) {
  if (overflow && *overflow != 0) return;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    stf<To>(out, i, ldf<Ti>(in, i));
}

// ---- multi-tensor variants (one workgroup per chunk of the plan) ----
template <typename T>
BH_DEVICE T* plan_ptr(const MTAView& v, int d, int t, int64_t base) {
  return reinterpret_cast<T*>(v.ptrs[(int64_t)d * v.T + t]) + base;
}

template <typename P, typename G, typename C>
__global__ __launch_bounds__(kBlock) void k_adam_mt(MTAView view, LegacyAdamArgs a) {
  const int c = blockIdx.x;
  const int t = view.chunk_tensor[c];
  const int64_t base = (int64_t)view.chunk_local[c] * view.chunk;
  const int64_t n = min((int64_t)view.chunk, view.numel[t] - base);
  P* p = plan_ptr<P>(view, 0, t, base);
  P* m = plan_ptr<P>(view, 1, t, base);
  P* v = plan_ptr<P>(view, 2, t, base);
  const G* g = plan_ptr<const G>(view, 3, t, base);
  C* pc = view.depth > 4 ? plan_ptr<C>(view, 4, t, base) : nullptr;
  using A = typename Acc<P>::type;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    A pv = (A)p[i], mv = (A)m[i], vv = (A)v[i];
    A gv = (A)to_f<G>(g[i]);
    if constexpr (sizeof(G) == 8) gv = (A)g[i];
    AdamStep<A>::apply(pv, mv, vv, gv, a, false);
    p[i] = (P)pv;
    m[i] = (P)mv;
    v[i] = (P)vv;
    if (pc) stf<C>(pc, i, (float)pv);
  }
}

template <typename Ti, typename To>
__global__ __launch_bounds__(kBlock) void k_cast_mt(MTAView view, const int* overflow) {
  if (overflow && *overflow != 0) return;
  const int c = blockIdx.x;
  const int t = view.chunk_tensor[c];
  const int64_t base = (int64_t)view.chunk_local[c] * view.chunk;
  const int64_t n = min((int64_t)view.chunk, view.numel[t] - base);
  const Ti* in = plan_ptr<const Ti>(view, 0, t, base);
  To* out = plan_ptr<To>(view, 1, t, base);
  for (int64_t i = threadIdx.x; i < n; i += kBlock) stf<To>(out, i, ldf<Ti>(in, i));
}

// ---- distributed LAMB stages (device-resident scalars; noop-gated) ----
template <typename P, typename G>
__global__ __launch_bounds__(kBlock) void k_distlamb_s1(MTAView view, DistLambStage1Args a, const int* noop) {
  if (*noop != 0) return;  // overflow: leave every state untouched
  const int c = blockIdx.x;
  const int t = view.chunk_tensor[c];
  const int64_t base = (int64_t)view.chunk_local[c] * view.chunk;
  const int64_t n = min((int64_t)view.chunk, view.numel[t] - base);
  const G* g = plan_ptr<const G>(view, 0, t, base);
  const P* p = plan_ptr<const P>(view, 1, t, base);
  P* m = plan_ptr<P>(view, 2, t, base);
  P* v = plan_ptr<P>(view, 3, t, base);
  float* u = plan_ptr<float>(view, 4, t, base);
  const float gs = *a.global_scale;
  float combined = gs;
  if (a.max_grad_norm > 0.f) {
    const float clip = a.max_grad_norm / (*a.global_grad_norm / gs + 1e-6f);
    combined = gs / fminf(1.f, clip);
  }
  const float b1 = a.beta1[t], b2 = a.beta2[t], b3 = a.beta3[t], eps = a.eps[t], decay = a.decay[t];
  float c1 = 1.f, c2 = 1.f;
  if (a.bias_correction[t] == 1) {
    c1 = 1.f - powf(b1, (float)*a.step);
    c2 = 1.f - powf(b2, (float)*a.step);
  }
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    float sg = to_f<G>(g[i]) / combined;
    const float pv = decay != 0.f ? to_f<P>(p[i]) : 0.f;
    if (a.mode == 0) sg += decay * pv;
    const float mv = to_f<P>(m[i]) * b1 + b3 * sg;
    const float vv = to_f<P>(v[i]) * b2 + (1.f - b2) * sg * sg;
    float upd = (mv / c1) / (sqrtf(vv / c2) + eps);
    if (a.mode != 0) upd += decay * pv;
    m[i] = from_f<P>(mv);
    v[i] = from_f<P>(vv);
    u[i] = upd;
  }
}

template <typename P, typename C>
__global__ __launch_bounds__(kBlock) void k_distlamb_s2(MTAView view, DistLambStage2Args a, const int* noop) {
  if (*noop != 0) return;
  const int c = blockIdx.x;
  const int t = view.chunk_tensor[c];
  const int64_t base = (int64_t)view.chunk_local[c] * view.chunk;
  const int64_t n = min((int64_t)view.chunk, view.numel[t] - base);
  P* p = plan_ptr<P>(view, 0, t, base);
  const float* u = plan_ptr<const float>(view, 1, t, base);
  C* pc = view.depth > 2 ? plan_ptr<C>(view, 2, t, base) : nullptr;
  float ratio = *a.lr;
  if (a.use_nvlamb || a.decay[t] != 0.f) {
    const float pn = a.param_norm[t], un = a.update_norm[a.update_norm_offset[t]];
    ratio = (un != 0.f && pn != 0.f) ? *a.lr * (pn / un) : *a.lr;
  }
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const float pv = to_f<P>(p[i]) - ratio * u[i];
    p[i] = from_f<P>(pv);
    if (pc) stf<C>(pc, i, pv);
  }
}

template <typename P, typename G, typename C>
__global__ __launch_bounds__(kBlock) void k_distadam(MTAView view, DistAdamArgs a) {
  const int c = blockIdx.x;
  const int t = view.chunk_tensor[c];
  const int64_t base = (int64_t)view.chunk_local[c] * view.chunk;
  const int64_t n = min((int64_t)view.chunk, view.numel[t] - base);
  P* p = plan_ptr<P>(view, 0, t, base);
  P* m = plan_ptr<P>(view, 1, t, base);
  P* v = plan_ptr<P>(view, 2, t, base);
  const G* g = plan_ptr<const G>(view, 3, t, base);
  C* pc = view.depth > 4 ? plan_ptr<C>(view, 4, t, base) : nullptr;
  const float b1 = a.beta1[t], b2 = a.beta2[t], eps = a.eps[t], decay = a.decay[t];
  float c1 = 1.f, c2 = 1.f;
  if (a.bias_correction[t] == 1) {
    c1 = 1.f - powf(b1, (float)a.step);
    c2 = 1.f - powf(b2, (float)a.step);
  }
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const float sg = to_f<G>(g[i]) / a.grad_scale;
    const float pv = to_f<P>(p[i]);
    const float mv = b1 * to_f<P>(m[i]) + (1.f - b1) * sg;
    const float vv = b2 * to_f<P>(v[i]) + (1.f - b2) * sg * sg;
    const float vh = vv / c2;
    const float denom = a.mode == 0 ? sqrtf(vh + eps) : sqrtf(vh) + eps;
    const float np = pv - a.lr * ((mv / c1) / denom + decay * pv);
    m[i] = from_f<P>(mv);
    v[i] = from_f<P>(vv);
    p[i] = from_f<P>(np);
    if (pc) stf<C>(pc, i, np);
  }
}

int grid_for(int64_t n, int per_thread) {
  const int64_t b = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 256 * 8));
}

#define LG_PARAM(code, T, ...)                                            \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF64: { using T = double; __VA_ARGS__; } break;                  \
    default: throw std::runtime_error("fused_adam_cuda: params must be fp32 or fp64"); \
  }
#define LG_GRAD(code, T, ...)                                             \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    case kF64: { using T = double; __VA_ARGS__; } break;                  \
    default: throw std::runtime_error("fused_adam_cuda: unsupported grad dtype " + std::to_string(code)); \
  }
#define LG_COPY(code, T, ...)                                             \
  switch (code) {                                                         \
    case -1: { using T = NoCopy; __VA_ARGS__; } break;                    \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    case kU8: { using T = E5M2; __VA_ARGS__; } break;                     \
    default: throw std::runtime_error("fused_adam_cuda: unsupported copy dtype " + std::to_string(code)); \
  }
// maybe_cast types: fp32, fp16, bf16, e5m2 byte
#define LG_CAST(code, T, ...)                                             \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    case kU8: { using T = E5M2; __VA_ARGS__; } break;                     \
    default: throw std::runtime_error("maybe_cast: unsupported dtype " + std::to_string(code)); \
  }

}  // namespace

void legacy_adam(int64_t n, int dt_p, void* p, int dt_copy, void* p_copy, void* m, void* v, int dt_g,
                 const void* g, const LegacyAdamArgs& a, hipStream_t s) {
  if (n == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G, LG_COPY(p_copy ? dt_copy : -1, C,
      hipLaunchKernelGGL((k_adam<P, G, C>), dim3(grid_for(n, 4)), dim3(kBlock), 0, s, n, (P*)p, (C*)p_copy, (P*)m,
                         (P*)v, (const G*)g, a, false, nullptr))));
  check_launch("fused_adam_cuda.adam");
}

void legacy_reversible_adam(int64_t n, int dt_p, void* p, int dt_copy, void* p_copy, void* m, void* v,
                            int dt_g, const void* g, const LegacyAdamArgs& a, int* scratch, hipStream_t s) {
  if (n == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G, LG_COPY(p_copy ? dt_copy : -1, C, {
      hipLaunchKernelGGL((k_adam<P, G, C>), dim3(grid_for(n, 4)), dim3(kBlock), 0, s, n, (P*)p, (C*)p_copy, (P*)m,
                         (P*)v, (const G*)g, a, true, scratch);
      if (p_copy) hipLaunchKernelGGL((k_mark_inf<C>), dim3(1), dim3(1), 0, s, (const int*)scratch, (C*)p_copy);
  })));
  check_launch("fused_adam_cuda.reversible_adam");
}

void legacy_adam_mt(const MTAView& view, int dt_g, int dt_p, int dt_copy, const LegacyAdamArgs& a,
                    hipStream_t s) {
  if (view.C == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G, LG_COPY(view.depth > 4 ? dt_copy : -1, C,
      hipLaunchKernelGGL((k_adam_mt<P, G, C>), dim3(view.C), dim3(kBlock), 0, s, view, a))));
  check_launch("fused_adam_cuda.adam_mt");
}

void legacy_adam_undo(int64_t n, const int* overflow, int dt_p, void* p, void* m, void* v, int dt_g,
                      const void* g, const LegacyAdamArgs& a, hipStream_t s) {
  if (n == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G,
      hipLaunchKernelGGL((k_adam_undo<P, G>), dim3(grid_for(n, 1)), dim3(kBlock), 0, s, n, overflow, (P*)p, (P*)m,
                         (P*)v, (const G*)g, a)));
  check_launch("fused_adam_cuda.maybe_adam_undo");
}

void strided_check_finite(int64_t n, int* flag, int dt, const void* x, int stride, bool clear_first,
                          hipStream_t s) {
  if (clear_first) hipLaunchKernelGGL(k_clear, dim3(1), dim3(1), 0, s, flag);
  if (n == 0) return;
  if (stride < 1) throw std::runtime_error("strided_check_finite: stride must be >= 1");
  LG_CAST(dt, T,
      hipLaunchKernelGGL((k_strided_finite<T>), dim3(grid_for((n + stride - 1) / stride, 1)), dim3(kBlock), 0, s, n,
                         flag, (const T*)x, stride));
  check_launch("fused_adam_cuda.strided_check_finite");
}

void maybe_cast(int64_t n, const int* overflow, int dt_in, const void* in, int dt_out, void* out, hipStream_t s) {
  if (n == 0) return;
  LG_CAST(dt_in, Ti, LG_CAST(dt_out, To,
      hipLaunchKernelGGL((k_cast<Ti, To>), dim3(grid_for(n, 1)), dim3(kBlock), 0, s, n, overflow, (const Ti*)in,
                         (To*)out)));
  check_launch("fused_adam_cuda.maybe_cast");
}

void maybe_cast_mt(const MTAView& view, const int* overflow, int dt_in, int dt_out, hipStream_t s) {
  if (view.C == 0) return;
  LG_CAST(dt_in, Ti, LG_CAST(dt_out, To,
      hipLaunchKernelGGL((k_cast_mt<Ti, To>), dim3(view.C), dim3(kBlock), 0, s, view, overflow)));
  check_launch("fused_adam_cuda.maybe_cast_mt");
}

void distopt_adam(const MTAView& view, int dt_p, int dt_g, int dt_copy, const DistAdamArgs& a, hipStream_t s) {
  if (view.C == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G, LG_COPY(view.depth > 4 ? dt_copy : -1, C,
      hipLaunchKernelGGL((k_distadam<P, G, C>), dim3(view.C), dim3(kBlock), 0, s, view, a))));
  check_launch("distributed_adam_cuda.multi_tensor_fused_adam");
}

void distopt_lamb_stage1(const MTAView& view, int dt_g, int dt_p, const DistLambStage1Args& a, const int* noop,
                         hipStream_t s) {
  if (view.C == 0) return;
  LG_PARAM(dt_p, P, LG_GRAD(dt_g, G,
      hipLaunchKernelGGL((k_distlamb_s1<P, G>), dim3(view.C), dim3(kBlock), 0, s, view, a, noop)));
  check_launch("distributed_lamb_cuda.multi_tensor_lamb_compute_update_term");
}

void distopt_lamb_stage2(const MTAView& view, int dt_p, int dt_copy, const DistLambStage2Args& a, const int* noop,
                         hipStream_t s) {
  if (view.C == 0) return;
  LG_PARAM(dt_p, P, LG_COPY(view.depth > 2 ? dt_copy : -1, C,
      hipLaunchKernelGGL((k_distlamb_s2<P, C>), dim3(view.C), dim3(kBlock), 0, s, view, a, noop)));
  check_launch("distributed_lamb_cuda.multi_tensor_lamb_update_weights");
}

}  // namespace bh
