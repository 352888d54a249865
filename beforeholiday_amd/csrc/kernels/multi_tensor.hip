// Multi-tensor-apply kernels for gfx950 (amp_C equivalent).
//
// Reference behaviour: csrc/multi_tensor_{scale,axpby,l2norm,l2norm_mp,l2norm_scale,adam,
// sgd,lamb,lamb_mp,novograd,adagrad,lars}*.cu and the launcher csrc/multi_tensor_apply.cuh.
//
// MI355X design (not a translation):
//  * ONE launch per op regardless of the number of tensors: the (tensor, chunk) schedule is a
//    device-resident plan built and cached by the front-end (bh::MTAView), instead of a
//    by-value kernarg table that is refilled and relaunched every 36-110 tensors.
//  * 256-thread workgroups (4 wave64s), 8 elements per thread per access (16-byte loads for
//    16-bit types, 2x16 B for fp32), fp32 math.
//  * Reductions are deterministic: one partial per chunk, then a per-tensor finalize kernel
//    (no float atomics, bitwise reproducible norms).
//  * LAMB is re-associated: stage 1 fuses the param-norm and update-norm reductions into the
//    moment update, and stage 2 recomputes the update from (p, m, v) instead of round-tripping
//    it through the gradient buffer: 2 streaming passes instead of 4, grads left intact.
#include "bh/api.h"
#include "bh/device.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

struct NoT {};  // absent optional list

#define BH_DISPATCH_FLOAT(code, T, ...)                                   \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    case kF64: { using T = double; __VA_ARGS__; } break;                  \
    default: throw std::runtime_error("multi_tensor: unsupported dtype " + std::to_string(code)); \
  }

// optional copy-out type: -1 (absent), f16, bf16, f32
#define BH_DISPATCH_COPY(code, T, ...)                                    \
  switch (code) {                                                         \
    case -1: { using T = NoT; __VA_ARGS__; } break;                       \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    default: throw std::runtime_error("multi_tensor: unsupported copy dtype " + std::to_string(code)); \
  }

#define MTA_PROLOGUE(v)                                                   \
  const int cidx = blockIdx.x;                                            \
  const int t = v.chunk_tensor[cidx];                                     \
  const int64_t base = (int64_t)v.chunk_local[cidx] * v.chunk;            \
  const int64_t n = min((int64_t)v.chunk, v.numel[t] - base);             \
  const bool al = v.aligned[t] != 0;

template <typename T>
BH_DEVICE T* mta_ptr(const MTAView& v, int d, int t, int64_t base) {
  return reinterpret_cast<T*>(v.ptrs[(int64_t)d * v.T + t]) + base;
}

template <typename T> struct IsNo { static constexpr bool value = false; };
template <> struct IsNo<NoT> { static constexpr bool value = true; };

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------------------------------
// scale: out = in * scale; non-finite input -> *noop = 1
// ------------------------------------------------------------------------------------
template <typename Ti, typename To>
__global__ __launch_bounds__(kBlock) void k_scale(MTAView v, float scale, const float* scale_dev, int* noop) {
  MTA_PROLOGUE(v);
  if (scale_dev) scale = *scale_dev;  // device-resident factor (e.g. a clip coefficient): no host sync
  const Ti* in = mta_ptr<const Ti>(v, 0, t, base);
  To* out = mta_ptr<To>(v, 1, t, base);
  bool finite = true;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float r[kVec];
    load_vec(in, i, n, al, r);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      finite &= is_finite(r[k]);
      r[k] *= scale;
    }
    store_vec(out, i, n, al, r);
  }
  if (!finite) *noop = 1;  // benign race: every writer stores the same value
}

// ------------------------------------------------------------------------------------
// axpby: out = a*x + b*y; finiteness checked on x (0), y (1) or both (-1)
// ------------------------------------------------------------------------------------
template <typename Tx, typename Ty, typename To>
__global__ __launch_bounds__(kBlock) void k_axpby(MTAView v, float a, float b, int check, int* noop) {
  MTA_PROLOGUE(v);
  const Tx* x = mta_ptr<const Tx>(v, 0, t, base);
  const Ty* y = mta_ptr<const Ty>(v, 1, t, base);
  To* out = mta_ptr<To>(v, 2, t, base);
  bool finite = true;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rx[kVec], ry[kVec];
    load_vec(x, i, n, al, rx);
    load_vec(y, i, n, al, ry);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      if (check == -1) finite &= is_finite(rx[k]) && is_finite(ry[k]);
      else if (check == 0) finite &= is_finite(rx[k]);
      else if (check == 1) finite &= is_finite(ry[k]);
      rx[k] = a * rx[k] + b * ry[k];
    }
    store_vec(out, i, n, al, rx);
  }
  if (!finite) *noop = 1;
}

// ------------------------------------------------------------------------------------
// norm partials (one float per chunk), optional scaled copy (l2norm_scale)
// ------------------------------------------------------------------------------------
template <typename Ti, typename To>
__global__ __launch_bounds__(kBlock) void k_norm_partials(MTAView v, int norm_type, float scale,
                                                          float* partials, int* noop, bool skip) {
  __shared__ float red[kBlock / kWave];
  if (skip && *noop) return;
  MTA_PROLOGUE(v);
  const Ti* in = mta_ptr<const Ti>(v, 0, t, base);
  To* out = nullptr;
  if constexpr (!IsNo<To>::value) out = mta_ptr<To>(v, 1, t, base);
  float acc = 0.f;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float r[kVec];
    load_vec(in, i, n, al, r);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      if (norm_type == 0) acc = fmaxf(acc, fabsf(r[k]));
      else acc = fmaf(r[k], r[k], acc);
    }
    if constexpr (!IsNo<To>::value) {
#pragma unroll
      for (int k = 0; k < kVec; ++k) r[k] *= scale;
      store_vec(out, i, n, al, r);
    }
  }
  const float tot = (norm_type == 0) ? block_max(acc, red) : block_sum(acc, red);
  if (threadIdx.x == 0) {
    partials[cidx] = tot;
    if (!is_finite(tot)) *noop = 1;
  }
}

// grid = T (+1 if totals): block b<T reduces tensor b's chunks, block T reduces everything.
__global__ __launch_bounds__(kBlock) void k_norm_finalize(MTAView v, const float* partials, int nstat,
                                                          int norm_type, float* per_tensor,
                                                          float* totals, bool blend, float alpha,
                                                          float beta, int* noop, bool skip) {
  __shared__ float red[kBlock / kWave];
  if (skip && *noop) return;
  const int b = blockIdx.x;
  const bool all = (per_tensor == nullptr) || (b == v.T);
  const int lo = all ? 0 : v.chunk0[b];
  const int hi = all ? v.C : v.chunk0[b + 1];
  for (int s = 0; s < nstat; ++s) {
    const float* p = partials + (int64_t)s * v.C;
    float acc = 0.f;
    for (int i = lo + threadIdx.x; i < hi; i += kBlock) {
      if (norm_type == 0) acc = fmaxf(acc, p[i]);
      else acc += p[i];
    }
    const float tot = (norm_type == 0) ? block_max(acc, red) : block_sum(acc, red);
    if (threadIdx.x == 0) {
      if (all) {
        if (totals) totals[s] = (norm_type == 0) ? tot : sqrtf(tot);
      } else {
        float* dst = per_tensor + (int64_t)s * v.T + b;
        if (blend) {
          const float old = *dst;
          *dst = (norm_type == 0) ? alpha * old + beta * tot : sqrtf(alpha * old * old + beta * tot);
        } else {
          *dst = (norm_type == 0) ? tot : sqrtf(tot);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Adam / AdamW (+ optional reduced-precision copy of the new params)
// ------------------------------------------------------------------------------------
template <typename Tg, typename Tp, typename Ts, typename Tc>
__global__ __launch_bounds__(kBlock) void k_adam(MTAView v, AdamArgs a) {
  if ((a.found_inf && *a.found_inf != 0.f) || (a.noop && *a.noop)) return;
  MTA_PROLOGUE(v);
  const Tg* g = mta_ptr<const Tg>(v, 0, t, base);
  Tp* p = mta_ptr<Tp>(v, 1, t, base);
  Ts* m = mta_ptr<Ts>(v, 2, t, base);
  Ts* vv = mta_ptr<Ts>(v, 3, t, base);
  Tc* cp = nullptr;
  if constexpr (!IsNo<Tc>::value) cp = mta_ptr<Tc>(v, 4, t, base);
  const float lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  float bc1 = a.bc1, bc2 = a.bc2;
  if (a.step_ptr && a.bias_correction) {
    const float st = (float)*a.step_ptr;
    bc1 = 1.f - powf(a.beta1, st);
    bc2 = 1.f - powf(a.beta2, st);
  }
  const float inv = a.inv_scale ? *a.inv_scale : 1.f;
  const float rbc1 = 1.f / bc1, rbc2 = 1.f / bc2;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec], rv[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(m, i, n, al, rm);
    load_vec(vv, i, n, al, rv);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      float gk = rg[k] * inv;
      if (a.mode == 0) gk += a.decay * rp[k];
      rm[k] = a.beta1 * rm[k] + (1.f - a.beta1) * gk;
      rv[k] = a.beta2 * rv[k] + (1.f - a.beta2) * gk * gk;
      const float denom = sqrtf(rv[k] * rbc2) + a.eps;
      float upd = (rm[k] * rbc1) / denom;
      if (a.mode == 1) upd += a.decay * rp[k];
      rp[k] -= lr * upd;
    }
    store_vec(p, i, n, al, rp);
    store_vec(m, i, n, al, rm);
    store_vec(vv, i, n, al, rv);
    if constexpr (!IsNo<Tc>::value) store_vec(cp, i, n, al, rp);
  }
}

// ------------------------------------------------------------------------------------
// SGD with momentum / nesterov / dampening, optional model-weight copy
// ------------------------------------------------------------------------------------
template <typename Tg, typename Tp, typename Tc>
__global__ __launch_bounds__(kBlock) void k_sgd(MTAView v, SGDArgs a, const int* noop) {
  if (*noop) return;
  MTA_PROLOGUE(v);
  const Tg* g = mta_ptr<const Tg>(v, 0, t, base);
  Tp* p = mta_ptr<Tp>(v, 1, t, base);
  Tp* mom = mta_ptr<Tp>(v, 2, t, base);
  Tc* cp = nullptr;
  if constexpr (!IsNo<Tc>::value) cp = mta_ptr<Tc>(v, 3, t, base);
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    if (a.momentum != 0.f) load_vec(mom, i, n, al, rm);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      float gk = rg[k] * a.scale;
      if (a.wd != 0.f && !a.wd_after_momentum) gk += a.wd * rp[k];
      if (a.momentum != 0.f) {
        rm[k] = a.first_run ? gk : rm[k] * a.momentum + (1.f - a.dampening) * gk;
        gk = a.nesterov ? gk + a.momentum * rm[k] : rm[k];
      }
      if (a.wd != 0.f && a.wd_after_momentum) gk += a.wd * rp[k];
      rp[k] -= a.lr * gk;
    }
    store_vec(p, i, n, al, rp);
    if (a.momentum != 0.f) store_vec(mom, i, n, al, rm);
    if constexpr (!IsNo<Tc>::value) store_vec(cp, i, n, al, rp);
  }
}

// ------------------------------------------------------------------------------------
// LAMB
// ------------------------------------------------------------------------------------
struct LambScalars {
  float bc1, bc2, lr, clip, inv;
};
BH_DEVICE LambScalars lamb_scalars(const LambArgs& a) {
  LambScalars s;
  s.bc1 = a.bc1;
  s.bc2 = a.bc2;
  if (a.step_ptr && a.bias_correction) {
    const float st = (float)*a.step_ptr;
    s.bc1 = 1.f - powf(a.beta1, st);
    s.bc2 = 1.f - powf(a.beta2, st);
  }
  s.lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  const float gn = a.grad_norm ? *a.grad_norm : 0.f;
  const float mx = a.max_norm_ptr ? *a.max_norm_ptr : a.max_grad_norm;
  s.clip = (mx > 0.f && gn > mx) ? gn / mx : 1.f;
  s.inv = a.inv_scale ? *a.inv_scale : 1.f;
  return s;
}
BH_DEVICE bool lamb_skip(const LambArgs& a) {
  return (a.noop && *a.noop) || (a.found_inf && *a.found_inf != 0.f);
}
// the LAMB update direction from the (already updated) moments
BH_DEVICE float lamb_update(const LambArgs& a, const LambScalars& s, float m, float v, float p) {
  const float denom = sqrtf(v / s.bc2) + a.eps;
  float u = (m / s.bc1) / denom;
  if (a.mode == 1) u += a.decay * p;
  return u;
}

template <typename Tg, typename Tp, typename Ts>
__global__ __launch_bounds__(kBlock) void k_lamb1(MTAView v, LambArgs a, float* partials) {
  __shared__ float red[kBlock / kWave];
  const int cidx0 = blockIdx.x;
  if (lamb_skip(a)) {
    if (threadIdx.x == 0) {
      partials[cidx0] = 0.f;
      partials[v.C + cidx0] = 0.f;
    }
    return;
  }
  MTA_PROLOGUE(v);
  const LambScalars s = lamb_scalars(a);
  const Tg* g = mta_ptr<const Tg>(v, 0, t, base);
  const Tp* p = mta_ptr<const Tp>(v, 1, t, base);
  Ts* m = mta_ptr<Ts>(v, 2, t, base);
  Ts* vv = mta_ptr<Ts>(v, 3, t, base);
  const float gscale = s.inv / s.clip;
  float pp = 0.f, uu = 0.f;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec], rv[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(m, i, n, al, rm);
    load_vec(vv, i, n, al, rv);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      float gk = rg[k] * gscale;
      if (a.mode == 0) gk += a.decay * rp[k];
      rm[k] = rm[k] * a.beta1 + a.beta3 * gk;
      rv[k] = rv[k] * a.beta2 + (1.f - a.beta2) * gk * gk;
      const float u = lamb_update(a, s, rm[k], rv[k], rp[k]);
      pp = fmaf(rp[k], rp[k], pp);
      uu = fmaf(u, u, uu);
    }
    store_vec(m, i, n, al, rm);
    store_vec(vv, i, n, al, rv);
  }
  const float tp = block_sum(pp, red);
  const float tu = block_sum(uu, red);
  if (threadIdx.x == 0) {
    partials[cidx] = tp;
    partials[v.C + cidx] = tu;
  }
}

template <typename Tp, typename Ts, typename Tc>
__global__ __launch_bounds__(kBlock) void k_lamb2(MTAView v, LambArgs a, const float* norms) {
  if (lamb_skip(a)) return;
  MTA_PROLOGUE(v);
  const LambScalars s = lamb_scalars(a);
  Tp* p = mta_ptr<Tp>(v, 1, t, base);
  const Ts* m = mta_ptr<const Ts>(v, 2, t, base);
  const Ts* vv = mta_ptr<const Ts>(v, 3, t, base);
  Tc* cp = nullptr;
  if constexpr (!IsNo<Tc>::value) cp = mta_ptr<Tc>(v, 4, t, base);
  float ratio = s.lr;
  if (a.use_nvlamb || a.decay != 0.f) {
    const float pn = norms[t], un = norms[v.T + t];
    ratio = (pn != 0.f && un != 0.f) ? s.lr * (pn / un) : s.lr;
  }
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rp[kVec], rm[kVec], rv[kVec];
    load_vec(p, i, n, al, rp);
    load_vec(m, i, n, al, rm);
    load_vec(vv, i, n, al, rv);
#pragma unroll
    for (int k = 0; k < kVec; ++k) rp[k] -= ratio * lamb_update(a, s, rm[k], rv[k], rp[k]);
    store_vec(p, i, n, al, rp);
    if constexpr (!IsNo<Tc>::value) store_vec(cp, i, n, al, rp);
  }
}

// ------------------------------------------------------------------------------------
// NovoGrad, Adagrad, LARS
// ------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_novograd(MTAView v, float lr, float beta1, float beta3,
                                                     float bc1, float bc2, float eps, int mode,
                                                     float decay, const float* gnorms) {
  MTA_PROLOGUE(v);
  const T* g = mta_ptr<const T>(v, 0, t, base);
  T* p = mta_ptr<T>(v, 1, t, base);
  T* m = mta_ptr<T>(v, 2, t, base);
  const float denom = gnorms[t] / bc2 + eps;
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(m, i, n, al, rm);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      if (mode == 0) {
        const float gk = rg[k] / denom + decay * rp[k];
        rm[k] = beta1 * rm[k] + beta3 * gk;
        rp[k] -= lr * (rm[k] / bc1);
      } else {
        rm[k] = beta1 * rm[k] + beta3 * rg[k];
        rp[k] -= lr * ((rm[k] / bc1) / denom + decay * rp[k]);
      }
    }
    store_vec(p, i, n, al, rp);
    store_vec(m, i, n, al, rm);
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_adagrad(MTAView v, float lr, float eps, int mode, float decay) {
  MTA_PROLOGUE(v);
  const T* g = mta_ptr<const T>(v, 0, t, base);
  T* p = mta_ptr<T>(v, 1, t, base);
  T* h = mta_ptr<T>(v, 2, t, base);
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rh[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(h, i, n, al, rh);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      if (mode == 0) {
        const float gk = rg[k] + decay * rp[k];
        rh[k] += gk * gk;
        rp[k] -= lr * (gk / (sqrtf(rh[k]) + eps));
      } else {
        rh[k] += rg[k] * rg[k];
        rp[k] -= lr * (rg[k] / (sqrtf(rh[k]) + eps) + decay * rp[k]);
      }
    }
    store_vec(p, i, n, al, rp);
    store_vec(h, i, n, al, rh);
  }
}

template <typename Tg, typename Tp, typename Tc>
__global__ __launch_bounds__(kBlock) void k_lars(MTAView v, LarsArgs a, const float* gnorms,
                                                 const float* pnorms, const int* noop) {
  if (*noop) return;
  MTA_PROLOGUE(v);
  const Tg* g = mta_ptr<const Tg>(v, 0, t, base);
  Tp* p = mta_ptr<Tp>(v, 1, t, base);
  Tp* mom = mta_ptr<Tp>(v, 2, t, base);
  Tc* cp = nullptr;
  if constexpr (!IsNo<Tc>::value) cp = mta_ptr<Tc>(v, 3, t, base);
  float slr = a.lr;
  if (!a.is_skipped) {
    const float pn = pnorms[t], gn = gnorms[t];
    float trust = 1.f;
    if (gn > 0.f && pn > 0.f) trust = a.trust_coefficient * pn / (gn + pn * a.wd + a.eps);
    slr = a.lr * trust;
  }
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(mom, i, n, al, rm);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      const float gk = rg[k] * a.scale + a.wd * rp[k];
      rm[k] = rm[k] * a.momentum - slr * gk;
      if (a.nesterov) rp[k] += rm[k] * a.momentum - slr * gk;
      else rp[k] += rm[k];
    }
    store_vec(p, i, n, al, rp);
    store_vec(mom, i, n, al, rm);
    if constexpr (!IsNo<Tc>::value) store_vec(cp, i, n, al, rp);
  }
}

// ------------------------------------------------------------------------------------
// standalone LAMB stages (csrc/multi_tensor_lamb_stage_{1,2}.cu API): update materialised
// ------------------------------------------------------------------------------------
template <typename Tg, typename Tp, typename Tu>
__global__ __launch_bounds__(kBlock) void k_lamb_s1(MTAView v, const float* decay_t, float beta1,
                                                    float beta2, float bc1, float bc2, float eps,
                                                    float clipped) {
  MTA_PROLOGUE(v);
  const Tg* g = mta_ptr<const Tg>(v, 0, t, base);
  const Tp* p = mta_ptr<const Tp>(v, 1, t, base);
  Tp* m = mta_ptr<Tp>(v, 2, t, base);
  Tp* vv = mta_ptr<Tp>(v, 3, t, base);
  Tu* u = mta_ptr<Tu>(v, 4, t, base);
  const float decay = decay_t[t];
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rg[kVec], rp[kVec], rm[kVec], rv[kVec];
    load_vec(g, i, n, al, rg);
    load_vec(p, i, n, al, rp);
    load_vec(m, i, n, al, rm);
    load_vec(vv, i, n, al, rv);
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
      const float sg = rg[k] / clipped;
      rm[k] = rm[k] * beta1 + (1.f - beta1) * sg;
      rv[k] = rv[k] * beta2 + (1.f - beta2) * sg * sg;
      rp[k] = (rm[k] / bc1) / (sqrtf(rv[k] / bc2) + eps) + decay * rp[k];
    }
    store_vec(u, i, n, al, rp);
    store_vec(m, i, n, al, rm);
    store_vec(vv, i, n, al, rv);
  }
}

template <typename Tp, typename Tu>
__global__ __launch_bounds__(kBlock) void k_lamb_s2(MTAView v, const float* pn_t, const float* un_t,
                                                    float lr, float decay, bool nvlamb) {
  MTA_PROLOGUE(v);
  Tp* p = mta_ptr<Tp>(v, 0, t, base);
  const Tu* u = mta_ptr<const Tu>(v, 1, t, base);
  float ratio = lr;
  if (nvlamb || decay != 0.f) {
    const float pn = pn_t[t], un = un_t[t];
    ratio = (un != 0.f && pn != 0.f) ? lr * (pn / un) : lr;
  }
  for (int64_t i = (int64_t)threadIdx.x * kVec; i < n; i += (int64_t)kBlock * kVec) {
    float rp[kVec], ru[kVec];
    load_vec(p, i, n, al, rp);
    load_vec(u, i, n, al, ru);
#pragma unroll
    for (int k = 0; k < kVec; ++k) rp[k] -= ratio * ru[k];
    store_vec(p, i, n, al, rp);
  }
}

}  // namespace

// ======================================================================================
// launchers
// ======================================================================================
void mta_scale(const MTAView& v, int dt_in, int dt_out, float scale, int* noop, hipStream_t s,
               const float* scale_dev) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_in, Ti, BH_DISPATCH_FLOAT(dt_out, To,
      hipLaunchKernelGGL((k_scale<Ti, To>), dim3(v.C), dim3(kBlock), 0, s, v, scale, scale_dev, noop)));
  check_launch("multi_tensor_scale");
}

void mta_axpby(const MTAView& v, int dt_x, int dt_y, int dt_out, float a, float b, int arg_to_check,
               int* noop, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_x, Tx, BH_DISPATCH_FLOAT(dt_y, Ty, BH_DISPATCH_FLOAT(dt_out, To,
      hipLaunchKernelGGL((k_axpby<Tx, Ty, To>), dim3(v.C), dim3(kBlock), 0, s, v, a, b,
                         arg_to_check, noop))));
  check_launch("multi_tensor_axpby");
}

void mta_norm_partials(const MTAView& v, int dt_in, int dt_out, int norm_type, float scale,
                       float* partials, int* noop, bool skip_if_noop, hipStream_t s) {
  if (v.C == 0) return;
  if (v.depth == 1) {
    BH_DISPATCH_FLOAT(dt_in, Ti,
        hipLaunchKernelGGL((k_norm_partials<Ti, NoT>), dim3(v.C), dim3(kBlock), 0, s, v, norm_type,
                           scale, partials, noop, skip_if_noop));
  } else {
    BH_DISPATCH_FLOAT(dt_in, Ti, BH_DISPATCH_FLOAT(dt_out, To,
        hipLaunchKernelGGL((k_norm_partials<Ti, To>), dim3(v.C), dim3(kBlock), 0, s, v, norm_type,
                           scale, partials, noop, skip_if_noop)));
  }
  check_launch("multi_tensor_norm_partials");
}

void mta_norm_finalize(const MTAView& v, const float* partials, int nstat, int norm_type,
                       float* per_tensor, float* totals, bool blend, float alpha, float beta,
                       int* noop, bool skip_if_noop, hipStream_t s) {
  const int grid = (per_tensor ? v.T : 0) + (totals ? 1 : 0);
  if (grid == 0) return;
  if (v.C == 0) {
    // empty lists: norms are zero
    if (totals) (void)hipMemsetAsync(totals, 0, sizeof(float) * nstat, s);
    return;
  }
  // when per_tensor is null the single block reduces everything (b == 0 acts as "all")
  hipLaunchKernelGGL(k_norm_finalize, dim3(grid), dim3(kBlock), 0, s, v, partials, nstat, norm_type,
                     per_tensor, totals, blend, alpha, beta, noop, skip_if_noop);
  check_launch("multi_tensor_norm_finalize");
}

void mta_adam(const MTAView& v, int dt_g, int dt_p, int dt_s, int dt_copy, const AdamArgs& a,
              hipStream_t s) {
  if (v.C == 0) return;
  if (dt_s != dt_p && dt_s != kF32) throw std::runtime_error("multi_tensor_adam: state dtype must match params or be fp32");
  if (dt_g == dt_p) {
    BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_COPY(dt_copy, Tc,
        if (dt_s == dt_p) {
          hipLaunchKernelGGL((k_adam<Tp, Tp, Tp, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a);
        } else {
          hipLaunchKernelGGL((k_adam<Tp, Tp, float, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a);
        }));
  } else if (dt_p == kF32 && dt_s == kF32 && (dt_g == kF16 || dt_g == kBF16)) {
    // fp32 master params updated straight from 16-bit model grads (no upcast pass)
    BH_DISPATCH_FLOAT(dt_g, Tg, BH_DISPATCH_COPY(dt_copy, Tc,
        hipLaunchKernelGGL((k_adam<Tg, float, float, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a)));
  } else {
    throw std::runtime_error("multi_tensor_adam: unsupported grad/param dtype combination");
  }
  check_launch("multi_tensor_adam");
}

void mta_sgd(const MTAView& v, int dt_g, int dt_p, int dt_copy, const SGDArgs& a, const int* noop,
             hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_g, Tg, BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_COPY(dt_copy, Tc,
      hipLaunchKernelGGL((k_sgd<Tg, Tp, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a, noop))));
  check_launch("multi_tensor_sgd");
}

void mta_lamb_stage1(const MTAView& v, int dt_g, int dt_p, int dt_s, const LambArgs& a,
                     float* partials, hipStream_t s) {
  if (v.C == 0) return;
  if (dt_s != dt_p && dt_s != kF32) throw std::runtime_error("multi_tensor_lamb: state dtype must match params or be fp32");
  BH_DISPATCH_FLOAT(dt_g, Tg, BH_DISPATCH_FLOAT(dt_p, Tp,
      if (dt_s == dt_p) {
        hipLaunchKernelGGL((k_lamb1<Tg, Tp, Tp>), dim3(v.C), dim3(kBlock), 0, s, v, a, partials);
      } else {
        hipLaunchKernelGGL((k_lamb1<Tg, Tp, float>), dim3(v.C), dim3(kBlock), 0, s, v, a, partials);
      }));
  check_launch("multi_tensor_lamb_stage1");
}

void mta_lamb_stage2(const MTAView& v, int dt_p, int dt_s, int dt_copy, const LambArgs& a,
                     const float* norms, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_COPY(dt_copy, Tc,
      if (dt_s == dt_p) {
        hipLaunchKernelGGL((k_lamb2<Tp, Tp, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a, norms);
      } else {
        hipLaunchKernelGGL((k_lamb2<Tp, float, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a, norms);
      }));
  check_launch("multi_tensor_lamb_stage2");
}

void mta_novograd(const MTAView& v, int dt, float lr, float beta1, float beta3, float bc1, float bc2,
                  float eps, int mode, float decay, const float* grad_norms, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt, T,
      hipLaunchKernelGGL((k_novograd<T>), dim3(v.C), dim3(kBlock), 0, s, v, lr, beta1, beta3, bc1,
                         bc2, eps, mode, decay, grad_norms));
  check_launch("multi_tensor_novograd");
}

void mta_adagrad(const MTAView& v, int dt, float lr, float eps, int mode, float decay, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt, T,
      hipLaunchKernelGGL((k_adagrad<T>), dim3(v.C), dim3(kBlock), 0, s, v, lr, eps, mode, decay));
  check_launch("multi_tensor_adagrad");
}

void mta_lars(const MTAView& v, int dt_g, int dt_p, int dt_copy, const LarsArgs& a,
              const float* grad_norms, const float* param_norms, const int* noop, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_g, Tg, BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_COPY(dt_copy, Tc,
      hipLaunchKernelGGL((k_lars<Tg, Tp, Tc>), dim3(v.C), dim3(kBlock), 0, s, v, a, grad_norms,
                         param_norms, noop))));
  check_launch("multi_tensor_lars");
}

void mta_lamb_stage1_standalone(const MTAView& v, int dt_g, int dt_p, int dt_u,
                                 const float* per_tensor_decay, float beta1, float beta2, float bc1,
                                 float bc2, float eps, float clipped_norm, hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_g, Tg, BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_FLOAT(dt_u, Tu,
      hipLaunchKernelGGL((k_lamb_s1<Tg, Tp, Tu>), dim3(v.C), dim3(kBlock), 0, s, v, per_tensor_decay,
                         beta1, beta2, bc1, bc2, eps, clipped_norm))));
  check_launch("multi_tensor_lamb_stage1_cuda");
}

void mta_lamb_stage2_standalone(const MTAView& v, int dt_p, int dt_u, const float* pnorm,
                                const float* unorm, float lr, float decay, bool use_nvlamb,
                                hipStream_t s) {
  if (v.C == 0) return;
  BH_DISPATCH_FLOAT(dt_p, Tp, BH_DISPATCH_FLOAT(dt_u, Tu,
      hipLaunchKernelGGL((k_lamb_s2<Tp, Tu>), dim3(v.C), dim3(kBlock), 0, s, v, pnorm, unorm, lr, decay,
                         use_nvlamb)));
  check_launch("multi_tensor_lamb_stage2_cuda");
}

// ---- graph-capture-safe upload of a small host table ---------------------------------------------
// While a stream is being captured, a pinned staging buffer + async copy is not allowed; the bytes
// travel instead as kernel arguments (captured by value into the graph node), up to 3.5 KiB per launch.
namespace {
constexpr int kUploadVecs = 224;
struct UploadPayload {
  uint4 d[kUploadVecs];
};
__global__ __launch_bounds__(256) void k_upload(uint4* __restrict__ dst, UploadPayload p, int n) {
  const int i = threadIdx.x;
  if (i < n) dst[i] = p.d[i];
}
}  // namespace

void upload_bytes(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes % 16 != 0 || reinterpret_cast<uintptr_t>(dst) % 16 != 0)
    throw std::runtime_error("upload_bytes: 16-byte multiples / alignment only");
  const uint4* in = reinterpret_cast<const uint4*>(src);
  uint4* out = reinterpret_cast<uint4*>(dst);
  const size_t nvec = bytes / 16;
  for (size_t off = 0; off < nvec; off += kUploadVecs) {
    UploadPayload p;
    const int n = (int)std::min<size_t>(kUploadVecs, nvec - off);
    for (int i = 0; i < n; ++i) p.d[i] = in[off + i];
    hipLaunchKernelGGL(k_upload, dim3(1), dim3(256), 0, s, out + off, p, n);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("upload_bytes: ") + hipGetErrorString(e));
}

// ------------------------------------------------------------------------------------
// amp's device-resident dynamic loss scale, one backward pass's bookkeeping in one launch (reference
// semantics: apex/amp/scaler.py:197-226): fold the pass's overflow flag into the step flag, then
// overflow -> scale / factor (>= min), counter 0; else counter + 1 and scale * factor (<= max) when the
// counter reaches the window (then counter 0). Replaces ~10 tiny torch ops per step.
// ------------------------------------------------------------------------------------
namespace {
__global__ void k_update_scale(float* scale, int* unskipped, const int* overflow, int* step_flag, float factor,
                               int window, float min_scale, float max_scale) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool ov = *overflow > 0;
  if (step_flag && ov) *step_flag = 1;
  const float s = *scale;
  if (ov) {
    float d = s / factor;
    if (min_scale > 0.f) d = fmaxf(d, min_scale);
    *scale = d;
    *unskipped = 0;
    return;
  }
  const int cnt = *unskipped + 1;
  if (cnt >= window) {
    *scale = fminf(s * factor, max_scale);
    *unskipped = 0;
  } else {
    *unskipped = cnt;
  }
}
}  // namespace

void amp_update_scale(float* scale, int* unskipped, const int* overflow, int* step_flag, float factor, int window,
                      float min_scale, float max_scale, hipStream_t s) {
  hipLaunchKernelGGL(k_update_scale, dim3(1), dim3(64), 0, s, scale, unskipped, overflow, step_flag, factor, window,
                     min_scale, max_scale);
  check_launch("amp_update_scale");
}

namespace {
__global__ void k_norm_blend(const float* plain, const float* scaled, const float* inv_scale, float* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float u = *scaled * *inv_scale;
  const float p = plain ? *plain : 0.f;
  *out = sqrtf(fmaf(p, p, u * u));
}
}  // namespace

void norm_blend(const float* plain, const float* scaled, const float* inv_scale, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_blend, dim3(1), dim3(64), 0, s, plain, scaled, inv_scale, out);
  check_launch("norm_blend");
}

}  // namespace bh
