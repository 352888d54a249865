// Host-side launcher API shared by the torch-free HIP kernel translation units
// (csrc/kernels/*.hip) and the pybind/ATen front-end (csrc/bindings/*.cpp).
//
// Kernels never see at::Tensor: the front-end validates tensors and passes raw pointers,
// dtype codes and the current HIP stream. This keeps the .hip TUs free of torch headers
// (fast, torch-ABI independent builds) and makes every launcher graph-capturable
// (no allocation, no synchronisation inside a launcher).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// Summation order of G partial rows (per channel) shared by the BatchNorm partial-sum kernels (batchnorm.hip
// k_merge_parts / k_merge_segs, conv_bn.hip k_sum_parts), so every path gives the same bits: SG contiguous
// segments of ceil(G / SG) rows, each summed as 16 strided row groups added in order, then the segment
// totals in order. From 1024 rows (a 28x28 3x3 convolution leaves ~7000) the segments are summed in parallel.
__host__ __device__ inline int bn_part_segments(int G) { return G >= 1024 ? (G / 256 < 32 ? G / 256 : 32) : 1; }

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kF64 = 3, kU8 = 4, kI32 = 5, kI64 = 6, kBool = 7 };

// ---------------------------------------------------------------------------------
// Multi-tensor apply (replacement for csrc/multi_tensor_apply.cuh).
//
// The front-end packs, once per distinct tensor-list signature, a device-resident plan:
//   ptrs[depth][T]   u64   base pointer of tensor t in list d
//   numel[T]         i64
//   aligned[T]       i32   all `depth` pointers of tensor t are 16-byte aligned
//   chunk0[T+1]      i32   first global chunk id of tensor t (prefix sum)
//   chunk_tensor[C]  i32   tensor of global chunk c
//   chunk_local[C]   i32   chunk index of c inside its tensor
// One workgroup per chunk; there is no tensors-per-launch limit and no relaunch loop.
// ---------------------------------------------------------------------------------
struct MTAView {
  const uint64_t* ptrs;
  const int64_t* numel;
  const int* aligned;
  const int* chunk0;
  const int* chunk_tensor;
  const int* chunk_local;
  int T;
  int C;
  int depth;
  int chunk;
};

// scale_dev (optional): device fp32 scalar used instead of `scale`
// copy a small host table (multiple of 16 bytes) to the device as kernel arguments: legal while the
// stream is being captured into a HIP graph (no staging buffer, no memcpy node)
void upload_bytes(void* dst, const void* src, size_t bytes, hipStream_t s);
void mta_scale(const MTAView& v, int dt_in, int dt_out, float scale, int* noop, hipStream_t s,
               const float* scale_dev = nullptr);
void mta_axpby(const MTAView& v, int dt_x, int dt_y, int dt_out, float a, float b, int arg_to_check,
               int* noop, hipStream_t s);
// Per-chunk partial reductions of list 0: norm_type 2 -> sum of squares, 0 -> max |x|.
// If `skip_if_noop` and *noop != 0 the kernel does nothing (the "_mp" variants).
// If v.depth == 2 also writes list1 = list0 * scale (the l2norm_scale variant).
void mta_norm_partials(const MTAView& v, int dt_in, int dt_out, int norm_type, float scale,
                       float* partials, int* noop, bool skip_if_noop, hipStream_t s);
// Reduce `nstat` partial arrays (layout [nstat][C]) into per-tensor values
// per_tensor[nstat][T] (may be null) and totals[nstat] (may be null).
// norm_type 2: sqrt(sum); 0: max. If blend: per_tensor = sqrt(a*old^2 + b*new^2) (L2)
// or a*old + b*new (Linf) with old read from per_tensor.
void mta_norm_finalize(const MTAView& v, const float* partials, int nstat, int norm_type,
                       float* per_tensor, float* totals, bool blend, float alpha, float beta,
                       int* noop, bool skip_if_noop, hipStream_t s);

struct AdamArgs {
  float lr, beta1, beta2, eps, bc1, bc2, decay;
  int mode;  // 0: L2 (Adam), 1: decoupled (AdamW)
  const float* lr_ptr;       // optional device lr (capturable)
  const float* inv_scale;    // optional grad unscale factor (device)
  const float* found_inf;    // optional: skip when != 0
  const int* step_ptr;       // optional device step: bias corrections computed on device
  int bias_correction;
  const int* noop;           // optional skip flag (int; amp's device-resident overflow)
};
// lists: g, p, m, v [, p_copy]  (depth 4 or 5)
void mta_adam(const MTAView& v, int dt_g, int dt_p, int dt_s, int dt_copy, const AdamArgs& a,
              hipStream_t s);

struct SGDArgs {
  float wd, momentum, dampening, lr, scale;
  bool nesterov, first_run, wd_after_momentum;
};
// lists: g, p, mom [, p_copy]; early-exits if *noop
void mta_sgd(const MTAView& v, int dt_g, int dt_p, int dt_copy, const SGDArgs& a, const int* noop,
             hipStream_t s);

struct LambArgs {
  float lr, beta1, beta2, beta3, bc1, bc2, eps, decay, max_grad_norm;
  int mode;  // 0: L2, 1: decoupled
  bool use_nvlamb;
  int bias_correction;
  const float* grad_norm;       // global grad norm (device)
  const float* max_norm_ptr;    // optional device max_grad_norm
  const float* lr_ptr;          // optional device lr
  const int* step_ptr;          // optional device step
  const float* inv_scale;       // optional grad unscale
  const float* found_inf;       // optional skip flag
  const int* noop;              // optional skip flag (int)
};
// Stage 1: g,p,m,v -> m,v updated; partials[2][C] = (sum p^2, sum u^2) per chunk.
void mta_lamb_stage1(const MTAView& v, int dt_g, int dt_p, int dt_s, const LambArgs& a,
                     float* partials, hipStream_t s);
// Stage 2: recompute u from (p, m, v), apply trust ratio from norms[2][T]; lists g,p,m,v[,copy]
void mta_lamb_stage2(const MTAView& v, int dt_p, int dt_s, int dt_copy, const LambArgs& a,
                     const float* per_tensor_norms, hipStream_t s);

// lists g, p, m; grad_norms[T] already blended
void mta_novograd(const MTAView& v, int dt, float lr, float beta1, float beta3, float bc1,
                  float bc2, float eps, int mode, float decay, const float* grad_norms,
                  hipStream_t s);
// lists g, p, h
void mta_adagrad(const MTAView& v, int dt, float lr, float eps, int mode, float decay,
                 hipStream_t s);

struct LarsArgs {
  float lr, trust_coefficient, eps, wd, momentum, dampening, scale;
  bool nesterov, first_run, wd_after_momentum, is_skipped;
};
// lists g, p, mom [, p_copy]
void mta_lars(const MTAView& v, int dt_g, int dt_p, int dt_copy, const LarsArgs& a,
              const float* grad_norms, const float* param_norms, const int* noop, hipStream_t s);

// standalone stages (lists g,p,m,v,update  /  p,update)
void mta_lamb_stage1_standalone(const MTAView& v, int dt_g, int dt_p, int dt_u,
                                 const float* per_tensor_decay, float beta1, float beta2, float bc1,
                                 float bc2, float eps, float clipped_norm, hipStream_t s);
void mta_lamb_stage2_standalone(const MTAView& v, int dt_p, int dt_u, const float* pnorm,
                                const float* unorm, float lr, float decay, bool use_nvlamb,
                                hipStream_t s);

// out[0] = sqrt(plain[0]^2 + (scaled[0] inv_scale[0])^2) (plain may be null): a loss-scaled norm blended with
// the norm of already-unscaled gradients in one launch (FusedLAMB's global gradient norm under amp)
void norm_blend(const float* plain, const float* scaled, const float* inv_scale, float* out, hipStream_t s);

// amp device loss scale: step_flag |= overflow; then the dynamic-scale update (see multi_tensor.hip)
void amp_update_scale(float* scale, int* unskipped, const int* overflow, int* step_flag, float factor, int window,
                      float min_scale, float max_scale, hipStream_t s);

}  // namespace bh
