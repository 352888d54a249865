// LayerNorm / RMSNorm launcher API (kernels: csrc/kernels/layer_norm.hip).
// Rows: n1 (product of the leading dims), row length n2 (product of normalized_shape).
// `vec` = n2 % 8 == 0 and every pointer 16-byte aligned (host decides).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// y = (x - mean) * invvar * gamma + beta   (rms: mean = 0, no beta); gamma/beta may be null.
// dt_w = -1 when there are no affine params. mean may be null for rms.
void ln_forward(int64_t n1, int n2, int dt_x, const void* x, int dt_w, const void* gamma, const void* beta,
                int dt_y, void* y, float* mean, float* invvar, float eps, bool rms, bool vec, hipStream_t st);
// dx; xin is the input x, or the output y when from_output (memory-efficient mode)
void ln_backward_dx(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                    const float* invvar, int dt_w, const void* gamma, const void* beta, void* dx, bool rms,
                    bool from_output, bool vec, hipStream_t st, const void* dresid = nullptr);
// (dresid: optional [n1, n2] tensor of dx's dtype added to dx in the same pass -- the gradient the
// residual branch of a pre-LN block sends to the same input, reference layer_norm.cuh:474 dout_resid)
int ln_wgrad_splits(int64_t n1, int n2);
// dx AND grad_gamma / grad_beta from one pass over dy and x (rows <= 2048 elements): 0 when the shape is not
// covered, else the number of partial rows (partials: 2 * blocks * n2 floats of scratch)
int ln_bwd_fused_blocks(int64_t n1, int n2);
void ln_backward_fused(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                       const float* invvar, int dt_w, const void* gamma, const void* beta, void* dx, void* grad_gamma,
                       void* grad_beta, float* partials, int blocks, bool rms, bool from_output, bool vec,
                       hipStream_t st, const void* dresid);
// grad_gamma / grad_beta (may be null); partials: 2 * splits * n2 floats of scratch
void ln_backward_wgrad(int64_t n1, int n2, int dt_dy, const void* dy, int dt_x, const void* xin, const float* mean,
                       const float* invvar, int dt_w, const void* gamma, const void* beta, void* grad_gamma,
                       void* grad_beta, float* partials, int splits, bool rms, bool from_output, bool vec,
                       hipStream_t st);

}  // namespace bh
