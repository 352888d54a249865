// contrib launcher API (kernels: csrc/kernels/contrib.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// focal loss: x [rows, C] logits, y [rows] labels (-1 background, -2 ignore). Writes the per-element
// partial gradient (unnormalised) and loss[0] = sum / num_pos[0]. part: focal_loss_parts(numel) floats.
int focal_loss_parts(int64_t numel);
void focal_loss_forward(int dt, const void* x, const int64_t* y, void* pgrad, float* part, int nparts,
                        const float* num_pos, float* loss, int64_t rows, int C, int real_C, float alpha, float gamma,
                        float smoothing, hipStream_t st);
// in place: g *= gout[0] / num_pos[0]
void focal_loss_backward(int dt, void* g, const float* gout, const float* num_pos, int64_t n, hipStream_t st);

// index_mul_2d: out[i] = in1[idx[i]] * in2[i] (rows of width F)
void index_mul_2d_forward(int dt, void* out, const void* in1, const void* in2, const int64_t* idx, int64_t n, int F,
                          hipStream_t st);
// acc1: zeroed fp32 [n1, F] accumulation buffer; gin1 (dtype dt) receives it converted (null: acc1 IS the result)
void index_mul_2d_backward(int dt, float* acc1, void* gin1, int64_t n1, void* gin2, const void* gout, const void* in1,
                           const void* in2, const int64_t* idx, int64_t n, int F, hipStream_t st);
void index_mul_2d_backward_backward(int dt, void* ggo, float* acc1, void* gin1, int64_t n1, void* gin2,
                                    const void* gout, const void* gg1, const void* gg2, const void* in1,
                                    const void* in2, const int64_t* idx, int64_t n, int F, hipStream_t st);

}  // namespace bh
