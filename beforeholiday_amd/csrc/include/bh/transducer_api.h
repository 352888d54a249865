// RNN-T loss launcher API (kernels: csrc/kernels/transducer.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// x: log-probs, padded [B, max_t, max_u1, V] or packed [sum f_len*(y_len+1), V] (batch_offset =
// inclusive cumsum). alpha/beta: [B, max_t, max_u1] fp32; loss: [B] fp32.
void transducer_loss_forward(int dt, const void* x, const int64_t* label, int label_stride, const int* f_len,
                             const int* y_len, const int64_t* batch_offset, int B, int max_t, int max_u1, int V,
                             int blank, float* alpha, float* beta, float* loss, hipStream_t st);
void transducer_loss_backward(int dt, const void* x, const float* loss_grad, const float* alpha, const float* beta,
                              const int64_t* label, int label_stride, const int* f_len, const int* y_len,
                              const int64_t* batch_offset, int B, int max_t, int max_u1, int V, int blank,
                              bool fuse_softmax, void* dx, hipStream_t st);

}  // namespace bh
