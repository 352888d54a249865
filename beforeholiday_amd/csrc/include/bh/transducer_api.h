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

namespace bh {

// RNN-T joint: out(b,t,u,:) = f(b,t,:) + g(b,u,:) (+ ReLU) (+ dropout), for t < f_len[b], u < g_len[b].
// Padded output [B, T, U, H] (invalid rows zero) or packed [rows, H] with row
// (b ? batch_offset[b-1] : 0) + t*g_len[b] + u. Dropout keep bits come from a keyed counter hash of the
// (b, t, u, h) index, so the backward regenerates them (no mask tensor); with ReLU the backward mask
// is (out > 0). mask (optional, uint8 per output element) is only written for the mask probe.
struct JointArgs {
  int B, T, U, H;
  int64_t rows;  // rows of the output / grad tensor (bounds every access)
  const int* f_len;
  const int* g_len;
  const int64_t* batch_offset;  // null: padded output
  bool relu, dropout;
  uint32_t keep_thresh;  // keep iff hash >= keep_thresh
  float scale;           // 1 / (1 - p)
  uint32_t seed;
};
void transducer_joint_forward(const JointArgs& a, int dt, const void* f, const void* g, void* out, uint8_t* mask,
                              hipStream_t st);
// df [B, T, H], dg [B, U, H] (both fully written; zeros outside the valid ranges)
void transducer_joint_backward(const JointArgs& a, int dt, const void* grad, const void* out, void* df, void* dg,
                               hipStream_t st);

}  // namespace bh
