// Attention softmax / cross-entropy launcher API (kernels: csrc/kernels/softmax.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

int softmax_max_sk();
// rows = number of softmax rows; mode 0: none, 1: padding mask [mask_batches, 1, sq, sk] (uint8,
// nonzero = masked -> -10000), 2: causal (row r masks columns > r % sq). y may alias x.
void softmax_forward(int dt, const void* x, const uint8_t* mask, void* y, int64_t rows, int sq, int sk, int heads,
                     int mask_batches, int mode, float scale, bool vec, hipStream_t st);
// dx = scale * y * (dy - sum(dy*y)); dx may alias dy
void softmax_backward(int dt, const void* dy, const void* y, void* dx, int64_t rows, int sq, int sk, int mode,
                      float scale, bool vec, hipStream_t st);
void xentropy_forward(int dt, const void* x, const int64_t* labels, int dt_loss, void* loss, float* lse, int64_t rows,
                      int V, float smoothing, bool vec, hipStream_t st);
void xentropy_backward(int dt, const void* x, int dt_g, const void* gloss, const float* lse, const int64_t* labels,
                       void* dx, int64_t rows, int V, float smoothing, bool vec, hipStream_t st);

// vocab-parallel cross-entropy: per-row shard partials stats[rows][4] = {max, sumexp, target logit, 0}
void vocab_xent_stats(int dt, const void* x, const int64_t* target, float* stats, int64_t rows, int V, int64_t start,
                      bool vec, hipStream_t st);
// stats [world][rows][4] -> loss[rows] (dtype dt_loss), lse[rows]
void vocab_xent_combine(const float* stats, int world, int64_t rows, int dt_loss, void* loss, float* lse,
                        hipStream_t st);

}  // namespace bh
