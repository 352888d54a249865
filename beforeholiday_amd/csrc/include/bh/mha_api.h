// Multi-head-attention softmax launcher API (kernels: csrc/kernels/mha.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

int mha_max_sk();
// x: scores [rows = B*heads*sq, sk]. mask_mode 0 none, 1 key padding bool [B, sk], 2 additive [B, sk]
// (dtype dt_mask), 3 time bool [sq, sk]. Writes softmax `sm` and (if non-null) dropped probabilities.
// Dropout keep-mask = Philox(seed, row, offset + col/4) <= 1 - p_drop (regenerated in backward).
void mha_softmax_dropout_forward(int dt, const void* x, int mask_mode, int dt_mask, const void* mask, void* sm,
                                 void* dropped, int64_t rows, int sq, int sk, int heads, float p_drop, uint64_t seed,
                                 uint64_t offset, bool vec, hipStream_t st);
// dx = sm * (g - sum(g*sm)), g = dy * keep / (1 - p) when use_dropout. dx may alias dy.
void mha_softmax_dropout_backward(int dt, const void* dy, const void* sm, void* dx, int64_t rows, int sk, float p_drop,
                                  uint64_t seed, uint64_t offset, bool use_dropout, bool vec, hipStream_t st);

}  // namespace bh
