// Dense-layer epilogue launcher API (kernels: csrc/kernels/dense.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

enum DenseAct { kActNone = 0, kActRelu = 1, kActSigmoid = 2, kActGelu = 3, kActGeluTanh = 4 };

// y[M,N] = act(x (+ bias[N])); y may alias x. vec: N % 8 == 0 and 16-byte aligned pointers.
void dense_act_forward(int dt, const void* x, const void* bias, void* y, int64_t M, int N, int act, bool vec,
                       hipStream_t st);
// number of row splits used by dense_act_backward (partial buffer = splits * N floats)
int dense_bgrad_splits(int64_t M, int N);
// dx = dy * act'(aux) (dx may be null: bias-grad only; may alias dy), bgrad[N] = sum_m dx (null: skip).
// aux is the activation OUTPUT for ReLU / sigmoid and the PRE-activation for GELU.
void dense_act_backward(int dt, const void* dy, const void* aux, void* dx, void* bgrad, float* part, int splits,
                        int64_t M, int N, int act, bool vec, hipStream_t st);

}  // namespace bh
