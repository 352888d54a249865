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

// out[M,N] = residual + dropout(x + bias[N]) (bias may be null); keep: uint8 [M*N/8] keep bits (null: no
// dropout, p ignored). N % 8 == 0, 16-byte aligned pointers. Bits are a seed-keyed hash of the element index.
void dense_bias_dropout_add(int dt, const void* x, const void* bias, const void* residual, void* out, uint8_t* keep,
                            int64_t M, int N, float p, uint32_t seed, hipStream_t st,
                            const int64_t* seed_dev = nullptr);  // device step seed (utils/graph_rng.py)
// dx = dy * keep * keep_scale (dx may be null), bgrad[N] = sum_m dx (null: skip); N % 8 == 0, aligned.
void dense_dropout_backward(int dt, const void* dy, const uint8_t* keep, float keep_scale, void* dx, void* bgrad,
                            float* part, int splits, int64_t M, int N, hipStream_t st);

// C[M, 64] = A[M, K] . B[64, K]^T (+ resid[M, 64] if non-null), K in {64, 128, 256}, M % 32 == 0,
// 16-byte aligned row-major operands (kernels/gemm_n64.hip)
bool gemm_n64_supported(int64_t M, int K, int N);
void gemm_n64(int dt, const void* a, const void* b, const void* resid, void* c, int64_t M, int K, hipStream_t st);

// embedding weight gradient dw[V, H] (zero-filled by the caller) from dy[n, H] and the stably sorted
// token ids + permutation; piece = fp32 [n, H] scratch. Deterministic, no host synchronisation.
void embedding_backward(int dt, const int64_t* sorted, const int64_t* perm, const void* dy, float* piece, void* dw,
                        int64_t n, int H, int64_t padding_idx, hipStream_t st);

}  // namespace bh
