// BatchNorm backward folded into the neighbouring 1x1 convolution by linear algebra (kernels/bn_fold.hip,
// models/resnet.py `_ConvBNResFn`).
//
// A training BatchNorm after a 1x1 convolution y = a . W^T has the input gradient
//   gx = A[n] g + B[n] y + D[n]            (per output channel n; g the BatchNorm's output gradient)
// with A, B, D from the batch statistics and the two sums  sum_m g  and  sum_m g (y - mean). Because y is
// linear in a, everything the convolution's backward needs follows from g, a and small matrices:
//   sum_m g y        = rowdot(W, P),                 P  = g^T a        [N, K]  (the raw weight gradient)
//   dW               = A (.) P + B (.) (W Gm) + D (x) S_a,  Gm = a^T a [K, K], S_a = colsum(a)
// so the BatchNorm's backward-reduce pass and the conv weight gradient's read of gx disappear; the data
// gradient forms gx per fragment from (g, y) inside its GEMM (conv_bn.hip's BatchNorm-backward prologue).
// (da could also be written as g . (A W) + a . (W^T diag(B) W) + W^T D without y, but that sums large
// terms that cancel after 16-bit rounding of the small matrices: measured 40x less accurate.)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// Gram matrix of a [M, K] (16-bit, row-major) with an optional BatchNorm + ReLU prologue
// a' = relu(a * pro_scale[k] + pro_shift[k]) rounded to the input type: fp32 partials
// gram_part[s][K][K] (s < gram_splits) and column sums colsum_part[s][K]. K % 64 == 0.
int gram_splits(int64_t M, int K);
// s2_H > 0: row m is pixel (n, 2y, 2x) of an [.., s2_H, s2_W, K] input (M = its quarter-resolution rows)
void gram_partials(int dt, const void* a, int64_t M, int K, const float* pro_scale, const float* pro_shift,
                   float* gram_part, float* colsum_part, hipStream_t st, int s2_H = 0, int s2_W = 0);

// g_pre[m, n] = bits(m, n) ? g[m, n] : 0 with bits [M, N/8] (bit n % 8 of byte n / 8), and the column sums
// of g_pre as fp32 partials colsum_part[s][N] (s < mask_colsum_splits). N % 8 == 0.
int mask_colsum_splits(int64_t M, int N);
void mask_colsum(int dt, const void* g, const uint8_t* bits, void* g_pre, int64_t M, int N, float* colsum_part,
                 hipStream_t st);

// ---- combine (ops/bn_fold.py: the small-matrix algebra, one launch per stage) ----
// stage 1: P [N, K] = sum of the S1 rows of p_ws [S1, N K] (the fp32 weight-gradient partials), Gm [K, K] and
// Sa [K] from g_ws [S2, K K] / sa_ws [S2, K], Sg = sum of the S3 rows of sg_ws [S3, N]; then this rank's
// sums [2N] = [Sg, rowdot(W, P) - mean Sg] and bn_grads [2N] = [sums[N:] invstd, Sg] (fixed-order sums)
void fold_reduce(int dt, const void* W, const float* p_ws, int S1, const float* g_ws, const float* sa_ws, int S2,
                 const float* sg_ws, int S3, const float* mean, const float* invstd, int N, int K, float* P, float* Gm,
                 float* Sa, float* sums, float* bn_grads, hipStream_t st);
// stage 2, from the (all-reduced) sums: abd [3N] = (A, B, D) -- the BatchNorm input gradient is A g + B y + D --
// and dW [N, K] (W's 16-bit type) = A P + (B W) Gm + D (x) Sa   (weight may be null = 1)
void fold_finish(int dt, const void* W, const float* sums, const float* count, const float* mean, const float* invstd,
                 const float* weight, const float* P, const float* Gm, const float* Sa, int N, int K, float* abd,
                 void* dW, hipStream_t st);

}  // namespace bh
