// MFMA GEMM with fused dense-layer epilogues (kernels: csrc/kernels/gemm.hip).
//
//   C[M,N] = epilogue( A[M,K] . B[N,K]^T )      A, B, C row-major, fp16 or bf16, fp32 accumulate
//
// Forward epilogue (bwd_act == false):  v = acc (+ bias[n]);  pre_out[m,n] = v (if given);
//                                       C = act(v)
// Backward epilogue (bwd_act == true):  v = acc * act'(aux_in[m,n]) (ReLU / sigmoid: aux is the
//                                       activation OUTPUT, GELU: the pre-activation); C = v; and, if
//                                       bgrad_part is given, bgrad_part[r][n] = sum over the r-th
//                                       64-row slab of v (fixed-order, no atomics; finalise with
//                                       gemm_colsum_finalize).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

struct GemmEpilogue {
  const void* bias = nullptr;     // [N]
  int act = 0;                    // DenseAct
  bool bwd_act = false;
  void* pre_out = nullptr;        // [M, ld_aux] forward pre-activation (GELU aux)
  const void* aux_in = nullptr;   // [M, ld_aux] backward
  int64_t ld_aux = 0;
  float* bgrad_part = nullptr;    // [gemm_bgrad_slabs(M), N]
  // [M, ldc] added to the accumulator before the epilogue (C = A.B^T + resid; forward epilogues of the
  // ping-pong kernel only: a call with resid needs K % 64 == 0)
  const void* resid = nullptr;
  // BatchNorm statistics of the output, per 64-row slab into stat_part [2][slabs][N] (no activation /
  // bias with these):
  //   1: sums of (c - kshift[n]) and its square, c the stored value (the next BatchNorm's statistics);
  //   2: with y = bn_y[m, n] (ld = ldc): dz = c * (y * bn_scale + bn_shift > 0 | !bn_relu), sums of dz
  //      and dz * (y - bn_mean[n]) (the previous BatchNorm's backward reduction)
  int bn_stats = 0;
  float* stat_part = nullptr;
  const float* kshift = nullptr;
  const void* bn_y = nullptr;
  const float* bn_scale = nullptr;
  const float* bn_shift = nullptr;
  const float* bn_mean = nullptr;
  bool bn_relu = true;
};

// Shape / layout requirements of the MFMA path (else the caller must fall back):
// K % 8 == 0, N % 8 == 0, lda / ldb / ldc / ld_aux % 8 == 0, 16-byte aligned bases.
bool gemm_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const void* A,
                    const void* B, const void* C);
int64_t gemm_bgrad_slabs(int64_t M);
void gemm_nt(int dt, const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
             int64_t N, int64_t K, const GemmEpilogue& epi, hipStream_t st);
// kernel choice: 0 auto (ping-pong 256x256 on large grids), 1 128x128, 2 256x256 one-barrier,
// 3 256x128 three-stage, 4 ping-pong forced (K % 64 == 0 only); default from BH_GEMM_TILE
int gemm_tile_mode();
void gemm_set_tile_mode(int mode);
// C [M, N] (16-bit) = At^T . Bt for At [K, M] (row stride lda) and Bt [K, N] (row stride ldb), both contiguous
// along M / N: a dense layer's weight gradient dY^T X (kernels/gemm_tn.hip, the ping-pong schedule with
// K-major LDS images and transposed fragment reads). M, N % 256 == 0, K % 64 == 0. splits > 1: split-K over
// the token axis into ws (fp32 [splits, M, N]) and a fixed-order reduction into C. accum: 0 C = result (16-bit),
// 1 C (fp32) += result, 2 C (16-bit) += result -- the last two always through ws (fused_weight_gradient_mlp's
// main_grad accumulation).
bool gemm_tn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* At, const void* Bt,
                       const void* C);
int gemm_tn_splits(int64_t M, int64_t N, int64_t K);
void gemm_tn(int dt, const void* At, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
             int64_t K, float* ws, int splits, hipStream_t st, int accum = 0);
// C [M, N] (16-bit) = A . Bt for row-major A [M, K] (lda) and Bt [K, N] (ldb, N-contiguous): a dense layer's
// data gradient dY . W, on the same kernel (A staged row-major, Bt through the transposed reads); split-K as
// gemm_tn (gemm_tn_splits picks the count).
bool gemm_nn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A, const void* Bt,
                       const void* C);
void gemm_nn(int dt, const void* A, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
             int64_t K, float* ws, int splits, hipStream_t st);
// out [C, R] = in [R, C]^T, 16-bit elements (R, C multiples of 8, 16-byte aligned)
void transpose16(const void* in, int64_t R, int64_t C, void* out, hipStream_t st);
// out[N] (dtype dt) = sum_r part[r][N]
void gemm_colsum_finalize(int dt, const float* part, int64_t slabs, int64_t N, void* out, hipStream_t st);

}  // namespace bh
