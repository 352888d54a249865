// Batch-norm launcher API (kernels: csrc/kernels/batchnorm.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

// Element (o, c, i) lives at o*C*inner + c*inner + i.
//   NCHW:           outer = N, inner = H*W
//   channels_last:  outer = N*H*W, inner = 1, channels_last = true (requires C % 8 == 0)
struct BNShape {
  int64_t outer;
  int C;
  int64_t inner;
  bool channels_last;
};

// Outputs of a statistics finalize / rank merge (any pointer may be null = not wanted).
struct BNFinal {
  float* mean;
  float* invstd;
  float* scale;   // w * invstd
  float* shift;   // b - mean * w * invstd
  float* count;   // total element count per channel (1 float)
  float eps;
  float momentum;        // running stats EMA factor; < 0 means cumulative average (momentum=None)
  int64_t* num_batches;  // optional num_batches_tracked counter, incremented on the device
};

int bn_num_splits(const BNShape& s);         // statistics partials
int bn_num_splits_reduce(const BNShape& s, bool masked = false);  // backward-reduction partials
// partial Welford stats: pmean/pm2 [splits][C]; pn [splits] (channels_last) or [splits][C] (NCHW)
void bn_stats(const BNShape& s, int dt_x, const void* x, int splits, float* pmean, float* pm2, float* pn,
              hipStream_t st);
// merge partials. out_local (may be null) receives [mean(C), var_biased(C), count(1)] (the
// all_gather payload); fin (if fin.mean) receives the single-rank final values.
void bn_stats_finalize(const BNShape& s, int splits, const float* pmean, const float* pm2, const float* pn,
                       float* out_local, const BNFinal& fin, int dt_w, const void* w, const void* b, void* rmean,
                       void* rvar, hipStream_t st, const void* kref = nullptr, float* out_sums = nullptr);
// out_sums (optional, [2C+1]): the all_reduce(SUM) payload [sum(x-K), sum((x-K)^2), n] about the shared
// per-channel reference K = kref (dtype dt_w; null = 0), finalized by bn_merge_sums after the reduction
void bn_merge_sums(int C, const float* sums, const BNFinal& fin, int dt_w, const void* w, const void* b, void* rmean,
                   void* rvar, hipStream_t st);
// single rank: sum a convolution epilogue's partials part [2][G][C] (the fixed bn_part_segments order) and
// finalize as bn_merge_sums with element count `count` -- one launch, or two with a segment workspace
// seg_ws [bn_part_segments(G)][2][C] fp32 when bn_part_segments(G) > 1
// (bump: also num_batches += 1, for a fixed momentum only)
void bn_merge_parts(int G, int C, const float* part, float count, const BNFinal& fin, int dt_w, const void* w,
                    const void* b, void* rmean, void* rvar, hipStream_t st, bool bump = false,
                    float* seg_ws = nullptr);
// merge W gathered rows [W][2C+1] into final stats (+ running stats update, scale/shift)
void bn_merge_ranks(int W, int C, const float* gathered, const BNFinal& fin, int dt_w, const void* w,
                    const void* b, void* rmean, void* rvar, float* var_unbiased, hipStream_t st);
// y = x*scale + shift (+z) (relu); dt_z = -1 when z is null
void bn_forward(const BNShape& s, int dt_x, const void* x, int dt_z, const void* z, int dt_y, void* y,
                const float* scale, const float* shift, bool relu, int64_t* counter, hipStream_t st,
                uint8_t* mbits = nullptr,  // mbits: optional [rows][C/8] ReLU bit mask (NHWC, C % 8 == 0)
                const float* zscale = nullptr, const float* zshift = nullptr);  // z -> z * zscale + zshift
// partial sums of dy' and dy'*(x-mean); dy' = dy masked by (x*scale+shift(+z) > 0) when relu
void bn_backward_reduce(const BNShape& s, int dt, const void* dy, const void* x, int dt_z, const void* z,
                        const float* mean, const float* scale, const float* shift, bool relu, int splits,
                        float* p_dy, float* p_dyx, hipStream_t st, const uint8_t* mbits = nullptr);
// sums[2C] = (sum_dy, sum_dy_xmu); grad_w = sum_dy_xmu*invstd; grad_b = sum_dy (may be null)
void bn_backward_reduce_finalize(int C, int splits, const float* p_dy, const float* p_dyx, const float* invstd,
                                 float* sums, int dt_w, void* gw, void* gb, hipStream_t st);
// dx (and dz = dy' when dz != null); count = total elements per channel across ranks (device)
void bn_backward_dgrad(const BNShape& s, int dt, const void* dy, const void* x, int dt_z, const void* z,
                       const float* mean, const float* invstd, int dt_w, const void* w, const float* sums,
                       const float* count, const float* scale, const float* shift, bool relu, void* dx, void* dz,
                       hipStream_t st, const uint8_t* mbits = nullptr);

}  // namespace bh
