// 2:4 sparsity channel-permutation search launchers (kernels: csrc/kernels/sparsity.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

constexpr int kStripeSplits = 35;  // ways to split 8 columns into two unordered groups of 4

// Sum of |m| kept by 2:4 pruning along rows of m [R, C] (fp32, C % 4 == 0) -> out[0] (fp32).
// `part` holds perm_sum_parts() floats of scratch.
int perm_sum_parts(int64_t R, int64_t C);
void perm_sum_after_2to4(const float* m, int64_t R, int64_t C, float* part, float* out, hipStream_t st);

// For each stripe pair (pairs[2p], pairs[2p+1]) (a stripe = 4 consecutive columns): the best of the
// 35 re-splits of their 8 columns into two stripes, as gain over the current split of the kept 2:4
// magnitude summed over the R rows (gain[p]) and the split index (split[p], 0 = current layout).
void perm_stripe_pair_gains(const float* m, int64_t R, int64_t C, const int32_t* pairs, int64_t npairs, float* gain,
                            int32_t* split, hipStream_t st);

}  // namespace bh
