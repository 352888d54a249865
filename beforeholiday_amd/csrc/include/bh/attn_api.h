// Fused short-sequence attention (kernels/attn.hip): head_dim 64, sk <= 128, fp16 / bf16.
// Tensors are addressed as base + t * st + bh * sbh + d (t = time index, bh = batch*heads index,
// d < 64 contiguous), so q / k / v can be strided views into a fused QKV projection output and the
// gradients can be written straight into the fused QKV gradient.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

struct AttnArgs {
  const void* q = nullptr;
  const void* k = nullptr;
  const void* v = nullptr;
  void* o = nullptr;
  int64_t q_st = 0, q_sbh = 0, k_st = 0, k_sbh = 0, v_st = 0, v_sbh = 0, o_st = 0, o_sbh = 0;
  int sq = 0, sk = 0, heads = 1, BH = 0;
  int mask_mode = 0;            // 0 none, 1 key padding uint8 [B, sk], 2 additive fp32 [B, sk], 3 time uint8 [sq, sk]
  const void* mask = nullptr;
  float scale = 1.f, p_drop = 0.f;
  bool training = false;
  uint64_t seed = 0, offset = 0;
  // backward
  const void* dout = nullptr;
  int64_t do_st = 0, do_sbh = 0;
  void* dq = nullptr;
  void* dk = nullptr;
  void* dv = nullptr;
  int64_t dq_st = 0, dq_sbh = 0, dk_st = 0, dk_sbh = 0, dv_st = 0, dv_sbh = 0;
};

int attn_max_sk();
void attn_forward(int dt, const AttnArgs& a, hipStream_t st);
void attn_backward(int dt, const AttnArgs& a, hipStream_t st);

}  // namespace bh
