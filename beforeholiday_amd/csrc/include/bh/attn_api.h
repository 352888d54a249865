// Fused attention (kernels/attn.hip), head_dim 64, fp16 / bf16:
//  * attn_forward / attn_backward: short sequences (sk <= 128), whole key row in registers.
//  * flash_forward / flash_backward: any length, 64-key blocks with online softmax; forward also
//    writes the per-row log-sum-exp (fp32 [BH, sq]) that backward uses to rebuild P, and backward
//    takes delta = rowsum(dO * O) (fp32 [BH, sq], flash_delta) and runs a dK/dV kernel (one
//    workgroup per key block) plus a dQ kernel (one per query block): no atomics, deterministic.
// Tensors are addressed as base + t * st + bh * sbh + d (t = time index, bh = batch*heads index,
// d < 64 contiguous), so q / k / v can be strided views into a fused QKV projection output and the
// gradients can be written straight into the fused QKV gradient.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace bh {

struct AttnArgs {
  const void* q = nullptr;
  const void* k = nullptr;
  const void* v = nullptr;
  void* o = nullptr;
  int64_t q_st = 0, q_sbh = 0, k_st = 0, k_sbh = 0, v_st = 0, v_sbh = 0, o_st = 0, o_sbh = 0;
  int sq = 0, sk = 0, heads = 1, BH = 0;
  // 0 none, 1 key padding uint8 [B, sk], 2 additive fp32 [B, sk], 3 time uint8 [sq, sk],
  // 4 full uint8 [B, sq, sk] (broadcast over heads), 5 causal (key > query masked, no tensor)
  int mask_mode = 0;
  float mask_fill = -INFINITY;  // value of a masked score (-inf: MHA semantics; -10000: Megatron)
  const void* mask = nullptr;
  float scale = 1.f, p_drop = 0.f;
  bool training = false;
  uint64_t seed = 0, offset = 0;
  // device-resident step seed (utils/graph_rng.py: a captured step replays with a fresh one): the
  // dropout then keys on seed ^ (*seed_dev * golden ratio), read once per row hash (scalar load)
  const int64_t* seed_dev = nullptr;
  // backward
  const void* dout = nullptr;
  int64_t do_st = 0, do_sbh = 0;
  void* dq = nullptr;
  void* dk = nullptr;
  void* dv = nullptr;
  int64_t dq_st = 0, dq_sbh = 0, dk_st = 0, dk_sbh = 0, dv_st = 0, dv_sbh = 0;
  // flash
  float* lse = nullptr;          // [BH, sq]
  const float* delta = nullptr;  // [BH, sq]
  // mode 4 as bits for the 32x32 flash kernels (flash_mask_bits): mbits [B, sq, ceil(sk/32)] words
  // over keys (bit j of word w = key 32w+j), mbits_t [B, sk, ceil(sq/32)] words over queries
  const uint32_t* mbits = nullptr;
  const uint32_t* mbits_t = nullptr;
  // varlen: int32 [B + 1] prefix sums of the sequence lengths (device). The q/k/v/o/grad tensors are
  // then packed [total_tokens, heads, 64] (st = token stride, sbh = head stride), BH = B * heads,
  // sq = sk = max_s, lse / delta [BH, max_s]. Flash 32x32 kernels, mask modes 0 / 5.
  const int* cu_seqlens = nullptr;
};

int attn_max_sk();
void attn_forward(int dt, const AttnArgs& a, hipStream_t st);
void attn_backward(int dt, const AttnArgs& a, hipStream_t st);
void flash_forward(int dt, const AttnArgs& a, hipStream_t st);          // needs a.lse
// delta[bh, q] = sum_d dout * o  (o given in a.o / a.o_st / a.o_sbh, dout in a.dout)
void flash_delta(int dt, const AttnArgs& a, float* delta, hipStream_t st);
void flash_backward(int dt, const AttnArgs& a, hipStream_t st);         // needs a.lse, a.delta
// packs the mode-4 uint8 mask a.mask into bits (see AttnArgs::mbits); bits_t may be null
void flash_mask_bits(const AttnArgs& a, uint32_t* bits, uint32_t* bits_t, hipStream_t st);

}  // namespace bh
