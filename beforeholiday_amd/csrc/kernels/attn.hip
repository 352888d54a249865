// Fused short-sequence attention for the contrib multi-head-attention block (gfx950, MFMA).
//
// Replaces the reference's strided-batched-GEMM -> masked softmax -> dropout -> strided-batched-GEMM
// pipeline (apex/contrib/csrc/multihead_attn/self_multihead_attn_cuda.cu, softmax.cuh,
// dropout.cuh) for head_dim 64 and up to 128 keys (the reference MHA benchmark runs seq 64,
// apex/contrib/examples/multihead_attn/perf_test_multihead_attn.py:9): scores, probabilities and
// the dropout mask never touch HBM.
//
// Forward, one workgroup = 4 waves = 64 query rows of one (batch, head):
//  * K and V of the head are staged once in LDS (128-B rows, XOR-swizzled 16-B chunks); each wave
//    keeps its 16 query rows' Q fragments in registers (read straight from the strided QKV
//    projection output: no transpose copy).
//  * S = Q.K^T with v_mfma_f32_16x16x32; the whole key row lives in one 16-lane group, so the
//    masked softmax is an in-register max/sum with 4 xor-shuffles, exact (no online rescaling).
//  * dropout: Philox4x32-10 keyed by (seed, head, 4-row group, key) -> one call per lane per
//    16-key tile; regenerated in backward, never stored.
//  * P goes through a per-wave LDS image into the A operand of O = P.V; V^T fragments come from
//    the row-major V image through ds_read_b64_tr_b16 (hardware transpose read).
//  * O is written in [time, batch*heads, 64] order = the [tokens, embed] input of the output
//    projection.
// Backward, one workgroup = one (batch, head), looping over 64-row query blocks:
//  * recompute S and P exactly (full rows), dP = dO.V^T, delta = rowsum(P * dP_dropped),
//    dS = P * (dP_dropped - delta) * scale;
//  * dQ = dS.K per wave (own rows), dV += Pd^T.dO and dK += dS^T.Q with the transposed operands
//    read by ds_read_b64_tr_b16 from the row-major Pd / dS / dO / Q images; dK and dV stay in
//    registers across query blocks (no atomics), written once at the end straight into the
//    [time, batch*heads, {q,k,v}, 64] gradient of the QKV projection.
#include "bh/api.h"
#include "bh/attn_api.h"
#include "bh/device.h"

#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <string>

namespace bh {
namespace {

// the dropout seed of a launch: the host seed, keyed by the device step seed when one is given
BH_DEVICE uint64_t eff_seed(const AttnArgs& a) {
  return a.seed_dev ? a.seed ^ ((uint64_t)*a.seed_dev * 0x9E3779B97F4A7C15ull) : a.seed;
}

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;

constexpr int D = 64;          // head dim
constexpr int kThreads = 256;  // 4 waves
constexpr int kQB = 64;        // query rows per block

template <typename T> struct Mfma;
template <> struct Mfma<f16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma<bf16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0,
                                                   0);
  }
};

// byte offset of 16-B chunk `ch` of `row` in a row-major image with `rb`-byte rows (XOR swizzle)
BH_DEVICE int img_off(int row, int ch, int rb) { return row * rb + ((ch ^ ((row >> 1) & 7)) << 4); }
// byte offset of element (row, col) (16-bit elements)
BH_DEVICE int img_elem(int row, int col, int rb) { return img_off(row, col >> 3, rb) + ((col & 7) << 1); }

// 16x16x32 operand fragment read by rows: lane holds image[r0 + (lane&15)][c0 + 8*(lane>>4) + 0..7]
BH_DEVICE i4v frag_row(const char* img, int rb, int r0, int c0, int lane) {
  return *reinterpret_cast<const i4v*>(img + img_off(r0 + (lane & 15), (c0 >> 3) + (lane >> 4), rb));
}
// transposed fragment: lane holds image[k0 + 8*(lane>>4) + 0..7][n0 + (lane&15)] (two tr16 reads)
BH_DEVICE i4v frag_tr(const char* img, int rb, int k0, int n0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r = k0 + 8 * g + q;
  const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + img_elem(r, n0 + 4 * p, rb)));
  const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + img_elem(r + 4, n0 + 4 * p, rb)));
  i4v out;
  out[0] = (int)(uint16_t)lo[0] | ((int)(uint16_t)lo[1] << 16);
  out[1] = (int)(uint16_t)lo[2] | ((int)(uint16_t)lo[3] << 16);
  out[2] = (int)(uint16_t)hi[0] | ((int)(uint16_t)hi[1] << 16);
  out[3] = (int)(uint16_t)hi[2] | ((int)(uint16_t)hi[3] << 16);
  return out;
}

// stage `rows` x 64 head rows (16-bit) from global (row stride `st` elements) into an image with
// 128-B rows; rows >= valid are zero-filled.
template <typename T>
BH_DEVICE void stage_rows(char* img, const T* src, int64_t st, int rows, int valid, int tid) {
  for (int idx = tid; idx < rows * 8; idx += kThreads) {
    const int r = idx >> 3, ch = idx & 7;
    i4v v = i4v{0, 0, 0, 0};
    if (r < valid) v = *reinterpret_cast<const i4v*>(src + (int64_t)r * st + ch * 8);
    *reinterpret_cast<i4v*>(img + img_off(r, ch, 128)) = v;
  }
}

BH_DEVICE float wmax16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
BH_DEVICE float wsum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// masked, scaled score of (query row q, key col k); -inf when masked / out of range
BH_DEVICE float apply_mask(float s, const AttnArgs& a, int b, int q, int k) {
  if (k >= a.sk) return -INFINITY;  // padding columns of the last key block never count
  const uint8_t* m8 = reinterpret_cast<const uint8_t*>(a.mask);
  switch (a.mask_mode) {
    case 1: return m8[(int64_t)b * a.sk + k] ? a.mask_fill : s;
    case 2: return s + reinterpret_cast<const float*>(a.mask)[(int64_t)b * a.sk + k];
    case 3: return (q < a.sq && m8[(int64_t)q * a.sk + k]) ? a.mask_fill : s;
    case 4: return (q < a.sq && m8[((int64_t)b * a.sq + q) * a.sk + k]) ? a.mask_fill : s;
    case 5: return k > q ? a.mask_fill : s;
    default: return s;
  }
}

// true when the mask REPLACES the score (fill value; blocks the gradient like masked_fill)
BH_DEVICE bool is_masked(const AttnArgs& a, int b, int q, int k) {
  if (k >= a.sk) return true;
  const uint8_t* m8 = reinterpret_cast<const uint8_t*>(a.mask);
  switch (a.mask_mode) {
    case 1: return m8[(int64_t)b * a.sk + k] != 0;
    case 3: return q < a.sq && m8[(int64_t)q * a.sk + k] != 0;
    case 4: return q < a.sq && m8[((int64_t)b * a.sq + q) * a.sk + k] != 0;
    case 5: return k > q;
    default: return false;
  }
}

// P (softmax of one wave's 16 rows, C/D layout: row 4*(lane>>4)+j, key 16n+(lane&15)) from S
template <int NT>
BH_DEVICE void softmax_rows(f4v (&S)[NT], const AttnArgs& a, int b, int qbase, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = apply_mask(S[n][j] * a.scale, a, b, qbase + 4 * fq + j, 16 * n + fr);
      S[n][j] = v;
      mx[j] = fmaxf(mx[j], v);
    }
  float sum[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mx[j] = wmax16(mx[j]);
    sum[j] = 0.f;
  }
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = mx[j] == -INFINITY ? 0.f : __expf(S[n][j] - mx[j]);
      S[n][j] = e;
      sum[j] += e;
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s = wsum16(sum[j]);
    sum[j] = s > 0.f ? 1.f / s : 0.f;  // fully masked row -> zeros
  }
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int j = 0; j < 4; ++j) S[n][j] *= sum[j];
}

// keep flags of the 4 rows (4-row group starting at qrow4) for key col
BH_DEVICE float4 keep4(const AttnArgs& a, int bh, int qrow4, int col, int skt) {
  Philox ph(eff_seed(a), ((uint64_t)bh * (uint64_t)a.sq + (uint64_t)qrow4) * (uint64_t)skt + (uint64_t)col, a.offset);
  const float4 u = ph.uniform4();
  const float pk = 1.f - a.p_drop;
  return make_float4(u.x <= pk, u.y <= pk, u.z <= pk, u.w <= pk);
}

template <typename T, int SKT>
__global__ __launch_bounds__(kThreads) void k_attn_fwd(AttnArgs a) {
  constexpr int NT = SKT / 16;
  constexpr int PRB = SKT * 2;  // P image row bytes
  __shared__ __attribute__((aligned(16))) char smem[2 * SKT * 128 + kQB * PRB];
  char* kimg = smem;
  char* vimg = smem + SKT * 128;
  char* pimg = smem + 2 * SKT * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.y, b = bh / a.heads;
  const int qbase = blockIdx.x * kQB + wave * 16;

  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  stage_rows<T>(kimg, K, a.k_st, SKT, a.sk, tid);
  stage_rows<T>(vimg, V, a.v_st, SKT, a.sk, tid);
  i4v qa[2];
  {
    const int qr = min(qbase + fr, a.sq - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qa[s] = *reinterpret_cast<const i4v*>(Q + (int64_t)qr * a.q_st + 32 * s + 8 * fq);
  }
  __syncthreads();

  f4v S[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    S[n] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) S[n] = Mfma<T>::run(qa[s], frag_row(kimg, 128, 16 * n, 32 * s, lane), S[n]);
  }
  softmax_rows<NT>(S, a, b, qbase, lane);
  const bool drop = a.training && a.p_drop > 0.f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  T* prow = reinterpret_cast<T*>(pimg);
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    float4 kp = make_float4(1.f, 1.f, 1.f, 1.f);
    if (drop) kp = keep4(a, bh, qbase + 4 * fq, 16 * n + fr, SKT);
    const float kk[4] = {kp.x * kscale, kp.y * kscale, kp.z * kscale, kp.w * kscale};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float pv = drop ? S[n][j] * kk[j] : S[n][j];
      const int row = wave * 16 + 4 * fq + j;
      *reinterpret_cast<T*>(pimg + img_elem(row, 16 * n + fr, PRB)) = from_f<T>(pv);
    }
  }
  (void)prow;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's P rows are written (wave-private)

  f4v O[4];
#pragma unroll
  for (int dn = 0; dn < 4; ++dn) O[dn] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < SKT / 32; ++ks) {
    const i4v pa = frag_row(pimg, PRB, wave * 16, 32 * ks, lane);
#pragma unroll
    for (int dn = 0; dn < 4; ++dn) O[dn] = Mfma<T>::run(pa, frag_tr(vimg, 128, 32 * ks, 16 * dn, lane), O[dn]);
  }
  T* Out = reinterpret_cast<T*>(a.o) + (int64_t)bh * a.o_sbh;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = qbase + 4 * fq + j;
    if (q < a.sq) {
#pragma unroll
      for (int dn = 0; dn < 4; ++dn) Out[(int64_t)q * a.o_st + 16 * dn + fr] = from_f<T>(O[dn][j]);
    }
  }
}

template <typename T, int SKT>
__global__ __launch_bounds__(kThreads) void k_attn_bwd(AttnArgs a) {
  constexpr int NT = SKT / 16;
  constexpr int PRB = SKT * 2;
  constexpr int MT = SKT / 64;  // 16-row key tiles owned per wave for dK / dV
  __shared__ __attribute__((aligned(16))) char smem[2 * SKT * 128 + 2 * kQB * 128 + 2 * kQB * PRB];
  char* kimg = smem;
  char* vimg = kimg + SKT * 128;
  char* qimg = vimg + SKT * 128;
  char* doimg = qimg + kQB * 128;
  char* pdimg = doimg + kQB * 128;
  char* dsimg = pdimg + kQB * PRB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.x, b = bh / a.heads;

  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)bh * a.do_sbh;
  stage_rows<T>(kimg, K, a.k_st, SKT, a.sk, tid);
  stage_rows<T>(vimg, V, a.v_st, SKT, a.sk, tid);

  f4v dK[MT][4], dV[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) dK[m][n] = dV[m][n] = f4v{0.f, 0.f, 0.f, 0.f};

  const bool drop = a.training && a.p_drop > 0.f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  T* dQ = reinterpret_cast<T*>(a.dq) + (int64_t)bh * a.dq_sbh;

  for (int q0 = 0; q0 < a.sq; q0 += kQB) {
    const int valid = min(kQB, a.sq - q0);
    stage_rows<T>(qimg, Q + (int64_t)q0 * a.q_st, a.q_st, kQB, valid, tid);
    stage_rows<T>(doimg, dO + (int64_t)q0 * a.do_st, a.do_st, kQB, valid, tid);
    __syncthreads();
    const int qbase = q0 + wave * 16;
    f4v S[NT], dP[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      S[n] = dP[n] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        S[n] = Mfma<T>::run(frag_row(qimg, 128, wave * 16, 32 * s, lane), frag_row(kimg, 128, 16 * n, 32 * s, lane),
                            S[n]);
        dP[n] = Mfma<T>::run(frag_row(doimg, 128, wave * 16, 32 * s, lane),
                             frag_row(vimg, 128, 16 * n, 32 * s, lane), dP[n]);
      }
    }
    softmax_rows<NT>(S, a, b, qbase, lane);
    // dropout on dP, delta = rowsum(P * dPd)
    float delta[4] = {0.f, 0.f, 0.f, 0.f};
    float4 keeps[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      keeps[n] = make_float4(1.f, 1.f, 1.f, 1.f);
      if (drop) keeps[n] = keep4(a, bh, qbase + 4 * fq, 16 * n + fr, SKT);
      const float kk[4] = {keeps[n].x, keeps[n].y, keeps[n].z, keeps[n].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool rv = qbase + 4 * fq + j < a.sq;
        if (!rv) S[n][j] = 0.f;
        dP[n][j] = drop ? dP[n][j] * kk[j] * kscale : dP[n][j];
        delta[j] += S[n][j] * dP[n][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) delta[j] = wsum16(delta[j]);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const float kk[4] = {keeps[n].x, keeps[n].y, keeps[n].z, keeps[n].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wave * 16 + 4 * fq + j;
        const float ds = S[n][j] * (dP[n][j] - delta[j]) * a.scale;
        const float pd = drop ? S[n][j] * kk[j] * kscale : S[n][j];
        *reinterpret_cast<T*>(pdimg + img_elem(row, 16 * n + fr, PRB)) = from_f<T>(pd);
        *reinterpret_cast<T*>(dsimg + img_elem(row, 16 * n + fr, PRB)) = from_f<T>(ds);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // dQ (own rows) = dS . K
    {
      f4v acc[4];
#pragma unroll
      for (int dn = 0; dn < 4; ++dn) acc[dn] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < SKT / 32; ++ks) {
        const i4v da = frag_row(dsimg, PRB, wave * 16, 32 * ks, lane);
#pragma unroll
        for (int dn = 0; dn < 4; ++dn) acc[dn] = Mfma<T>::run(da, frag_tr(kimg, 128, 32 * ks, 16 * dn, lane), acc[dn]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = qbase + 4 * fq + j;
        if (q < a.sq) {
#pragma unroll
          for (int dn = 0; dn < 4; ++dn) dQ[(int64_t)q * a.dq_st + 16 * dn + fr] = from_f<T>(acc[dn][j]);
        }
      }
    }
    __syncthreads();  // Pd / dS images complete
    // dV += Pd^T . dO, dK += dS^T . Q over this block's 64 query rows (2 k-slices of 32)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int key0 = wave * (SKT / 4) + 16 * m;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const i4v pa = frag_tr(pdimg, PRB, 32 * ks, key0, lane);
        const i4v sa = frag_tr(dsimg, PRB, 32 * ks, key0, lane);
#pragma unroll
        for (int dn = 0; dn < 4; ++dn) {
          dV[m][dn] = Mfma<T>::run(pa, frag_tr(doimg, 128, 32 * ks, 16 * dn, lane), dV[m][dn]);
          dK[m][dn] = Mfma<T>::run(sa, frag_tr(qimg, 128, 32 * ks, 16 * dn, lane), dK[m][dn]);
        }
      }
    }
    __syncthreads();  // before the next block restages the images
  }
  T* dKp = reinterpret_cast<T*>(a.dk) + (int64_t)bh * a.dk_sbh;
  T* dVp = reinterpret_cast<T*>(a.dv) + (int64_t)bh * a.dv_sbh;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = wave * (SKT / 4) + 16 * m + 4 * fq + j;
      if (key < a.sk) {
#pragma unroll
        for (int dn = 0; dn < 4; ++dn) {
          dKp[(int64_t)key * a.dk_st + 16 * dn + fr] = from_f<T>(dK[m][dn][j]);
          dVp[(int64_t)key * a.dv_st + 16 * dn + fr] = from_f<T>(dV[m][dn][j]);
        }
      }
    }
}

// =============================================================================================
// Flash kernels: 64-key blocks, online softmax (forward), LSE-rebuilt probabilities (backward).
// Dropout keep flags use the same Philox mapping as the short kernels with skt = round_up(sk, 64).
// Every streamed 64-row operand block is prefetched into registers while the previous block is
// being computed and written to the other of two LDS buffers afterwards (one barrier per block);
// mask data for the block (key flags / additive row / [64 q x 64 k] byte tile) rides along, so the
// inner loop never issues a global load.
// =============================================================================================
constexpr int kKB = 64;  // keys per block

BH_DEVICE int skt_pad(int sk) { return (sk + kKB - 1) / kKB * kKB; }

// XCD-aware (tile, head) of a flash workgroup on a (tiles, BH) grid. Workgroups are dispatched in
// x-fastest order and dealt round-robin to the 8 XCDs (linear id % 8), so the natural mapping
// spreads the tiles of one head over all 8 XCDs and every XCD's L2 misses on the same K / V
// (or Q / dO) panels. This bijection keeps all tiles of a head on one XCD: the 8 XCDs each own
// every 8th head. Falls back to the natural order when BH % 8 != 0.
BH_DEVICE void flash_tile(int& tile, int& bh) {
  const int nx = gridDim.x, ny = gridDim.y;
  if (ny & 7) {
    tile = blockIdx.x;
    bh = blockIdx.y;
    return;
  }
  const int id = blockIdx.x + blockIdx.y * nx;
  const int slot = id >> 3;
  tile = slot % nx;
  bh = (slot / nx) * 8 + (id & 7);
}

// Variable-length packed sequences (AttnArgs::cu_seqlens; the reference's fmhalib takes cu_seqlens,
// apex/contrib/csrc/fmha/fmha_api.cpp:358-360): problem bh = (sequence b, head hd) owns tokens
// cu[b] .. cu[b+1]-1 of the packed q / k / v / o / dO / dQ / dK / dV (token stride *_st, head stride
// *_sbh), and lse / delta stay [BH, max_s] with a.sq = a.sk = max_s on entry. The kernels address a
// problem as base + bh * sbh + row * st with a.sq / a.sk rows, so rebasing every pointer by
// (cu[b] * st + hd * sbh - bh * sbh) and setting sq = sk = the sequence length lets the same code run
// on the packed tokens: no padding copy, no host read of the lengths. Returns false when the tile
// starting at row ``first`` lies past the sequence (the whole workgroup exits).
template <typename T>
BH_DEVICE bool varlen_rebase(AttnArgs& a, int bh, int first) {
  const int b = bh / a.heads, hd = bh - b * a.heads;
  const int s0 = a.cu_seqlens[b];
  const int n = min(a.cu_seqlens[b + 1] - s0, a.sq);  // max_s bounds the lse / delta rows of a problem
  if (first >= n) return false;
  auto cshift = [&](const void*& p, int64_t st, int64_t sbh) {
    if (p) p = reinterpret_cast<const T*>(p) + (int64_t)s0 * st + (int64_t)hd * sbh - (int64_t)bh * sbh;
  };
  auto shift = [&](void*& p, int64_t st, int64_t sbh) {
    if (p) p = reinterpret_cast<T*>(p) + (int64_t)s0 * st + (int64_t)hd * sbh - (int64_t)bh * sbh;
  };
  cshift(a.q, a.q_st, a.q_sbh);
  cshift(a.k, a.k_st, a.k_sbh);
  cshift(a.v, a.v_st, a.v_sbh);
  cshift(a.dout, a.do_st, a.do_sbh);
  shift(a.o, a.o_st, a.o_sbh);
  shift(a.dq, a.dq_st, a.dq_sbh);
  shift(a.dk, a.dk_st, a.dk_sbh);
  shift(a.dv, a.dv_st, a.dv_sbh);
  const int64_t d = (int64_t)bh * (a.sq - n);  // lse[bh * max_s + q] == lse'[bh * n + q]
  if (a.lse) a.lse += d;
  if (a.delta) a.delta += d;
  a.sq = a.sk = n;
  return true;
}

// 64 rows x 128 B of a head operand: 2 x 16-byte chunks per thread. The loads are unconditional
// (rows past `valid` re-read the last valid row) and the zero fill of those rows happens when the
// registers are written to LDS: a select right after a load would make the compiler wait for the
// load there, in front of the block's compute, instead of letting it fly under it.
struct RowRegs {
  i4v v[2];
  int valid;
};
template <typename T>
BH_DEVICE void rows_load(RowRegs& r, const T* src, int64_t st, int valid, int tid) {
  r.valid = valid;
  if (valid >= 64) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * kThreads;
      r.v[i] = *reinterpret_cast<const i4v*>(src + (int64_t)(idx >> 3) * st + (idx & 7) * 8);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * kThreads;
      r.v[i] = *reinterpret_cast<const i4v*>(src + (int64_t)min(idx >> 3, valid - 1) * st + (idx & 7) * 8);
    }
  }
}
BH_DEVICE i4v rows_val(const RowRegs& r, int i, int tid) {
  return ((tid + i * kThreads) >> 3) < r.valid ? r.v[i] : i4v{0, 0, 0, 0};
}
BH_DEVICE void rows_store(char* img, const RowRegs& r, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + i * kThreads;
    *reinterpret_cast<i4v*>(img + img_off(idx >> 3, idx & 7, 128)) = rows_val(r, i, tid);
  }
}

// mask data of one (64 q rows) x (64 keys) block, staged in LDS: 4 KiB byte tile for modes 3 / 4,
// 64 key flags (mode 1) or 64 additive floats (mode 2)
constexpr int kMaskBytes = 64 * 64;
struct MaskRegs {
  int4 t;  // one 16-byte piece per thread (tile row = tid/4, cols 16*(tid%4)) or the key vector
};
template <int MODE>
BH_DEVICE void mask_load(MaskRegs& m, const AttnArgs& a, int b, int q0, int k0, int tid) {
  // one 16-byte vector load per thread when the piece is in bounds and aligned (every piece but the
  // key tail when sk % 16 == 0); the byte-wise tail path is taken by whole pieces, never per byte
  // inside a vector load (a per-element select there makes hipcc wait on every load).
  m.t = make_int4(0, 0, 0, 0);
  const uint8_t* m8 = reinterpret_cast<const uint8_t*>(a.mask);
  const bool aligned = (a.sk & 15) == 0;
  if (MODE == 3 || MODE == 4) {
    const int r = tid >> 2, c = (tid & 3) * 16, q = q0 + r;
    if (q < a.sq) {
      const uint8_t* src = (MODE == 3 ? m8 + (int64_t)q * a.sk : m8 + ((int64_t)b * a.sq + q) * a.sk) + k0 + c;
      if (aligned && k0 + c + 16 <= a.sk) {
        m.t = *reinterpret_cast<const int4*>(src);
      } else {
        uint8_t buf[16];
        for (int i = 0; i < 16; ++i) buf[i] = (k0 + c + i < a.sk) ? src[i] : 1;
        m.t = *reinterpret_cast<const int4*>(buf);
      }
    }
  } else if (MODE == 1 && tid < 4) {
    const uint8_t* src = m8 + (int64_t)b * a.sk + k0 + tid * 16;
    if (aligned && k0 + tid * 16 + 16 <= a.sk) {
      m.t = *reinterpret_cast<const int4*>(src);
    } else {
      uint8_t buf[16];
      for (int i = 0; i < 16; ++i) buf[i] = (k0 + tid * 16 + i < a.sk) ? src[i] : 1;
      m.t = *reinterpret_cast<const int4*>(buf);
    }
  } else if (MODE == 2 && tid < 16) {
    const float* src = reinterpret_cast<const float*>(a.mask) + (int64_t)b * a.sk + k0 + tid * 4;
    if ((a.sk & 3) == 0 && k0 + tid * 4 + 4 <= a.sk) {
      m.t = *reinterpret_cast<const int4*>(src);
    } else {
      float buf[4];
      for (int i = 0; i < 4; ++i) buf[i] = (k0 + tid * 4 + i < a.sk) ? src[i] : 0.f;
      m.t = *reinterpret_cast<const int4*>(buf);
    }
  }
}
template <int MODE>
BH_DEVICE void mask_store(char* img, const MaskRegs& m, const AttnArgs& a, int tid) {
  if (MODE == 3 || MODE == 4) *reinterpret_cast<int4*>(img + tid * 16) = m.t;
  else if ((MODE == 1 && tid < 4) || (MODE == 2 && tid < 16)) *reinterpret_cast<int4*>(img + tid * 16) = m.t;
}
// (masked?, score) for local query row ql (0..63 of the block), local key kl, global q / k
template <int MODE>
BH_DEVICE float mask_apply(float s, const AttnArgs& a, const char* mimg, int ql, int kl, int q, int k, bool& masked) {
  masked = false;
  if (k >= a.sk) {
    masked = true;
    return -INFINITY;
  }
  switch (MODE) {
    case 1: masked = mimg[kl] != 0; break;
    case 2: return s + reinterpret_cast<const float*>(mimg)[kl];
    case 3:
    case 4: masked = mimg[ql * 64 + kl] != 0; break;
    case 5: masked = k > q; break;
    default: break;
  }
  return masked ? a.mask_fill : s;
}

// ---- operand helpers of the register-resident P formulation ----------------------------------
// A 16x16x32 operand whose k index is the ROW of a row-major image, in the k order in which two
// stacked C/D tiles (rows 0-15, 16-31 of a 32-deep step) already sit in a lane's registers:
// element e of lane group g <-> row k0 + 16*(e>>2) + 4*g + (e&3). Two ds_read_b64_tr_b16.
BH_DEVICE i4v frag_tr_perm(const char* img, int rb, int k0, int n0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r = k0 + 4 * g + q;
  const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + img_elem(r, n0 + 4 * p, rb)));
  const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + img_elem(r + 16, n0 + 4 * p, rb)));
  // the two 4 x 16-bit results already sit in the operand's dword order: reinterpret, no repacking
  typedef int bh_i2v __attribute__((ext_vector_type(2)));
  const bh_i2v l = __builtin_bit_cast(bh_i2v, lo), h = __builtin_bit_cast(bh_i2v, hi);
  return i4v{l[0], l[1], h[0], h[1]};
}
// the matching B (or A) operand straight from two accumulator tiles (no lane movement, no LDS)
template <typename T> BH_DEVICE i4v pack_pair(const f4v& lo, const f4v& hi) {
  T v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = from_f<T>(lo[j]);
    v[4 + j] = from_f<T>(hi[j]);
  }
  return *reinterpret_cast<const i4v*>(v);
}
// store 4 consecutive head-dim values (C/D rows 4g..4g+3 of one d-tile) with one 8-byte store
template <typename T> BH_DEVICE void store4(T* dst, const f4v& v, float mul) {
  T o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = from_f<T>(v[j] * mul);
  *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(o);
}

// counter-based dropout for the flash kernels: a 32-bit avalanche hash of (seed, head, query) per
// row and of (row hash, key) per element. It is independent of the lane layout, so the forward
// and dQ kernels (query on the lane) and the dK/dV kernel (key on the lane) regenerate the same
// keep mask; cheaper per element than Philox4x32-10 split four ways.
BH_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
BH_DEVICE uint32_t row_hash(const AttnArgs& a, int bh, int q) {
  const uint64_t s = eff_seed(a);
  return mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) ^ ((uint32_t)bh * 0x9E3779B1u) ^ ((uint32_t)q * 0x85EBCA77u)));
}
// one 32-bit hash per (query, key pair): keys 2i and 2i+1 use its low / high 16 bits, so the
// query-on-lane kernels (forward, dQ) hash once per two scores; thresh is (1 - p) * 65536. The row
// hash is a full avalanche; per pair a Weyl step, a 16-bit fold, ONE 32-bit multiply and a fold
// (the multiply is a quarter-rate instruction: this is the per-score cost of dropout).
BH_DEVICE uint32_t fold16(uint32_t x) { return x ^ (x >> 16); }
BH_DEVICE uint32_t pair_hash(uint32_t rowh, int k) {
  return fold16(fold16(rowh + (uint32_t)(k >> 1) * 0x9E3779B9u) * 0x7feb352du);
}
BH_DEVICE bool keep_elem(uint32_t rowh, int k, uint32_t thresh) {
  const uint32_t h = pair_hash(rowh, k);
  return ((k & 1) ? (h >> 16) : (h & 0xffffu)) < thresh;
}
// keep flags of keys k0, k0+1 (k0 even)
BH_DEVICE void keep_pair(uint32_t rowh, int k0, uint32_t thresh, bool& a, bool& b) {
  const uint32_t h = pair_hash(rowh, k0);
  a = (h & 0xffffu) < thresh;
  b = (h >> 16) < thresh;
}
BH_DEVICE uint32_t keep_thresh(float p) {
  const double t = (1.0 - (double)p) * 65536.0;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}

// Forward. Workgroup = 64 query rows x one head; wave w = 16 rows, query on the LANE: S^T = K.Q^T
// puts each query's 16 scores of a 64-key block in one lane's registers, so the online-softmax max
// and sum are in-lane plus two xor-shuffles, and P^T feeds O^T = V^T.P^T as the B operand without
// leaving registers. K / V / mask blocks are double-buffered through LDS.
template <typename T, int MODE>
__global__ __launch_bounds__(kThreads) void k_flash_fwd(AttnArgs a) {
  constexpr int kBuf = 2 * kKB * 128 + kMaskBytes;
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  int qtile, bh;
  flash_tile(qtile, bh);
  const int b = bh / a.heads;
  const int q0 = qtile * kQB;
  const int myq = q0 + wave * 16 + fr;  // this lane's query

  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  i4v qb[2];
  {
    const int qr = min(myq, a.sq - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qb[s] = *reinterpret_cast<const i4v*>(Q + (int64_t)qr * a.q_st + 32 * s + 8 * fq);
  }
  const bool drop = a.training && a.p_drop > 0.f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  const uint32_t rowh = drop ? row_hash(a, bh, myq) : 0u;
  float m = -INFINITY, l = 0.f;
  f4v O[4];
#pragma unroll
  for (int dn = 0; dn < 4; ++dn) O[dn] = f4v{0.f, 0.f, 0.f, 0.f};
  const int kend = MODE == 5 ? min(a.sk, q0 + kQB) : a.sk;
  const int nb = (kend + kKB - 1) / kKB;

  RowRegs rk, rv;
  MaskRegs rm;
  rows_load<T>(rk, K, a.k_st, min(kKB, a.sk), tid);
  rows_load<T>(rv, V, a.v_st, min(kKB, a.sk), tid);
  mask_load<MODE>(rm, a, b, q0, 0, tid);
  rows_store(smem, rk, tid);
  rows_store(smem + kKB * 128, rv, tid);
  mask_store<MODE>(smem + 2 * kKB * 128, rm, a, tid);
  __syncthreads();
  for (int ib = 0; ib < nb; ++ib) {
    const int kb = ib * kKB;
    char* kimg = smem + (ib & 1) * kBuf;
    char* vimg = kimg + kKB * 128;
    const char* mimg = vimg + kKB * 128;
    if (ib + 1 < nb) {
      const int kn = kb + kKB;
      rows_load<T>(rk, K + (int64_t)kn * a.k_st, a.k_st, min(kKB, a.sk - kn), tid);
      rows_load<T>(rv, V + (int64_t)kn * a.v_st, a.v_st, min(kKB, a.sk - kn), tid);
      mask_load<MODE>(rm, a, b, q0, kn, tid);
    }
    f4v S[4];  // S^T: row = key 16mt + 4fq + j, column = this lane's query
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      S[mt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) S[mt] = Mfma<T>::run(frag_row(kimg, 128, 16 * mt, 32 * s, lane), qb[s], S[mt]);
    }
    float mb = -INFINITY;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bool mk;
        const int kl = 16 * mt + 4 * fq + j;
        S[mt][j] = mask_apply<MODE>(S[mt][j] * a.scale, a, mimg, myq - q0, kl, myq, kb + kl, mk);
        mb = fmaxf(mb, S[mt][j]);
      }
    mb = fmaxf(mb, __shfl_xor(mb, 16));
    mb = fmaxf(mb, __shfl_xor(mb, 32));
    const float mn = fmaxf(m, mb);
    const float corr = (m == -INFINITY) ? 0.f : __expf(m - mn);
    m = mn;
    float ls = 0.f;
    const float mref = m == -INFINITY ? 0.f : m;  // all scores -inf then: exp -> 0
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      bool kp[4] = {true, true, true, true};
      if (drop) {
        keep_pair(rowh, kb + 16 * mt + 4 * fq, thresh, kp[0], kp[1]);
        keep_pair(rowh, kb + 16 * mt + 4 * fq + 2, thresh, kp[2], kp[3]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __expf(S[mt][j] - mref);
        ls += p;
        S[mt][j] = kp[j] ? p : 0.f;
      }
    }
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    l = l * corr + ls;
#pragma unroll
    for (int dn = 0; dn < 4; ++dn) O[dn] *= corr;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const i4v pb = pack_pair<T>(S[2 * t], S[2 * t + 1]);
#pragma unroll
      for (int dn = 0; dn < 4; ++dn) O[dn] = Mfma<T>::run(frag_tr_perm(vimg, 128, 32 * t, 16 * dn, lane), pb, O[dn]);
    }
    if (ib + 1 < nb) {
      char* nk = smem + ((ib + 1) & 1) * kBuf;
      rows_store(nk, rk, tid);
      rows_store(nk + kKB * 128, rv, tid);
      mask_store<MODE>(nk + 2 * kKB * 128, rm, a, tid);
    }
    __syncthreads();
  }
  if (myq < a.sq) {
    const float inv = l > 0.f ? (drop ? kscale : 1.f) / l : 0.f;
    T* out = reinterpret_cast<T*>(a.o) + (int64_t)bh * a.o_sbh + (int64_t)myq * a.o_st;
#pragma unroll
    for (int dn = 0; dn < 4; ++dn) store4<T>(out + 16 * dn + 4 * fq, O[dn], inv);
    if (fq == 0) a.lse[(int64_t)bh * a.sq + myq] = l > 0.f ? m + __logf(l) : INFINITY;
  }
}

// =============================================================================================
// Flash forward, 32x32x16 form (mask modes 0 / 5: the GPT / BERT-without-padding shapes).
// Workgroup = 4 waves x 32 query rows. Each wave computes S^T = K.Q^T of a 64-key block as two
// 32x32 tiles (key on the register index, query on the lane): every K fragment read from LDS now
// feeds 32 queries, half the LDS bytes per FLOP of the 16x16x32 kernel above, which ran LDS-bound.
// Softmax runs in base 2 with the scale folded into one fma per score, the running max is raised
// only when some row's block max exceeds it by more than 2^8 (a wave-uniform vote; P <= 256 is
// exact enough in bf16 / f16 since the relative rounding is scale-free) and the row sum is kept
// per half-wave until the epilogue. P^T feeds O^T = V^T.P^T straight from the accumulators; V^T
// comes from the row-major V image through ds_read_b64_tr_b16. Causal: blocks past a wave's last
// query are skipped, only blocks crossing the diagonal are masked, tiles are issued heaviest first.
// =============================================================================================
typedef float f16v __attribute__((ext_vector_type(16)));

template <typename T> struct Mfma32;
template <> struct Mfma32<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0,
                                                   0);
  }
};

constexpr int kFQ = 128;  // query rows per workgroup of the 32x32 kernels

// 128-B-row image: chunk ^= ((row>>1)&1)<<2 | ((row>>2)&3). Conflict-free for the 32-row
// ds_read_b128 row reads (every 16-lane group hits 16 distinct 16-B slots) and for the 4-row
// ds_read_b64_tr_b16 column reads (rows r, r+2 of a 4-row block land in disjoint chunk halves).
BH_DEVICE int sw_off(int row, int ch) { return row * 128 + ((ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4); }

BH_DEVICE void rows_store_sw(char* img, const RowRegs& r, int tid) {
  if (r.valid >= 64) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * kThreads;
      *reinterpret_cast<i4v*>(img + sw_off(idx >> 3, idx & 7)) = r.v[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * kThreads;
      *reinterpret_cast<i4v*>(img + sw_off(idx >> 3, idx & 7)) = rows_val(r, i, tid);
    }
  }
}
// per-thread stream over 64-row blocks of one head operand: the row offsets are computed once, a
// block costs one scalar multiply (kn * st) plus the two loads; only a partial tail block clamps.
template <typename T> struct RowStream {
  const T* base;
  int64_t st;
  int64_t off[2];
  BH_DEVICE RowStream(const T* b, int64_t s, int tid) : base(b), st(s) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * kThreads;
      off[i] = (int64_t)(idx >> 3) * s + (idx & 7) * 8;
    }
  }
  BH_DEVICE void load(RowRegs& r, int kn, int n, int tid) const {
    const int valid = min(kKB, n - kn);
    if (valid >= kKB) {
      r.valid = kKB;
      const T* src = base + (int64_t)kn * st;
#pragma unroll
      for (int i = 0; i < 2; ++i) r.v[i] = *reinterpret_cast<const i4v*>(src + off[i]);
    } else {
      rows_load<T>(r, base + (int64_t)kn * st, st, valid, tid);
    }
  }
};

// 32x32x16 A operand = rows 32t.. of the image, k = columns 16s.. (lane: row r32, 8 columns at 8h)
BH_DEVICE i4v frag32_row(const char* img, int r0, int s, int lane) {
  return *reinterpret_cast<const i4v*>(img + sw_off(r0 + (lane & 31), 2 * s + (lane >> 5)));
}
// 32x32x16 A operand V^T[dims 32dn.., keys] whose k order matches an accumulator tile's register
// order: element j of half h <-> image row k0 + 4h + (j&3) + 8(j>>2); two transposed reads.
BH_DEVICE i4v frag32_tr(const char* img, int k0, int dn, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = k0 + 4 * (lane >> 5) + q, col = 32 * dn + 16 * (g & 1) + 4 * p;
  const int cb = (col & 7) << 1;
  const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + sw_off(row, col >> 3) + cb));
  const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + sw_off(row + 8, col >> 3) + cb));
  typedef int bh_i2v __attribute__((ext_vector_type(2)));
  const bh_i2v l = __builtin_bit_cast(bh_i2v, lo), hh = __builtin_bit_cast(bh_i2v, hi);
  return i4v{l[0], l[1], hh[0], hh[1]};
}
// registers 8u..8u+7 of an accumulator tile as a 16-bit operand (k = those 8 rows)
template <typename T> BH_DEVICE i4v pack8(const f16v& x, int u) {
  T v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = from_f<T>(x[8 * u + j]);
  return *reinterpret_cast<const i4v*>(v);
}
// max / sum of a value over the two half-waves (lanes l and l ^ 32): one v_permlane32_swap
BH_DEVICE float half_pair(float x, bool sum) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x),
                                                  false, false);
  const float a = __builtin_bit_cast(float, (unsigned)r[0]), b = __builtin_bit_cast(float, (unsigned)r[1]);
  return sum ? a + b : fmaxf(a, b);
}

// mode-4 mask words of a 32x32 tile (AttnArgs::mbits / mbits_t): word t covers rows 32t.. of the
// 64-row block at r0; shifted right by 4h so that register i tests bit (i&3) + 8(i>>2)
BH_DEVICE void mask_words(uint32_t (&w)[2], const uint32_t* row, int r0, int n, int h) {
#pragma unroll
  for (int t = 0; t < 2; ++t) w[t] = r0 + 32 * t < n ? row[(r0 >> 5) + t] >> (4 * h) : 0u;
}
BH_DEVICE bool reg_bit(uint32_t w, int i) { return (w >> ((i & 3) + 8 * (i >> 2))) & 1u; }

// attn.hip is built with -fno-honor-nans (no canonicalising v_max in front of every fmaxf of an
// MFMA result: the max trees below become pure v_max3_f32) and -fno-slp-vectorize (adjacent f32
// adds are not packed into v_pk_add_f32, which co-issues badly beside MFMAs); see _build.py.
BH_DEVICE float vmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
BH_DEVICE float vadd(float a, float b) { return a + b; }
// max of the 32 scores of a lane: 16 v_max3_f32, depth 4
BH_DEVICE float tree_max(const f16v (&S)[2]) {
  float r[5];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    r[2 * t] = vmax3(vmax3(S[t][0], S[t][1], S[t][2]), vmax3(S[t][3], S[t][4], S[t][5]),
                     vmax3(S[t][6], S[t][7], S[t][8]));
    r[2 * t + 1] = vmax3(vmax3(S[t][9], S[t][10], S[t][11]), vmax3(S[t][12], S[t][13], S[t][14]), S[t][15]);
  }
  return vmax3(vmax3(r[0], r[1], r[2]), r[3], r[3]);
}

// 3 waves per SIMD (<= 168 VGPRs): only the first half of the V^T fragments is read ahead of the
// softmax, the second half after it (measured: 1.13-1.19x over reading all of them ahead at 2 waves)
template <typename T, int MODE, bool DROP>
__global__ __launch_bounds__(kThreads, 3) void k_flash_fwd32(AttnArgs a) {
  constexpr int kImg = kKB * 128;
  __shared__ __attribute__((aligned(16))) char smem[4 * kImg];  // {K, V} x 2 buffers
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  int qtile, bh;
  flash_tile(qtile, bh);
  if (MODE == 5) qtile = gridDim.x - 1 - qtile;  // longest causal prefix first
  if (a.cu_seqlens && !varlen_rebase<T>(a, bh, qtile * kFQ)) return;
  const int q0w = qtile * kFQ + wave * 32;
  const int myq = q0w + r32;

  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  i4v qf[4];  // B operand of S^T = K.Q^T: Q[myq][16s + 8h + 0..7]
  {
    const int qr = min(myq, a.sq - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const i4v*>(Q + (int64_t)qr * a.q_st + 16 * s + 8 * h);
  }
  const float c = a.scale * 1.4426950408889634f;  // scores -> base-2 exponents
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  const uint32_t rowh = DROP ? row_hash(a, bh, myq) : 0u;
  // mode 4: this query's key bits; a masked raw score becomes mask_fill / scale (= mask_fill scaled)
  const uint32_t* mrow = MODE == 4 ? a.mbits + ((int64_t)(bh / a.heads) * a.sq + min(myq, a.sq - 1)) * ((a.sk + 31) >> 5)
                                   : nullptr;
  const float fillraw = a.mask_fill / a.scale;
  float m = -INFINITY, l = 0.f;  // running base-2 max (shared by both halves), this half's sum
  f16v O[2];                      // O^T: dims 32dn + (i&3) + 8(i>>2) + 4h, query myq
#pragma unroll
  for (int dn = 0; dn < 2; ++dn)
#pragma unroll
    for (int i = 0; i < 16; ++i) O[dn][i] = 0.f;
  const int q_last = min(q0w + 31, a.sq - 1);
  const int kend = MODE == 5 ? min(a.sk, min(qtile * kFQ + kFQ, a.sq)) : a.sk;
  const int nb = (kend + kKB - 1) / kKB;

  RowRegs rk, rv;
  const RowStream<T> ks(K, a.k_st, tid), vs(V, a.v_st, tid);
  ks.load(rk, 0, a.sk, tid);
  vs.load(rv, 0, a.sk, tid);
  rows_store_sw(smem, rk, tid);
  rows_store_sw(smem + kImg, rv, tid);
  __syncthreads();
  for (int ib = 0; ib < nb; ++ib) {
    const int kb = ib * kKB;
    const char* kimg = smem + (ib & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    if (ib + 1 < nb) {
      ks.load(rk, kb + kKB, a.sk, tid);
      vs.load(rv, kb + kKB, a.sk, tid);
    }
    if (MODE != 5 || kb <= q_last) {  // wave-uniform: a causal block past every query of the wave is skipped
      uint32_t mw[2] = {0u, 0u};
      if (MODE == 4) mask_words(mw, mrow, kb, a.sk, h);
      // all LDS reads of the block up front (K row fragments, then V^T fragments): the MFMAs then
      // wait on the first reads only and the V reads land under QK^T and the softmax
      i4v kf[2][4], vf[2][2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) kf[t][s] = frag32_row(kimg, 32 * t, s, lane);
#pragma unroll
      for (int t = 0; t < 1; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int dn = 0; dn < 2; ++dn) vf[t][u][dn] = frag32_tr(vimg, 32 * t + 16 * u, dn, lane);
      f16v S[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) S[t][i] = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) S[t] = Mfma32<T>::run(kf[t][s], qf[s], S[t]);
      }
      // masks as one compare of the register's key offset against a per-lane limit
      if (kb + kKB > a.sk) {
        const int lim = a.sk - kb - 4 * h;  // key offset (32t + (i&3) + 8(i>>2)) must stay below
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) >= lim) S[t][i] = -INFINITY;
      }
      if (MODE == 5 && kb + kKB - 1 > q0w) {
        const int lim = myq - kb - 4 * h;  // masked: key offset > lim
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) > lim) S[t][i] = -INFINITY;
      }
      if (MODE == 4 && __any((mw[0] | mw[1]) != 0u)) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (reg_bit(mw[t], i)) S[t][i] = fillraw;
      }
      const float mx = half_pair(tree_max(S), false) * c;
      if (__any(mx > m + 8.f)) {
        const float mn = fmaxf(m, mx);
        const float corr = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
#pragma unroll
        for (int dn = 0; dn < 2; ++dn)
#pragma unroll
          for (int i = 0; i < 16; ++i) O[dn][i] *= corr;
        m = mn;
      }
      const float nm = m == -INFINITY ? 0.f : -m;
      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(S[t][i], c, nm));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(S[t][i + 1], c, nm));
          const int ch = (i >> 1) & 3;
          ls[ch] = (t == 0 && i < 8) ? vadd(p0, p1) : vadd(vadd(ls[ch], p0), p1);
          if (DROP) {
            bool k0, k1;
            keep_pair(rowh, kb + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h, thresh, k0, k1);
            S[t][i] = k0 ? p0 : 0.f;
            S[t][i + 1] = k1 ? p1 : 0.f;
          } else {
            S[t][i] = p0;
            S[t][i + 1] = p1;
          }
        }
      l = vadd(l, vadd(vadd(ls[0], ls[1]), vadd(ls[2], ls[3])));
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int dn = 0; dn < 2; ++dn) vf[1][u][dn] = frag32_tr(vimg, 32 + 16 * u, dn, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const i4v pb = pack8<T>(S[t], u);
#pragma unroll
          for (int dn = 0; dn < 2; ++dn) O[dn] = Mfma32<T>::run(vf[t][u][dn], pb, O[dn]);
        }
    }
    if (ib + 1 < nb) {
      char* nk = smem + ((ib + 1) & 1) * 2 * kImg;
      rows_store_sw(nk, rk, tid);
      rows_store_sw(nk + kImg, rv, tid);
    }
    __syncthreads();
  }
  l = half_pair(l, true);
  if (myq < a.sq) {
    const float inv = l > 0.f ? (DROP ? kscale : 1.f) / l : 0.f;
    T* out = reinterpret_cast<T*>(a.o) + (int64_t)bh * a.o_sbh + (int64_t)myq * a.o_st;
#pragma unroll
    for (int dn = 0; dn < 2; ++dn)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f4v v4 = f4v{O[dn][4 * gq], O[dn][4 * gq + 1], O[dn][4 * gq + 2], O[dn][4 * gq + 3]};
        store4<T>(out + 32 * dn + 8 * gq + 4 * h, v4, inv);
      }
    if (h == 0) a.lse[(int64_t)bh * a.sq + myq] = l > 0.f ? (m + __log2f(l)) * 0.6931471805599453f : INFINITY;
  }
}

// dQ, 32x32x16 form (mask modes 0 / 4 / 5). Same layout as k_flash_fwd32 (query on the lane): S^T =
// K.Q^T and dP^T = V.dO^T from K / V row fragments, P^T rebuilt from the saved LSE in base 2,
// dS^T = P^T (dP^T - delta) stays in registers and feeds dQ^T = K^T.dS^T (K^T by transposed reads
// of the same K image); the softmax scale is applied once to dQ in the epilogue.
template <typename T, int MODE, bool DROP>
__global__ __launch_bounds__(kThreads, 2) void k_flash_dq32(AttnArgs a) {
  constexpr int kImg = kKB * 128;
  __shared__ __attribute__((aligned(16))) char smem[4 * kImg];  // {K, V} x 2 buffers
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  int qtile, bh;
  flash_tile(qtile, bh);
  if (MODE == 5) qtile = gridDim.x - 1 - qtile;
  if (a.cu_seqlens && !varlen_rebase<T>(a, bh, qtile * kFQ)) return;
  const int q0w = qtile * kFQ + wave * 32;
  const int myq = q0w + r32;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)bh * a.do_sbh;
  const int qr = min(myq, a.sq - 1);
  i4v qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const i4v*>(Q + (int64_t)qr * a.q_st + 16 * s + 8 * h);
    df[s] = *reinterpret_cast<const i4v*>(dO + (int64_t)qr * a.do_st + 16 * s + 8 * h);
  }
  const float c = a.scale * 1.4426950408889634f;
  const float lse = a.lse[(int64_t)bh * a.sq + qr];
  const float dl = a.delta[(int64_t)bh * a.sq + qr];
  const float nl = (myq < a.sq && lse != INFINITY) ? -lse * 1.4426950408889634f : -INFINITY;  // p = 2^(c*s + nl)
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  const uint32_t rowh = DROP ? row_hash(a, bh, myq) : 0u;
  // mode 4: a masked score's gradient is zero (masked_fill), so its P is dropped to 0 here
  const uint32_t* mrow = MODE == 4 ? a.mbits + ((int64_t)(bh / a.heads) * a.sq + qr) * ((a.sk + 31) >> 5) : nullptr;
  f16v acc[2];
#pragma unroll
  for (int dn = 0; dn < 2; ++dn)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dn][i] = 0.f;
  const int q_last = min(q0w + 31, a.sq - 1);
  const int kend = MODE == 5 ? min(a.sk, min(qtile * kFQ + kFQ, a.sq)) : a.sk;
  const int nb = (kend + kKB - 1) / kKB;
  RowRegs rk, rv;
  const RowStream<T> ks(K, a.k_st, tid), vs(V, a.v_st, tid);
  ks.load(rk, 0, a.sk, tid);
  vs.load(rv, 0, a.sk, tid);
  rows_store_sw(smem, rk, tid);
  rows_store_sw(smem + kImg, rv, tid);
  __syncthreads();
  for (int ib = 0; ib < nb; ++ib) {
    const int kb = ib * kKB;
    const char* kimg = smem + (ib & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    if (ib + 1 < nb) {
      ks.load(rk, kb + kKB, a.sk, tid);
      vs.load(rv, kb + kKB, a.sk, tid);
    }
    if (MODE != 5 || kb <= q_last) {
      uint32_t mw[2] = {0u, 0u};
      if (MODE == 4) mask_words(mw, mrow, kb, a.sk, h);
      f16v S[2], P[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        i4v kf[4], vf[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          kf[s] = frag32_row(kimg, 32 * t, s, lane);
          vf[s] = frag32_row(vimg, 32 * t, s, lane);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) S[t][i] = P[t][i] = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          S[t] = Mfma32<T>::run(kf[s], qf[s], S[t]);
          P[t] = Mfma32<T>::run(vf[s], df[s], P[t]);  // dP^T
        }
      }
      if (kb + kKB > a.sk) {
        const int lim = a.sk - kb - 4 * h;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) >= lim) S[t][i] = -INFINITY;
      }
      if (MODE == 5 && kb + kKB - 1 > q0w) {
        const int lim = myq - kb - 4 * h;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) > lim) S[t][i] = -INFINITY;
      }
      if (MODE == 4 && __any((mw[0] | mw[1]) != 0u)) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (reg_bit(mw[t], i)) S[t][i] = -INFINITY;
      }
      // dS'^T = P^T (dP^T_dropped - delta), into P (scale applied in the epilogue)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(S[t][i], c, nl));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(S[t][i + 1], c, nl));
          if (DROP) {
            bool k0, k1;
            keep_pair(rowh, kb + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h, thresh, k0, k1);
            P[t][i] = p0 * ((k0 ? P[t][i] * kscale : 0.f) - dl);
            P[t][i + 1] = p1 * ((k1 ? P[t][i + 1] * kscale : 0.f) - dl);
          } else {
            P[t][i] = p0 * (P[t][i] - dl);
            P[t][i + 1] = p1 * (P[t][i + 1] - dl);
          }
        }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const i4v sb = pack8<T>(P[t], u);
#pragma unroll
          for (int dn = 0; dn < 2; ++dn)
            acc[dn] = Mfma32<T>::run(frag32_tr(kimg, 32 * t + 16 * u, dn, lane), sb, acc[dn]);
        }
    }
    if (ib + 1 < nb) {
      char* nk = smem + ((ib + 1) & 1) * 2 * kImg;
      rows_store_sw(nk, rk, tid);
      rows_store_sw(nk + kImg, rv, tid);
    }
    __syncthreads();
  }
  if (myq < a.sq) {
    T* dq = reinterpret_cast<T*>(a.dq) + (int64_t)bh * a.dq_sbh + (int64_t)myq * a.dq_st;
#pragma unroll
    for (int dn = 0; dn < 2; ++dn)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f4v v4 = f4v{acc[dn][4 * gq], acc[dn][4 * gq + 1], acc[dn][4 * gq + 2], acc[dn][4 * gq + 3]};
        store4<T>(dq + 32 * dn + 8 * gq + 4 * h, v4, a.scale);
      }
  }
}

// dK / dV, 32x32x16 form (mask modes 0 / 4 / 5). Workgroup = 4 waves x 32 keys, key on the lane: S =
// Q.K^T and dP = dO.V^T per 32-query tile (A = Q / dO row fragments from LDS, B = K / V fragments
// held in registers), P from the per-query base-2 LSE row constants, and P_dropped / dS feed dV^T
// = dO^T.P and dK^T = Q^T.dS straight from the accumulators (dO^T, Q^T by transposed reads of the
// same images). Per 64-query block the LDS also carries the block's -LSE*log2(e), delta and (with
// dropout) row hashes, read as float4 broadcasts. Causal: key tiles start at the diagonal block and
// blocks entirely above a wave's keys are skipped; the heaviest key tiles (lowest keys) go first.
template <typename T, int MODE, bool DROP>
__global__ __launch_bounds__(kThreads, 2) void k_flash_dkdv32(AttnArgs a) {
  constexpr int kImg = kQB * 128;
  constexpr int kBuf = 2 * kImg + 3 * kQB * 4;  // Q, dO images; -lse2, delta, row hash
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  int ktile, bh;
  flash_tile(ktile, bh);
  if (a.cu_seqlens && !varlen_rebase<T>(a, bh, ktile * kFQ)) return;
  const int k0w = ktile * kFQ + wave * 32;
  const int mykey = k0w + r32;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)bh * a.do_sbh;
  i4v kf[4], vf[4];  // B operands: K[mykey][16s + 8h ..], V[mykey][16s + 8h ..]
  {
    const int kr = min(mykey, a.sk - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = *reinterpret_cast<const i4v*>(K + (int64_t)kr * a.k_st + 16 * s + 8 * h);
      vf[s] = *reinterpret_cast<const i4v*>(V + (int64_t)kr * a.v_st + 16 * s + 8 * h);
    }
  }
  const float c = a.scale * 1.4426950408889634f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  // mode 4: this key's query bits; a masked score is mask_fill (P keeps it: dV) with dS = 0
  const uint32_t* mcol = MODE == 4 ? a.mbits_t + ((int64_t)(bh / a.heads) * a.sk + min(mykey, a.sk - 1)) *
                                                     ((a.sq + 31) >> 5)
                                   : nullptr;
  const float fillraw = a.mask_fill / a.scale;
  f16v dK[2], dV[2];  // dims 32dn + (i&3) + 8(i>>2) + 4h, key mykey
#pragma unroll
  for (int dn = 0; dn < 2; ++dn)
#pragma unroll
    for (int i = 0; i < 16; ++i) dK[dn][i] = dV[dn][i] = 0.f;
  const int qstart = MODE == 5 ? (ktile * kFQ / kQB) * kQB : 0;
  const int nqb = a.sq > qstart ? (a.sq - qstart + kQB - 1) / kQB : 0;
  const int k_last = min(k0w + 31, a.sk - 1);
  const float* lseg = a.lse + (int64_t)bh * a.sq;
  const float* dlg = a.delta + (int64_t)bh * a.sq;
  RowRegs rq, rd;
  const RowStream<T> qs(Q, a.q_st, tid), ds(dO, a.do_st, tid);
  float rl = 0.f;
  auto load_blk = [&](int q0) {
    qs.load(rq, q0, a.sq, tid);
    ds.load(rd, q0, a.sq, tid);
    if (tid < 3 * kQB) {  // tid / 64: 0 -> -lse*log2(e), 1 -> delta, 2 -> row hash
      const int q = q0 + (tid & (kQB - 1)), w = tid >> 6;
      const int qc = min(q, a.sq - 1);
      if (w == 0) {
        const float l = lseg[qc];
        rl = (q < a.sq && l != INFINITY) ? -l * 1.4426950408889634f : -INFINITY;
      } else if (w == 1) {
        rl = q < a.sq ? dlg[qc] : 0.f;
      } else {
        rl = DROP ? __builtin_bit_cast(float, row_hash(a, bh, q)) : 0.f;
      }
    }
  };
  auto store_blk = [&](char* buf) {
    rows_store_sw(buf, rq, tid);
    rows_store_sw(buf + kImg, rd, tid);
    if (tid < 3 * kQB) reinterpret_cast<float*>(buf + 2 * kImg)[tid] = rl;
  };
  if (nqb > 0) {
    load_blk(qstart);
    store_blk(smem);
  }
  __syncthreads();
  for (int iq = 0; iq < nqb; ++iq) {
    const int q0 = qstart + iq * kQB;
    const char* qimg = smem + (iq & 1) * kBuf;
    const char* dimg = qimg + kImg;
    const float* nlp = reinterpret_cast<const float*>(dimg + kImg);
    const float* dlp = nlp + kQB;
    const uint32_t* rhp = reinterpret_cast<const uint32_t*>(dlp + kQB);
    if (iq + 1 < nqb) load_blk(q0 + kQB);
    if (MODE != 5 || q0 + kQB - 1 >= k0w) {  // wave-uniform: some query of the block sees a key of the wave
      uint32_t mw[2] = {0u, 0u};
      if (MODE == 4) mask_words(mw, mcol, q0, a.sq, h);
      f16v S[2], P[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        i4v qa[4], da[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          qa[s] = frag32_row(qimg, 32 * t, s, lane);
          da[s] = frag32_row(dimg, 32 * t, s, lane);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) S[t][i] = P[t][i] = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          S[t] = Mfma32<T>::run(qa[s], kf[s], S[t]);
          P[t] = Mfma32<T>::run(da[s], vf[s], P[t]);  // dP
        }
      }
      if (MODE == 5 && q0 < k0w + 31) {  // diagonal: masked where key > query
        const int lim = mykey - q0 - 4 * h;  // masked: query offset (32t + (i&3) + 8(i>>2)) < lim
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) < lim) S[t][i] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ql = 32 * t + 8 * g + 4 * h;  // queries ql .. ql+3 in registers 4g .. 4g+3
          const f4v n4 = *reinterpret_cast<const f4v*>(nlp + ql);
          const f4v d4 = *reinterpret_cast<const f4v*>(dlp + ql);
          i4v r4 = i4v{0, 0, 0, 0};
          if (DROP) r4 = *reinterpret_cast<const i4v*>(rhp + ql);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * g + j;
            const bool mk = MODE == 4 && reg_bit(mw[t], i);  // mode 4: score mask_fill, dS 0
            const float p = __builtin_amdgcn_exp2f(fmaf(mk ? fillraw : S[t][i], c, n4[j]));
            if (DROP) {
              const bool kp = keep_elem((uint32_t)r4[j], mykey, thresh);
              const float kk = kp ? kscale : 0.f;
              S[t][i] = p * kk;                                // P dropped
              P[t][i] = mk ? 0.f : p * (P[t][i] * kk - d4[j]);  // dS'
            } else {
              S[t][i] = p;
              P[t][i] = mk ? 0.f : p * (P[t][i] - d4[j]);
            }
          }
        }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const i4v pb = pack8<T>(S[t], u);
          const i4v sb = pack8<T>(P[t], u);
#pragma unroll
          for (int dn = 0; dn < 2; ++dn) {
            dV[dn] = Mfma32<T>::run(frag32_tr(dimg, 32 * t + 16 * u, dn, lane), pb, dV[dn]);
            dK[dn] = Mfma32<T>::run(frag32_tr(qimg, 32 * t + 16 * u, dn, lane), sb, dK[dn]);
          }
        }
    }
    if (iq + 1 < nqb) store_blk(smem + ((iq + 1) & 1) * kBuf);
    __syncthreads();
  }
  (void)k_last;
  if (mykey < a.sk) {
    T* dk = reinterpret_cast<T*>(a.dk) + (int64_t)bh * a.dk_sbh + (int64_t)mykey * a.dk_st;
    T* dv = reinterpret_cast<T*>(a.dv) + (int64_t)bh * a.dv_sbh + (int64_t)mykey * a.dv_st;
#pragma unroll
    for (int dn = 0; dn < 2; ++dn)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f4v k4 = f4v{dK[dn][4 * gq], dK[dn][4 * gq + 1], dK[dn][4 * gq + 2], dK[dn][4 * gq + 3]};
        const f4v v4 = f4v{dV[dn][4 * gq], dV[dn][4 * gq + 1], dV[dn][4 * gq + 2], dV[dn][4 * gq + 3]};
        store4<T>(dk + 32 * dn + 8 * gq + 4 * h, k4, a.scale);
        store4<T>(dv + 32 * dn + 8 * gq + 4 * h, v4, 1.f);
      }
  }
}

// delta[bh, q] = sum_d dO[q, bh, d] * O[q, bh, d]; one 16-lane group per row
template <typename T>
__global__ __launch_bounds__(256) void k_flash_delta(AttnArgs a, float* __restrict__ delta) {
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 16;  // row = bh * sq + q
  const int sub = threadIdx.x & 15;
  if (row >= (int64_t)a.BH * a.sq) return;
  const int bh = (int)(row / a.sq), q = (int)(row % a.sq);
  if (a.cu_seqlens && !varlen_rebase<T>(a, bh, q)) {  // a padding row of a shorter sequence
    if (sub == 0) delta[row] = 0.f;
    return;
  }
  const T* o = reinterpret_cast<const T*>(a.o) + (int64_t)q * a.o_st + (int64_t)bh * a.o_sbh + sub * 4;
  const T* d = reinterpret_cast<const T*>(a.dout) + (int64_t)q * a.do_st + (int64_t)bh * a.do_sbh + sub * 4;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc += to_f<T>(o[i]) * to_f<T>(d[i]);
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) acc += __shfl_xor(acc, off);
  if (sub == 0) delta[row] = acc;
}

// dQ. Same layout as the forward (query on the lane): S^T = K.Q^T and dP^T = V.dO^T, P^T from
// the saved LSE, dS^T in registers feeds dQ^T = K^T.dS^T directly.
template <typename T, int MODE>
__global__ __launch_bounds__(kThreads) void k_flash_bwd_dq(AttnArgs a) {
  constexpr int kBuf = 2 * kKB * 128 + kMaskBytes;
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  int qtile, bh;
  flash_tile(qtile, bh);
  const int b = bh / a.heads;
  const int q0 = qtile * kQB;
  const int myq = q0 + wave * 16 + fr;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)bh * a.do_sbh;
  i4v qb[2], db[2];
  const int qr = min(myq, a.sq - 1);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    qb[s] = *reinterpret_cast<const i4v*>(Q + (int64_t)qr * a.q_st + 32 * s + 8 * fq);
    db[s] = *reinterpret_cast<const i4v*>(dO + (int64_t)qr * a.do_st + 32 * s + 8 * fq);
  }
  const float lse = a.lse[(int64_t)bh * a.sq + qr];
  const float dl = a.delta[(int64_t)bh * a.sq + qr];
  const bool rowok = myq < a.sq && lse != INFINITY;
  const bool drop = a.training && a.p_drop > 0.f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  const uint32_t rowh = drop ? row_hash(a, bh, myq) : 0u;
  f4v acc[4];
#pragma unroll
  for (int dn = 0; dn < 4; ++dn) acc[dn] = f4v{0.f, 0.f, 0.f, 0.f};
  const int kend = MODE == 5 ? min(a.sk, q0 + kQB) : a.sk;
  const int nb = (kend + kKB - 1) / kKB;
  RowRegs rk, rv;
  MaskRegs rm;
  rows_load<T>(rk, K, a.k_st, min(kKB, a.sk), tid);
  rows_load<T>(rv, V, a.v_st, min(kKB, a.sk), tid);
  mask_load<MODE>(rm, a, b, q0, 0, tid);
  rows_store(smem, rk, tid);
  rows_store(smem + kKB * 128, rv, tid);
  mask_store<MODE>(smem + 2 * kKB * 128, rm, a, tid);
  __syncthreads();
  for (int ib = 0; ib < nb; ++ib) {
    const int kb = ib * kKB;
    char* kimg = smem + (ib & 1) * kBuf;
    char* vimg = kimg + kKB * 128;
    const char* mimg = vimg + kKB * 128;
    if (ib + 1 < nb) {
      const int kn = kb + kKB;
      rows_load<T>(rk, K + (int64_t)kn * a.k_st, a.k_st, min(kKB, a.sk - kn), tid);
      rows_load<T>(rv, V + (int64_t)kn * a.v_st, a.v_st, min(kKB, a.sk - kn), tid);
      mask_load<MODE>(rm, a, b, q0, kn, tid);
    }
    f4v dS[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f4v S = f4v{0.f, 0.f, 0.f, 0.f}, dP = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        S = Mfma<T>::run(frag_row(kimg, 128, 16 * mt, 32 * s, lane), qb[s], S);
        dP = Mfma<T>::run(frag_row(vimg, 128, 16 * mt, 32 * s, lane), db[s], dP);
      }
      bool kp[4] = {true, true, true, true};
      if (drop) {
        keep_pair(rowh, kb + 16 * mt + 4 * fq, thresh, kp[0], kp[1]);
        keep_pair(rowh, kb + 16 * mt + 4 * fq + 2, thresh, kp[2], kp[3]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kl = 16 * mt + 4 * fq + j;
        bool mk;
        const float v = mask_apply<MODE>(S[j] * a.scale, a, mimg, myq - q0, kl, myq, kb + kl, mk);
        const float p = (rowok && v != -INFINITY) ? __expf(v - lse) : 0.f;
        const float dpd = drop ? (kp[j] ? dP[j] * kscale : 0.f) : dP[j];
        dS[mt][j] = mk ? 0.f : p * (dpd - dl) * a.scale;
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const i4v sb = pack_pair<T>(dS[2 * t], dS[2 * t + 1]);
#pragma unroll
      for (int dn = 0; dn < 4; ++dn)
        acc[dn] = Mfma<T>::run(frag_tr_perm(kimg, 128, 32 * t, 16 * dn, lane), sb, acc[dn]);
    }
    if (ib + 1 < nb) {
      char* nk = smem + ((ib + 1) & 1) * kBuf;
      rows_store(nk, rk, tid);
      rows_store(nk + kKB * 128, rv, tid);
      mask_store<MODE>(nk + 2 * kKB * 128, rm, a, tid);
    }
    __syncthreads();
  }
  if (myq < a.sq) {
    T* dq = reinterpret_cast<T*>(a.dq) + (int64_t)bh * a.dq_sbh + (int64_t)myq * a.dq_st;
#pragma unroll
    for (int dn = 0; dn < 4; ++dn) store4<T>(dq + 16 * dn + 4 * fq, acc[dn], 1.f);
  }
}

// dK / dV. Workgroup = 64 keys x one head, wave w owns keys 16w..16w+15 with the KEY on the lane:
// S = Q.K^T and dP = dO.V^T per 16-query tile put 4 queries of one key in a lane's registers, so
// Pd and dS feed dV^T = dO^T.Pd and dK^T = Q^T.dS as B operands straight from registers (no
// cross-wave reduction, no LDS round trip). Q / dO / LSE / delta / mask blocks are double-buffered.
// 3 waves per SIMD (<= 168 VGPRs): the LDS footprint (2 x 20.5 KiB) already caps the kernel at
// 3 workgroups per CU, so registers beyond that only cost occupancy
template <typename T, int MODE>
__global__ __launch_bounds__(kThreads, 3) void k_flash_bwd_dkdv(AttnArgs a) {
  constexpr int kBuf = 2 * kQB * 128 + kMaskBytes + 2 * kQB * 4;  // Q, dO, mask, LSE, delta
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  int ktile, bh;
  flash_tile(ktile, bh);
  const int b = bh / a.heads;
  const int kb = ktile * kKB;
  const int mykey = kb + wave * 16 + fr;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)bh * a.k_sbh;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)bh * a.v_sbh;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)bh * a.q_sbh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)bh * a.do_sbh;
  i4v kbf[2], vbf[2];
  {
    const int kr = min(mykey, a.sk - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      kbf[s] = *reinterpret_cast<const i4v*>(K + (int64_t)kr * a.k_st + 32 * s + 8 * fq);
      vbf[s] = *reinterpret_cast<const i4v*>(V + (int64_t)kr * a.v_st + 32 * s + 8 * fq);
    }
  }
  const bool drop = a.training && a.p_drop > 0.f;
  const float kscale = a.p_drop < 1.f ? 1.f / (1.f - a.p_drop) : 0.f;
  const uint32_t thresh = keep_thresh(a.p_drop);
  f4v dK[4], dV[4];
#pragma unroll
  for (int dn = 0; dn < 4; ++dn) dK[dn] = dV[dn] = f4v{0.f, 0.f, 0.f, 0.f};
  const int qstart = MODE == 5 ? (kb / kQB) * kQB : 0;
  const int nqb = (a.sq - qstart + kQB - 1) / kQB;
  const float* lseg = a.lse + (int64_t)bh * a.sq;
  const float* dlg = a.delta + (int64_t)bh * a.sq;
  RowRegs rq, rd;
  MaskRegs rm;
  float rl = 0.f;
  auto load_blk = [&](int qs) {
    rows_load<T>(rq, Q + (int64_t)qs * a.q_st, a.q_st, min(kQB, a.sq - qs), tid);
    rows_load<T>(rd, dO + (int64_t)qs * a.do_st, a.do_st, min(kQB, a.sq - qs), tid);
    mask_load<MODE>(rm, a, b, qs, kb, tid);
    if (tid < 2 * kQB) {
      const int q = min(qs + (tid & (kQB - 1)), a.sq - 1);
      const float v = tid < kQB ? lseg[q] : dlg[q];
      rl = qs + (tid & (kQB - 1)) < a.sq ? v : (tid < kQB ? INFINITY : 0.f);  // p = 0 there; keep dS finite
    }
  };
  auto store_blk = [&](char* buf) {
    rows_store(buf, rq, tid);
    rows_store(buf + kQB * 128, rd, tid);
    mask_store<MODE>(buf + 2 * kQB * 128, rm, a, tid);
    if (tid < 2 * kQB) reinterpret_cast<float*>(buf + 2 * kQB * 128 + kMaskBytes)[tid] = rl;
  };
  load_blk(qstart);
  store_blk(smem);
  __syncthreads();
  for (int iq = 0; iq < nqb; ++iq) {
    const int q0 = qstart + iq * kQB;
    char* qimg = smem + (iq & 1) * kBuf;
    char* doimg = qimg + kQB * 128;
    const char* mimg = doimg + kQB * 128;
    const float* lsel = reinterpret_cast<const float*>(mimg + kMaskBytes);
    const float* dll = lsel + kQB;
    if (iq + 1 < nqb) load_blk(q0 + kQB);
    f4v Pd[4], dS[4];  // row = query 16qt + 4fq + j of the block, column = this lane's key
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      f4v S = f4v{0.f, 0.f, 0.f, 0.f}, dP = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        S = Mfma<T>::run(frag_row(qimg, 128, 16 * qt, 32 * s, lane), kbf[s], S);
        dP = Mfma<T>::run(frag_row(doimg, 128, 16 * qt, 32 * s, lane), vbf[s], dP);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ql = 16 * qt + 4 * fq + j, q = q0 + ql;
        const float lse = lsel[ql], dl = dll[ql];
        bool mk;
        const float v = mask_apply<MODE>(S[j] * a.scale, a, mimg, ql, wave * 16 + fr, q, mykey, mk);
        const float p = (q < a.sq && v != -INFINITY && lse != INFINITY) ? __expf(v - lse) : 0.f;
        const float kk = drop ? (keep_elem(row_hash(a, bh, q), mykey, thresh) ? kscale : 0.f) : 1.f;
        Pd[qt][j] = p * kk;
        dS[qt][j] = mk ? 0.f : p * (dP[j] * kk - dl) * a.scale;
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const i4v pb = pack_pair<T>(Pd[2 * t], Pd[2 * t + 1]);
      const i4v sb = pack_pair<T>(dS[2 * t], dS[2 * t + 1]);
#pragma unroll
      for (int dn = 0; dn < 4; ++dn) {
        dV[dn] = Mfma<T>::run(frag_tr_perm(doimg, 128, 32 * t, 16 * dn, lane), pb, dV[dn]);
        dK[dn] = Mfma<T>::run(frag_tr_perm(qimg, 128, 32 * t, 16 * dn, lane), sb, dK[dn]);
      }
    }
    if (iq + 1 < nqb) store_blk(smem + ((iq + 1) & 1) * kBuf);
    __syncthreads();
  }
  if (mykey < a.sk) {
    T* dk = reinterpret_cast<T*>(a.dk) + (int64_t)bh * a.dk_sbh + (int64_t)mykey * a.dk_st;
    T* dv = reinterpret_cast<T*>(a.dv) + (int64_t)bh * a.dv_sbh + (int64_t)mykey * a.dv_st;
#pragma unroll
    for (int dn = 0; dn < 4; ++dn) {
      store4<T>(dk + 16 * dn + 4 * fq, dK[dn], 1.f);
      store4<T>(dv + 16 * dn + 4 * fq, dV[dn], 1.f);
    }
  }
}

// (dtype, mask mode) -> compile-time kernel instance: the per-score mask logic has no runtime switch
template <typename T> struct TypeTag { using type = T; };
template <typename F> void flash_modes(int mode, const char* what, F&& f) {
  switch (mode) {
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    default: throw std::runtime_error(std::string(what) + ": unknown mask mode");
  }
}
template <typename F> void flash_dispatch(int dt, int mode, const char* what, F&& f) {
  switch (dt) {
    case kF16: flash_modes(mode, what, [&](auto mm) { f(TypeTag<f16>{}, mm); }); break;
    case kBF16: flash_modes(mode, what, [&](auto mm) { f(TypeTag<bf16>{}, mm); }); break;
    default: throw std::runtime_error(std::string(what) + ": fp16 / bf16 only");
  }
}

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// mode-4 mask bits. bits: one thread per word (row r = b*sq + q, word w), 32 bytes of the row.
__global__ __launch_bounds__(256) void k_mask_bits(const uint8_t* __restrict__ m, uint32_t* __restrict__ bits,
                                                   int64_t rows, int sk) {
  const int mw = (sk + 31) >> 5;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * mw) return;
  const int64_t r = i / mw;
  const int w = (int)(i - r * mw), n = min(32, sk - 32 * w);
  const uint8_t* p = m + r * sk + 32 * w;
  uint32_t v = 0u;
  for (int j = 0; j < n; ++j) v |= (p[j] != 0 ? 1u : 0u) << j;
  bits[i] = v;
}
// bits_t: word (b, k, w) over queries 32w..; thread order (b, w, k) so a wave reads consecutive keys
__global__ __launch_bounds__(256) void k_mask_bits_t(const uint8_t* __restrict__ m, uint32_t* __restrict__ bits_t,
                                                     int B, int sq, int sk) {
  const int mw = (sq + 31) >> 5;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * mw * sk) return;
  const int k = (int)(i % sk);
  const int64_t bw = i / sk;
  const int w = (int)(bw % mw), b = (int)(bw / mw), n = min(32, sq - 32 * w);
  const uint8_t* p = m + ((int64_t)b * sq + 32 * w) * sk + k;
  uint32_t v = 0u;
  for (int j = 0; j < n; ++j) v |= (p[(int64_t)j * sk] != 0 ? 1u : 0u) << j;
  bits_t[((int64_t)b * sk + k) * mw + w] = v;
}

}  // namespace

void flash_mask_bits(const AttnArgs& a, uint32_t* bits, uint32_t* bits_t, hipStream_t st) {
  if (a.mask_mode != 4 || !a.mask) throw std::runtime_error("flash_mask_bits: needs a mode-4 mask");
  const int B = a.BH / a.heads;
  const auto* m = reinterpret_cast<const uint8_t*>(a.mask);
  const int64_t nw = (int64_t)B * a.sq * ((a.sk + 31) >> 5);
  if (bits) hipLaunchKernelGGL(k_mask_bits, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, m, bits,
                               (int64_t)B * a.sq, a.sk);
  const int64_t nt = (int64_t)B * a.sk * ((a.sq + 31) >> 5);
  if (bits_t) hipLaunchKernelGGL(k_mask_bits_t, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, m, bits_t, B,
                                 a.sq, a.sk);
  check_launch("flash_mask_bits");
}

int attn_max_sk() { return 128; }

void attn_forward(int dt, const AttnArgs& a, hipStream_t st) {
  if (a.sk < 1 || a.sk > 128 || a.sq < 1) throw std::runtime_error("attn_forward: need 1 <= sk <= 128");
  const dim3 grid((unsigned)((a.sq + kQB - 1) / kQB), (unsigned)a.BH);
  const bool small = a.sk <= 64;
#define BH_ATTN_FWD(T)                                                                            \
  if (small) hipLaunchKernelGGL((k_attn_fwd<T, 64>), grid, dim3(kThreads), 0, st, a);              \
  else hipLaunchKernelGGL((k_attn_fwd<T, 128>), grid, dim3(kThreads), 0, st, a);
  switch (dt) {
    case kF16: BH_ATTN_FWD(f16) break;
    case kBF16: BH_ATTN_FWD(bf16) break;
    default: throw std::runtime_error("attn_forward: fp16 / bf16 only");
  }
#undef BH_ATTN_FWD
  check_launch("attn_forward");
}

void attn_backward(int dt, const AttnArgs& a, hipStream_t st) {
  if (a.sk < 1 || a.sk > 128 || a.sq < 1) throw std::runtime_error("attn_backward: need 1 <= sk <= 128");
  const dim3 grid((unsigned)a.BH);
  const bool small = a.sk <= 64;
#define BH_ATTN_BWD(T)                                                                            \
  if (small) hipLaunchKernelGGL((k_attn_bwd<T, 64>), grid, dim3(kThreads), 0, st, a);              \
  else hipLaunchKernelGGL((k_attn_bwd<T, 128>), grid, dim3(kThreads), 0, st, a);
  switch (dt) {
    case kF16: BH_ATTN_BWD(f16) break;
    case kBF16: BH_ATTN_BWD(bf16) break;
    default: throw std::runtime_error("attn_backward: fp16 / bf16 only");
  }
#undef BH_ATTN_BWD
  check_launch("attn_backward");
}

void flash_forward(int dt, const AttnArgs& a, hipStream_t st) {
  if (a.sk < 1 || a.sq < 1 || !a.lse) throw std::runtime_error("flash_forward: bad shape or missing lse");
  if (a.cu_seqlens && a.mask_mode != 0 && a.mask_mode != 5)
    throw std::runtime_error("flash_forward: varlen runs the 32x32 kernels with mask mode 0 or 5 only");
  if ((a.mask_mode == 0 || a.mask_mode == 5 || (a.mask_mode == 4 && a.mbits))) {
    const dim3 grid((unsigned)((a.sq + kFQ - 1) / kFQ), (unsigned)a.BH);
    flash_dispatch(dt, a.mask_mode, "flash_forward", [&](auto tt, auto mm) {
      using T = typename decltype(tt)::type;
      constexpr int M = decltype(mm)::value;
      if constexpr (M == 0 || M == 4 || M == 5) {
        if (a.training && a.p_drop > 0.f) hipLaunchKernelGGL((k_flash_fwd32<T, M, true>), grid, dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((k_flash_fwd32<T, M, false>), grid, dim3(kThreads), 0, st, a);
      }
    });
    check_launch("flash_forward");
    return;
  }
  const dim3 grid((unsigned)((a.sq + kQB - 1) / kQB), (unsigned)a.BH);
  flash_dispatch(dt, a.mask_mode, "flash_forward", [&](auto tt, auto mm) {
    using T = typename decltype(tt)::type;
    hipLaunchKernelGGL((k_flash_fwd<T, decltype(mm)::value>), grid, dim3(kThreads), 0, st, a);
  });
  check_launch("flash_forward");
}

void flash_delta(int dt, const AttnArgs& a, float* delta, hipStream_t st) {
  const int64_t rows = (int64_t)a.BH * a.sq;
  const dim3 grid((unsigned)((rows * 16 + 255) / 256));
  switch (dt) {
    case kF16: hipLaunchKernelGGL((k_flash_delta<f16>), grid, dim3(256), 0, st, a, delta); break;
    case kBF16: hipLaunchKernelGGL((k_flash_delta<bf16>), grid, dim3(256), 0, st, a, delta); break;
    default: throw std::runtime_error("flash_delta: fp16 / bf16 only");
  }
  check_launch("flash_delta");
}

void flash_backward(int dt, const AttnArgs& a, hipStream_t st) {
  if (a.sk < 1 || a.sq < 1 || !a.lse || !a.delta) throw std::runtime_error("flash_backward: bad args");
  if (a.cu_seqlens && a.mask_mode != 0 && a.mask_mode != 5)
    throw std::runtime_error("flash_backward: varlen runs the 32x32 kernels with mask mode 0 or 5 only");
  if ((a.mask_mode == 0 || a.mask_mode == 5 || (a.mask_mode == 4 && a.mbits && a.mbits_t))) {
    const dim3 gq((unsigned)((a.sq + kFQ - 1) / kFQ), (unsigned)a.BH);
    const dim3 gk((unsigned)((a.sk + kFQ - 1) / kFQ), (unsigned)a.BH);
    const bool dr = a.training && a.p_drop > 0.f;
    flash_dispatch(dt, a.mask_mode, "flash_backward", [&](auto tt, auto mm) {
      using T = typename decltype(tt)::type;
      constexpr int M = decltype(mm)::value;
      if constexpr (M == 0 || M == 4 || M == 5) {
        if (dr) {
          hipLaunchKernelGGL((k_flash_dkdv32<T, M, true>), gk, dim3(kThreads), 0, st, a);
          hipLaunchKernelGGL((k_flash_dq32<T, M, true>), gq, dim3(kThreads), 0, st, a);
        } else {
          hipLaunchKernelGGL((k_flash_dkdv32<T, M, false>), gk, dim3(kThreads), 0, st, a);
          hipLaunchKernelGGL((k_flash_dq32<T, M, false>), gq, dim3(kThreads), 0, st, a);
        }
      }
    });
    check_launch("flash_backward");
    return;
  }
  const dim3 gq((unsigned)((a.sq + kQB - 1) / kQB), (unsigned)a.BH);
  const dim3 gk((unsigned)((a.sk + kKB - 1) / kKB), (unsigned)a.BH);
  flash_dispatch(dt, a.mask_mode, "flash_backward", [&](auto tt, auto mm) {
    using T = typename decltype(tt)::type;
    hipLaunchKernelGGL((k_flash_bwd_dkdv<T, decltype(mm)::value>), gk, dim3(kThreads), 0, st, a);
    hipLaunchKernelGGL((k_flash_bwd_dq<T, decltype(mm)::value>), gq, dim3(kThreads), 0, st, a);
  });
  check_launch("flash_backward");
}

}  // namespace bh
