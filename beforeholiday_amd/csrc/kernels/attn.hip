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

#include <stdexcept>
#include <string>

namespace bh {
namespace {

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
  if (k >= a.sk) return -INFINITY;
  switch (a.mask_mode) {
    case 1: return reinterpret_cast<const uint8_t*>(a.mask)[(int64_t)b * a.sk + k] ? -INFINITY : s;
    case 2: return s + reinterpret_cast<const float*>(a.mask)[(int64_t)b * a.sk + k];
    case 3: return (q < a.sq && reinterpret_cast<const uint8_t*>(a.mask)[(int64_t)q * a.sk + k]) ? -INFINITY : s;
    default: return s;
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
  Philox ph(a.seed, ((uint64_t)bh * (uint64_t)a.sq + (uint64_t)qrow4) * (uint64_t)skt + (uint64_t)col, a.offset);
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

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

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

}  // namespace bh
