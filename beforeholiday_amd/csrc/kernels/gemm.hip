// MFMA GEMM with fused dense-layer epilogues for gfx950 (CDNA4).
//
// Used where the reference calls hipBLASLt with an epilogue (csrc/fused_dense_cuda.cu:223-294:
// BIAS, GELU_AUX_BIAS, DGELU_BGRAD) or runs separate bias/activation kernels after a GEMM
// (csrc/mlp_cuda.cu:445-958): the activation / activation-derivative / bias-gradient work happens
// on the accumulator tile instead of in a second pass over the [M,N] activation.
//
// Kernel structure (C = A . B^T, A [M,K], B [N,K], both K-contiguous):
//  * 128x128 output tile per 256-thread workgroup; 4 waves in a 2x2 grid, each wave owns 64x64 =
//    4x4 tiles of v_mfma_f32_16x16x32_{f16,bf16} accumulators (64 fp32 VGPRs).
//  * BK = 64. Global -> register (16-byte loads, one 128-B row per 8 lanes) -> LDS staging with two
//    LDS buffers: the loads for K-step t+1 are issued before the MFMAs of step t and written to the
//    other buffer after them, so there is one barrier per K-step.
//  * LDS rows are 128 B; the 16-byte chunk index is XOR-swizzled with (row>>1)&7 so the 16 lanes of
//    a ds_read_b128 group (16 consecutive rows, same chunk) and of a ds_write_b128 group (2 rows x
//    8 chunks) each hit 16 distinct bank slots: conflict-free both ways.
//  * XCD-aware tile order: the bijective remap puts a contiguous range of tiles on each of the 8
//    XCDs (shared B panels stay in one L2).
//  * Epilogue: the fp32 tile is staged through LDS (68-float padded rows) and every lane then owns
//    8 consecutive columns of a row: bias, activation, pre-activation aux and dActivation run on
//    16-byte vectors, C is written with 16-byte stores, and bias-gradient column sums are reduced
//    over the wave's 64 rows with xor-shuffles into a deterministic per-slab partial.
#include "bh/act.h"
#include "bh/knobs.h"
#include "bh/api.h"
#include "bh/device.h"
#include "bh/gemm_api.h"

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int kEpiLd = 68;                          // padded fp32 row of the epilogue image
constexpr int kEpiWaveBytes = 64 * kEpiLd * 4;      // 17 KiB per wave

// Tile configurations: waves arranged WM x WN, each wave owns a (16*TM) x (16*TN) output sub-tile
// of 16x16 MFMA accumulators.
//   Small: 128x128, 4 waves of 64x64, 2 LDS stages (64 KiB, 2 workgroups/CU) - grids too small to
//          fill the chip with the big tile.
//   Big:   256x256, 8 waves of 128x64, 2 LDS stages (128 KiB, 1 workgroup/CU): half the L2 bytes
//          per FLOP of the small tile, 12 ds_read_b128 per 32 MFMAs.
// Tiles are walked in GROUP_M-row groups inside each XCD's contiguous range so the blocks that
// run together on one XCD share A row-panels and B column-panels in its L2.
template <int WM_, int WN_, int TM_, int TN_, int STAGES_> struct Cfg {
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_, STAGES = STAGES_;
  static constexpr int WTM = 16 * TM, WTN = 16 * TN;             // wave tile
  static constexpr int BM = WM * WTM, BN = WN * WTN;
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int kABytes = BM * BK * 2, kBBytes = BN * BK * 2;
  static constexpr int kStageBytes = kABytes + kBBytes;
  static constexpr int kPieces = (BM + BN) / 8;                   // 1-KiB LDS-DMA pieces per stage
  static constexpr int kPiecesPerWave = kPieces / (WM * WN);
  static constexpr int kMainBytes = STAGES * kStageBytes;
  static constexpr int kEpiBytes = WM * WN * kEpiWaveBytes;
  static constexpr int kSmemBytes = kMainBytes > kEpiBytes ? kMainBytes : kEpiBytes;
  static_assert(kPieces % (WM * WN) == 0, "pieces must split evenly over waves");
  static_assert(WTN == 64, "the epilogue image is 64 columns wide");
  static_assert(WTM % 64 == 0, "the epilogue walks 64-row chunks");
};
using CfgSmall = Cfg<2, 2, 4, 4, 2>;
using CfgBig = Cfg<2, 4, 8, 4, 2>;
using CfgMid = Cfg<4, 2, 4, 4, 3>;  // 256x128, 8 waves of 64x64, 3-stage LDS-DMA ring (144 KiB)
constexpr int kGroupM = 8;

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

typedef float f2v __attribute__((ext_vector_type(2)));

// sum over the 16 lanes of a DPP row (every lane gets it): quad_perm [1,0,3,2] and [2,3,0,1] sum each
// quad, row_half_mirror pairs the two quads of each half, row_mirror the two halves (fixed order)
BH_DEVICE float row16_sum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xF, 0xF, false));
  return x;
}

BH_DEVICE int swz(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

template <int N> BH_DEVICE void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// raw workgroup barrier (no implicit vmcnt(0) drain) that the compiler may not move LDS reads across
BH_DEVICE void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Args {
  const void* A;
  const void* B;
  void* C;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  GemmEpilogue epi;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 4 consecutive 16-bit elements <-> fp32 (one 8-byte access)
template <typename T> BH_DEVICE void load4(const T* p, float (&r)[4]) {
  typedef T t4 __attribute__((ext_vector_type(4)));
  const t4 v = *reinterpret_cast<const t4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = static_cast<float>(v[i]);
}
template <typename T> BH_DEVICE void store4(T* p, const float (&r)[4]) {
  typedef T t4 __attribute__((ext_vector_type(4)));
  t4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = static_cast<T>(r[i]);
  *reinterpret_cast<t4*>(p) = v;
}

// One K-step of A and B via LDS-DMA (global_load_lds, 16 B per lane): each wave-instruction fills
// one 1-KiB piece = 8 rows of 128 B. The LDS destination is lane-linear, so the XOR swizzle is
// applied to the per-lane SOURCE chunk (logical chunk = physical ^ ((row>>1)&7)). Pieces
// [0, BM/8) are A rows, the rest B rows. Source pointers are computed once per workgroup; a
// K-step only adds k0.
template <typename C, typename T> struct GldsSrc {
  const T* src[C::kPiecesPerWave];
  BH_DEVICE void init(const T* A, const T* B, int64_t lda, int64_t ldb, int brow, int bcol, int M, int N, int wave,
                      int lane) {
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < C::kPiecesPerWave; ++i) {
      const int piece = wave * C::kPiecesPerWave + i;
      const bool is_a = piece < C::BM / 8;
      const int row = (is_a ? piece : piece - C::BM / 8) * 8 + prow;
      const int ch = pch ^ ((row >> 1) & 7);
      src[i] = is_a ? A + (int64_t)min(brow + row, M - 1) * lda + ch * 8
                    : B + (int64_t)min(bcol + row, N - 1) * ldb + ch * 8;
    }
  }
  BH_DEVICE void issue(char* buf, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < C::kPiecesPerWave; ++i)
      __builtin_amdgcn_global_load_lds(src[i] + k0, (lds_ptr_t)(buf + (wave * C::kPiecesPerWave + i) * 1024), 16, 0,
                                       0);
  }
};

// GLDS: LDS-DMA staging (requires K % 64 == 0); otherwise register staging with zero-filled K tail
// (small config only).
template <typename C, typename T, bool GLDS>
__global__ __launch_bounds__(C::kThreads, 1) void k_gemm_nt(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[C::kSmemBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / C::WN, wc = wave % C::WN;

  // XCD-aware bijective remap of the linear workgroup id
  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = kGroupM * p.tiles_n;
  const int first_m = (wgid / per_group) * kGroupM;
  const int gsize = min(p.tiles_m - first_m, kGroupM);
  const int tm = first_m + (wgid % per_group) % gsize, tn = (wgid % per_group) / gsize;
  const int brow = tm * C::BM, bcol = tn * C::BN;

  const T* __restrict__ A = reinterpret_cast<const T*>(p.A);
  const T* __restrict__ B = reinterpret_cast<const T*>(p.B);

  f4v acc[C::TM][C::TN];
#pragma unroll
  for (int m = 0; m < C::TM; ++m)
#pragma unroll
    for (int n = 0; n < C::TN; ++n) acc[m][n] = f4v{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // Both 32-deep k-slices' fragments are read up front (the second slice's LDS latency hides
  // behind the first slice's MFMAs); sched_barrier keeps hipcc from re-interleaving the reads into
  // read-pair / lgkmcnt(0) / 8-MFMA groups.
  auto compute = [&](const char* sa) {
    const char* sb = sa + C::kABytes;
    i4v af[2][C::TM], bf[2][C::TN];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int n = 0; n < C::TN; ++n)
        bf[s][n] = *reinterpret_cast<const i4v*>(sb + swz(wc * C::WTN + n * 16 + fr, s * 4 + fq));
#pragma unroll
      for (int m = 0; m < C::TM; ++m)
        af[s][m] = *reinterpret_cast<const i4v*>(sa + swz(wr * C::WTM + m * 16 + fr, s * 4 + fq));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int m = 0; m < C::TM; ++m)
#pragma unroll
        for (int n = 0; n < C::TN; ++n) acc[m][n] = Mfma<T>::run(af[s][m], bf[s][n], acc[m][n]);
    }
  };

  const int nk = (p.K + BK - 1) / BK;
  if constexpr (GLDS) {
    static_assert(C::STAGES >= 2, "");
    GldsSrc<C, T> g;
    g.init(A, B, p.lda, p.ldb, brow, bcol, p.M, p.N, wave, lane);
    // prologue: STAGES-1 K-steps in flight
#pragma unroll
    for (int s = 0; s < C::STAGES - 1; ++s)
      if (s < nk) g.issue(smem + s * C::kStageBytes, s * BK, wave);
    if (C::STAGES == 3 && nk > 1) wait_vmcnt<C::kPiecesPerWave>();  // step 0 landed, step 1 may fly
    else wait_vmcnt<0>();
    raw_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const int nxt = kt + C::STAGES - 1;
      if (nxt < nk) g.issue(smem + (nxt % C::STAGES) * C::kStageBytes, nxt * BK, wave);
      compute(smem + (kt % C::STAGES) * C::kStageBytes);
      __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs ahead of the DMA wait + barrier
      // retire step kt+1 (leave the newest STAGES-2 steps in flight); then every wave's DMA for it
      // has landed once all waves pass the barrier. The barrier also orders this step's LDS reads
      // before the buffer is restaged.
      if (C::STAGES == 3 && nxt < nk) wait_vmcnt<C::kPiecesPerWave>();
      else wait_vmcnt<0>();
      raw_barrier();
    }
  } else {
    static_assert(C::BM == 128 && C::BN == 128 && C::kThreads == 256, "register staging: 128x128 config only");
    const int ld_row = tid >> 3, ld_ch = tid & 7;
    const T* a_src[4];
    const T* b_src[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a_src[i] = A + (int64_t)min(brow + ld_row + 32 * i, p.M - 1) * p.lda + ld_ch * 8;
      b_src[i] = B + (int64_t)min(bcol + ld_row + 32 * i, p.N - 1) * p.ldb + ld_ch * 8;
    }
    i4v ra[4], rb[4];
    auto load = [&](int kt) {
      const int k0 = kt * BK;
      const bool ok = k0 + ld_ch * 8 < p.K;
      const int koff = ok ? k0 : (p.K - 8 - ld_ch * 8);  // clamped, always in bounds (K >= 8)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        i4v va = *reinterpret_cast<const i4v*>(a_src[i] + koff);
        i4v vb = *reinterpret_cast<const i4v*>(b_src[i] + koff);
        ra[i] = ok ? va : i4v{0, 0, 0, 0};
        rb[i] = ok ? vb : i4v{0, 0, 0, 0};
      }
    };
    auto store = [&](int buf) {
      char* sa = smem + buf * C::kStageBytes;
      char* sb = sa + C::kABytes;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = ld_row + 32 * i;
        *reinterpret_cast<i4v*>(sa + swz(row, ld_ch)) = ra[i];
        *reinterpret_cast<i4v*>(sb + swz(row, ld_ch)) = rb[i];
      }
    };
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load(kt + 1);
      compute(smem + cur * C::kStageBytes);
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue, in 64-row chunks of the wave tile: stage the fp32 chunk in this wave's private
  // LDS image (C/D map: col = lane&15, row = 4*(lane>>4)+j), then every lane owns 8 consecutive
  // columns of 8 rows: 16-byte bias / aux loads, 16-byte C stores, shuffle-reduced bias-grad sums.
  __syncthreads();  // all waves are done reading the staging buffers
  float* img = reinterpret_cast<float*>(smem + wave * kEpiWaveBytes);
  const GemmEpilogue& e = p.epi;
  const int cg = lane & 7;
  const int gcol = bcol + wc * C::WTN + cg * 8;
  const bool col_ok = gcol < p.N;
  float bias[8];
  if (e.bias && col_ok && !e.bwd_act) {
    VecIO<T>::load(reinterpret_cast<const T*>(e.bias) + gcol, bias);
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c) bias[c] = 0.f;
  }
  T* __restrict__ Cp = reinterpret_cast<T*>(p.C);
  // BatchNorm statistics epilogue (e.bn_stats, see bh/gemm_api.h): per-column constants of this
  // lane's 8 columns, loaded once
  float bk[8], bsc[8], bsh[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) bk[c] = bsc[c] = bsh[c] = 0.f;
  if (e.bn_stats && col_ok) {
    if (e.bn_stats == 1) {
      if (e.kshift) VecIO<float>::load(e.kshift + gcol, bk);
    } else {
      VecIO<float>::load(e.bn_scale + gcol, bsc);
      VecIO<float>::load(e.bn_shift + gcol, bsh);
      VecIO<float>::load(e.bn_mean + gcol, bk);
    }
  }
#pragma unroll
  for (int chunk = 0; chunk < C::TM / 4; ++chunk) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < C::TN; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) img[(m * 16 + fq * 4 + j) * kEpiLd + n * 16 + fr] = acc[chunk * 4 + m][n][j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image is wave-private: in-order LDS suffices
    const int row0 = brow + wr * C::WTM + chunk * 64;
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float csq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int i = 0; i < 8; ++i) {
      const int lr = (lane >> 3) + 8 * i;
      const int grow = row0 + lr;
      float v[8];
      const f4v lo = *reinterpret_cast<const f4v*>(img + lr * kEpiLd + cg * 8);
      const f4v hi = *reinterpret_cast<const f4v*>(img + lr * kEpiLd + cg * 8 + 4);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
      if (grow < p.M && col_ok) {
        if (e.bwd_act) {
          if (e.act != kActNone) {
            float a[8];
            VecIO<T>::load(reinterpret_cast<const T*>(e.aux_in) + (int64_t)grow * e.ld_aux + gcol, a);
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] *= act_d(a[c], e.act);
          }
          // bias grad of the value actually stored (rounded like the reference's separate pass)
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            v[c] = to_f<T>(from_f<T>(v[c]));
            csum[c] += v[c];
          }
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] += bias[c];
          if (e.pre_out) VecIO<T>::store(reinterpret_cast<T*>(e.pre_out) + (int64_t)grow * e.ld_aux + gcol, v);
          if (e.act != kActNone) {
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = act_f(v[c], e.act);
          }
        }
        VecIO<T>::store(Cp + (int64_t)grow * p.ldc + gcol, v);
        if (e.bn_stats == 1) {  // statistics of the stored value, centred on kshift
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float d = to_f<T>(from_f<T>(v[c])) - bk[c];
            csum[c] += d;
            csq[c] = fmaf(d, d, csq[c]);
          }
        } else if (e.bn_stats == 2) {  // the previous BatchNorm's backward sums
          float y[8];
          VecIO<T>::load(reinterpret_cast<const T*>(e.bn_y) + (int64_t)grow * p.ldc + gcol, y);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float g = to_f<T>(from_f<T>(v[c]));
            const float dz = (!e.bn_relu || fmaf(y[c], bsc[c], bsh[c]) > 0.f) ? g : 0.f;
            csum[c] += dz;
            csq[c] = fmaf(dz, y[c] - bk[c], csq[c]);
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image reads done before the next chunk
    if (e.bn_stats) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = csum[c], b = csq[c];
        a += __shfl_xor(a, 8);
        b += __shfl_xor(b, 8);
        a += __shfl_xor(a, 16);
        b += __shfl_xor(b, 16);
        a += __shfl_xor(a, 32);
        b += __shfl_xor(b, 32);
        csum[c] = a;
        csq[c] = b;
      }
      const int64_t slab = row0 / 64, slabs = ((int64_t)p.M + 63) / 64;
      if (lane < 8 && col_ok && row0 < p.M) {
        float* d1 = e.stat_part + slab * p.N + gcol;
        float* d2 = e.stat_part + (slabs + slab) * p.N + gcol;
        VecIO<float>::store(d1, csum);
        VecIO<float>::store(d2, csq);
      }
    }
    if (e.bgrad_part) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float sacc = csum[c];
        sacc += __shfl_xor(sacc, 8);
        sacc += __shfl_xor(sacc, 16);
        sacc += __shfl_xor(sacc, 32);
        csum[c] = sacc;
      }
      const int slab = row0 / 64;  // global 64-row slab; slabs past M are never read
      if (lane < 8 && col_ok && row0 < p.M) {
        float* dst = e.bgrad_part + (int64_t)slab * p.N + gcol;
        *reinterpret_cast<float4*>(dst) = make_float4(csum[0], csum[1], csum[2], csum[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(csum[4], csum[5], csum[6], csum[7]);
      }
    }
  }
}

// ---- 256x256 ping-pong kernel (large grids, K % 64 == 0) ----------------------------------------
//
// 8 waves as 2 (rows) x 4 (cols), each owning 128x64 outputs (acc[8][4] of 16x16 tiles). A K-step
// of 64 is split into four phases, one per 64x32 quadrant of the wave tile (16 MFMAs each), and
// every phase is two barrier-delimited segments: R (ds_read the quadrant's fragments, issue one
// 8-KiB unit of the NEXT K-step's LDS-DMA, counted vmcnt) and M (the 16 MFMAs). The wave group
// wr == 1 executes one extra barrier up front, so on every SIMD - which holds one wave of each
// group - one wave runs its MFMA segment while the other reads LDS and issues loads: the matrix
// core never waits on LDS latency and the DMA of a unit has ~5 segments to land.
//
// Units (64 rows x 128 B) of a K-step, issued by group g in phase j: j0 A rows g*128+[0,64),
// j1 / j2 the ni = 0 / 1 column halves of B rows g*128+[0,128), j3 A rows g*128+[64,128). The
// `vmcnt(4)` in each R segment retires every unit issued two own-R-segments earlier, which is
// before the barrier ahead of its first reader (A halves are read only by their own group; a B
// unit of group h is first read one phase after it is retired, by either group). Reads of step t
// finish before step t+1's loads overwrite that buffer (two LDS buffers, 128 KiB).
//
// Loads are buffer_load ... lds through a per-workgroup buffer resource whose range ends at the
// last valid row, so rows past M / N land as zeros without clamped per-lane pointers; the per-lane
// VGPR offset carries the row (range-checked), the K offset rides in the scalar offset.
constexpr int kPPThreads = 512;
constexpr int kPPTile = 256;
constexpr int kPPBuf = 65536;  // A 32 KiB + B 32 KiB per K-step
constexpr int kPPSmem = 2 * kPPBuf;
constexpr unsigned kRsrcWord3 = 0x00020000u;

BH_DEVICE __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, int64_t rows_left, int64_t ld) {
  const int64_t bytes = rows_left * ld * 2;
  const int nrec = bytes >= 0xFFFFFFFFll ? (int)0xFFFFFFFFu : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, (int)kRsrcWord3);
}

// ACT / BWD as template parameters: one epilogue path per kernel (all of them in one function pushed
// the register allocator past 256 VGPRs and into scratch)
// STATS: 0 none, 1 forward statistics (bn_stats 1), 2 the previous BatchNorm's backward sums (bn_stats 2)
template <typename T, int ACT, bool BWD, int STATS = 0>
__global__ __launch_bounds__(kPPThreads, 1) void k_gemm_pp(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[kPPSmem];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = kGroupM * p.tiles_n;
  const int first_m = (wgid / per_group) * kGroupM;
  const int gsize = min(p.tiles_m - first_m, kGroupM);
  const int tm = first_m + (wgid % per_group) % gsize, tn = (wgid % per_group) / gsize;
  const int brow = tm * kPPTile, bcol = tn * kPPTile;

  const __amdgpu_buffer_rsrc_t rsA =
      tile_rsrc(reinterpret_cast<const T*>(p.A) + (int64_t)brow * p.lda, p.M - brow, p.lda);
  const __amdgpu_buffer_rsrc_t rsB =
      tile_rsrc(reinterpret_cast<const T*>(p.B) + (int64_t)bcol * p.ldb, p.N - bcol, p.ldb);
  const int lda2 = (int)p.lda * 2, ldb2 = (int)p.ldb * 2;
  // per-lane part of a 1-KiB piece (8 rows x 8 chunks): row prow, physical chunk pch holding
  // logical chunk pch ^ ((row >> 1) & 7); a piece's first row is a multiple of 8 whose parity of
  // row / 8 is the piece parity i, so the XOR is ((i << 2) | (prow >> 1)).
  const int prow = lane >> 3, pch = lane & 7;
  int voffA[2], voffB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = pch ^ ((i << 2) | (prow >> 1));
    voffA[i] = prow * lda2 + ch * 16;
    voffB[i] = prow * ldb2 + ch * 16;
  }

  f4v acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f4v{0.f, 0.f, 0.f, 0.f};

  // unit j of group wr for the K-step at byte offset kb, into buffer dst; wave wc takes pieces
  // 2wc, 2wc+1 of the unit's eight
  auto issue = [&](auto jc, char* dst, int kb) {
    constexpr int j = decltype(jc)::value;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (j == 0 || j == 3) {
        const int rb = wr * 128 + (j == 3 ? 64 : 0) + (2 * wc + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(dst + rb * 128), 16, voffA[i] + rb * lda2, kb, 0,
                                                 0);
      } else {
        const int rb = (2 * wr + (wc >> 1)) * 64 + (j == 2 ? 32 : 0) + (2 * (wc & 1) + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(dst + 32768 + rb * 128), 16, voffB[i] + rb * ldb2,
                                                 kb, 0, 0);
      }
    }
  };

  const int fr = lane & 15, fq = lane >> 4;
  i4v af[2][4], b0[2][2], b1[2][2];
  auto read_a = [&](const char* sa, int mi) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        af[s][m] = *reinterpret_cast<const i4v*>(sa + swz(wr * 128 + mi * 64 + m * 16 + fr, s * 4 + fq));
  };
  auto read_b = [&](const char* sb, int ni, i4v (&bf)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bf[s][n] = *reinterpret_cast<const i4v*>(sb + swz(wc * 64 + ni * 32 + n * 16 + fr, s * 4 + fq));
  };
  auto mfma_q = [&](int mi, int ni, const i4v (&bf)[2][2]) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[mi * 4 + m][ni * 2 + n] = Mfma<T>::run(bf[s][n], af[s][m], acc[mi * 4 + m][ni * 2 + n]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // one K-step from buffer cur; unless LAST, stage K-step byte offset kb into nxt
  auto step = [&](auto last, const char* cur, char* nxt, int kb) {
    constexpr bool LAST = decltype(last)::value;
    const char* sa = cur;
    const char* sb = cur + 32768;
    // phase 0: quadrant (0, 0)
    read_a(sa, 0);
    read_b(sb, 0, b0);
    if constexpr (!LAST) issue(std::integral_constant<int, 0>{}, nxt, kb);
    if constexpr (LAST) wait_vmcnt<2>(); else wait_vmcnt<4>();
    raw_barrier();
    mfma_q(0, 0, b0);
    raw_barrier();
    // phase 1: quadrant (0, 1)
    read_b(sb, 1, b1);
    if constexpr (!LAST) issue(std::integral_constant<int, 1>{}, nxt, kb);
    if constexpr (LAST) wait_vmcnt<0>(); else wait_vmcnt<4>();
    raw_barrier();
    mfma_q(0, 1, b1);
    raw_barrier();
    // phase 2: quadrant (1, 1)
    read_a(sa, 1);
    if constexpr (!LAST) issue(std::integral_constant<int, 2>{}, nxt, kb);
    if constexpr (!LAST) wait_vmcnt<4>();
    raw_barrier();
    mfma_q(1, 1, b1);
    raw_barrier();
    // phase 3: quadrant (1, 0), fragments already in registers
    if constexpr (!LAST) issue(std::integral_constant<int, 3>{}, nxt, kb);
    if constexpr (!LAST) wait_vmcnt<4>();
    raw_barrier();
    mfma_q(1, 0, b0);
    raw_barrier();
  };

  // prologue: the whole first K-step, then stagger the groups
  issue(std::integral_constant<int, 0>{}, smem, 0);
  issue(std::integral_constant<int, 1>{}, smem, 0);
  issue(std::integral_constant<int, 2>{}, smem, 0);
  issue(std::integral_constant<int, 3>{}, smem, 0);
  wait_vmcnt<0>();
  raw_barrier();
  if (wr == 1) raw_barrier();
  const int nk = p.K / BK;
  for (int kt = 0; kt + 1 < nk; ++kt)
    step(std::false_type{}, smem + (kt & 1) * kPPBuf, smem + ((kt + 1) & 1) * kPPBuf, (kt + 1) * BK * 2);
  step(std::true_type{}, smem + ((nk - 1) & 1) * kPPBuf, nullptr, 0);
  if (wr == 0) raw_barrier();

  // ---- epilogue. The MFMAs ran with B as the first operand, so acc[mt][nt][j] = C[row fr of 16-row
  // tile mt][column 4 * fq + j of 16-column tile nt]: a lane holds 4 consecutive columns of one row,
  // and 16 lanes of a store instruction would hit 16 rows with 8 bytes each (32-byte segments: the
  // output then leaves at a fraction of the HBM rate). Instead every result tensor goes through a
  // wave-private 128 x 64 LDS image (16 KiB per wave; the two 64 KiB main-loop buffers are free):
  // lanes write their 8-byte pieces (16-byte chunk index XOR-swizzled by row & 7, 2-way at worst),
  // then each lane reads one 16-byte chunk back and a store instruction covers 8 rows x 128 bytes.
  // The dGELU input aux_in comes in the same way in reverse (coalesced 16-byte loads -> image ->
  // the accumulator layout).
  const GemmEpilogue& e = p.epi;
  T* __restrict__ Cp = reinterpret_cast<T*>(p.C);
  const int col_l = bcol + wc * 64 + fq * 4;
  const int row_w = brow + wr * 128;  // first row of the wave tile
  __syncthreads();                     // every wave is past its last main-loop LDS read
  char* img = smem + wave * 16384;
  typedef T t4 __attribute__((ext_vector_type(4)));
  auto img_off = [&](int r, int chunk) { return r * 128 + ((chunk ^ (r & 7)) << 4); };
  auto put_h = [&](int mt, int nt, const t4& o) {
    const int r = mt * 16 + fr;
    *reinterpret_cast<t4*>(img + img_off(r, nt * 2 + (fq >> 1)) + (fq & 1) * 8) = o;
  };
  auto put = [&](int mt, int nt, const float (&v)[4]) {
    t4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = static_cast<T>(v[j]);
    put_h(mt, nt, o);
  };
  auto get = [&](int mt, int nt, float (&v)[4]) {
    const int r = mt * 16 + fr;
    const t4 o = *reinterpret_cast<const t4*>(img + img_off(r, nt * 2 + (fq >> 1)) + (fq & 1) * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = static_cast<float>(o[j]);
  };
  const int cc = lane & 7, rq = lane >> 3;
  const int fcol = bcol + wc * 64 + cc * 8;
  // (four 16-byte chunks in flight per lane at a time: the accumulators stay live across a flush)
  auto flush = [&](T* dst, int64_t ld) {  // image -> 128 rows x 64 columns of dst
#pragma unroll 1
    for (int i0 = 0; i0 < 16; i0 += 4) {
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i) {
        const int rr = i * 8 + rq, row = row_w + rr;
        const i4v v = *reinterpret_cast<const i4v*>(img + img_off(rr, cc));
        if (row < p.M && fcol < p.N) *reinterpret_cast<i4v*>(dst + (int64_t)row * ld + fcol) = v;
      }
    }
  };
  auto fill = [&](const T* src, int64_t ld) {  // 128 rows x 64 columns of src -> image
#pragma unroll 1
    for (int i0 = 0; i0 < 16; i0 += 4) {
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i) {
        const int rr = i * 8 + rq, row = row_w + rr;
        i4v v = i4v{0, 0, 0, 0};
        if (row < p.M && fcol < p.N) v = *reinterpret_cast<const i4v*>(src + (int64_t)row * ld + fcol);
        *reinterpret_cast<i4v*>(img + img_off(rr, cc)) = v;
      }
    }
  };
  {
    if constexpr (!BWD) {
      if (e.resid) {  // C = A.B^T + resid: the residual comes in through the image, then onto the accumulators
        fill(reinterpret_cast<const T*>(e.resid), p.ldc);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            float r[4];
            get(mt, nt, r);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[mt][nt][j] += r[j];
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image reads done before it is rewritten
      }
      // bias folded into the accumulators first (the pre-activation, kept in fp32 for the activation)
      if (e.bias) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int col = col_l + nt * 16;
          float b[4] = {0.f, 0.f, 0.f, 0.f};
          if (col < p.N) load4<T>(reinterpret_cast<const T*>(e.bias) + col, b);
#pragma unroll
          for (int mt = 0; mt < 8; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[mt][nt][j] += b[j];
        }
      }
      if (e.pre_out) {  // the pre-activation (aux) image first
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j];
            put(mt, nt, v);
          }
        flush(reinterpret_cast<T*>(e.pre_out), e.ld_aux);
      }
      // BatchNorm statistics of the stored values (bn_stats == 1): sums of c - kshift and its square
      // per column, accumulated while the tile goes into the image (the accumulators die there; the
      // stats never hold them live across the flush), over the wave's 128 rows (16 row lanes x 8
      // tiles), written to the 64-row slab of row_w (the next slab gets zeros, as the fixed-order
      // partial reduction expects every slab)
      // (packed fp32: v_pk_add_f32 / v_pk_fma_f32 on column pairs; the epilogue runs while the CU's
      // matrix cores idle, so its VALU count is step time)
      f2v s1[4][2] = {}, s2[4][2] = {}, kc[4][2] = {};
      if constexpr (STATS == 1) {
        if (e.kshift) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int col = col_l + nt * 16;
            if (col < p.N) {
              const float4 kv = *reinterpret_cast<const float4*>(e.kshift + col);
              kc[nt][0] = f2v{kv.x, kv.y};
              kc[nt][1] = f2v{kv.z, kv.w};
            }
          }
        }
      }
      if constexpr (STATS == 2) {
        // backward sums of the BatchNorm whose input y = bn_y feeds this layer's output gradient:
        // y comes into the image with coalesced loads; each (mt, nt) piece is read back in the
        // accumulator layout and replaced by the output (the dGELU pattern below). Column-tile
        // outer loop: one column tile's scale / shift / mean live at a time.
        fill(reinterpret_cast<const T*>(e.bn_y), p.ldc);
        const int64_t slabs = ((int64_t)p.M + 63) / 64, slab = row_w / 64;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int col = col_l + nt * 16;
          float sc[4] = {0.f, 0.f, 0.f, 0.f}, sh[4] = {0.f, 0.f, 0.f, 0.f}, mu[4] = {0.f, 0.f, 0.f, 0.f};
          if (col < p.N) {
            const float4 a = *reinterpret_cast<const float4*>(e.bn_scale + col);
            const float4 b = *reinterpret_cast<const float4*>(e.bn_shift + col);
            const float4 c = *reinterpret_cast<const float4*>(e.bn_mean + col);
            sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w;
            sh[0] = b.x; sh[1] = b.y; sh[2] = b.z; sh[3] = b.w;
            mu[0] = c.x; mu[1] = c.y; mu[2] = c.z; mu[3] = c.w;
          }
          float t1[4] = {0.f, 0.f, 0.f, 0.f}, t2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int mt = 0; mt < 8; ++mt) {
            const bool row_ok = row_w + mt * 16 + fr < p.M;
            float y[4], v[4];
            get(mt, nt, y);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j];
            put(mt, nt, v);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float g = to_f<T>(from_f<T>(v[j]));
              const bool pass = row_ok && (!e.bn_relu || fmaf(y[j], sc[j], sh[j]) > 0.f);
              const float dz = pass ? g : 0.f;
              t1[j] += dz;
              t2[j] = fmaf(dz, row_ok ? y[j] - mu[j] : 0.f, t2[j]);
            }
          }
          // this column tile's sums over the 16 row lanes, written right away (few live registers)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int m = 1; m < 16; m <<= 1) {
              t1[j] += __shfl_xor(t1[j], m);
              t2[j] += __shfl_xor(t2[j], m);
            }
          if (fr == 0 && row_w < p.M && col < p.N) {
            float* d1 = e.stat_part + slab * p.N + col;
            float* d2 = e.stat_part + (slabs + slab) * p.N + col;
            *reinterpret_cast<float4*>(d1) = make_float4(t1[0], t1[1], t1[2], t1[3]);
            *reinterpret_cast<float4*>(d2) = make_float4(t2[0], t2[1], t2[2], t2[3]);
            if (row_w + 64 < p.M) {
              *reinterpret_cast<float4*>(d1 + p.N) = make_float4(0.f, 0.f, 0.f, 0.f);
              *reinterpret_cast<float4*>(d2 + p.N) = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        const bool partial = row_w + 128 > p.M;  // wave-uniform: only the last row tile masks rows
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          const bool row_ok = row_w + mt * 16 + fr < p.M;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j];
            if constexpr (ACT != kActNone) {
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = act_f(v[j], ACT);
            }
            t4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = static_cast<T>(v[j]);
            put_h(mt, nt, o);
            if constexpr (STATS == 1) {  // statistics of the stored (rounded) values
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                f2v d = f2v{static_cast<float>(o[2 * h]), static_cast<float>(o[2 * h + 1])} - kc[nt][h];
                if (partial && !row_ok) d = f2v{0.f, 0.f};
                s1[nt][h] += d;
                s2[nt][h] = __builtin_elementwise_fma(d, d, s2[nt][h]);
              }
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      flush(Cp, p.ldc);
      if constexpr (STATS == 1) {
        float r1[4][4], r2[4][4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            r1[nt][j] = row16_sum(s1[nt][j >> 1][j & 1]);
            r2[nt][j] = row16_sum(s2[nt][j >> 1][j & 1]);
          }
        const int64_t slabs = ((int64_t)p.M + 63) / 64, slab = row_w / 64;
        if (fr == 0 && row_w < p.M) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int col = col_l + nt * 16;
            if (col >= p.N) continue;
            float* d1 = e.stat_part + slab * p.N + col;
            float* d2 = e.stat_part + (slabs + slab) * p.N + col;
            *reinterpret_cast<float4*>(d1) = make_float4(r1[nt][0], r1[nt][1], r1[nt][2], r1[nt][3]);
            *reinterpret_cast<float4*>(d2) = make_float4(r2[nt][0], r2[nt][1], r2[nt][2], r2[nt][3]);
            if (row_w + 64 < p.M) {
              *reinterpret_cast<float4*>(d1 + p.N) = make_float4(0.f, 0.f, 0.f, 0.f);
              *reinterpret_cast<float4*>(d2 + p.N) = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
        }
      }
    } else {
      float cs[4][4] = {};
      if constexpr (ACT != kActNone) fill(reinterpret_cast<const T*>(e.aux_in), e.ld_aux);
      // each (mt, nt) piece of the image is read (aux), replaced by the dActivation product (same
      // lane, same address) and the next piece follows: a piece's LDS read never waits behind more
      // than one row of tiles, and the accumulators are consumed as they go
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const bool row_ok = row_w + mt * 16 + fr < p.M;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          float v[4];
          if constexpr (ACT != kActNone) {
            float a[4];
            get(mt, nt, a);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j] * act_d(a[j], ACT);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j];
          }
          // bias grad of the value actually stored (rounded like the reference's separate pass)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = to_f<T>(from_f<T>(v[j]));
            if (row_ok && col_l + nt * 16 < p.N) cs[nt][j] += v[j];
          }
          put(mt, nt, v);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      flush(Cp, p.ldc);
      if (e.bgrad_part) {
        // sum over the 16 row lanes; the wave's 128 rows go to its first 64-row slab, the second
        // slab (if it exists) gets zeros so the fixed-order finalize still sees every slab written
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float t = cs[nt][j];
            t += __shfl_xor(t, 1);
            t += __shfl_xor(t, 2);
            t += __shfl_xor(t, 4);
            t += __shfl_xor(t, 8);
            cs[nt][j] = t;
          }
        const int row0 = row_w;
        if (fr == 0 && row0 < p.M) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int col = col_l + nt * 16;
            if (col < p.N) {
              float* dst = e.bgrad_part + (int64_t)(row0 / 64) * p.N + col;
              *reinterpret_cast<float4*>(dst) = make_float4(cs[nt][0], cs[nt][1], cs[nt][2], cs[nt][3]);
              if (row0 + 64 < p.M) *reinterpret_cast<float4*>(dst + p.N) = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
        }
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(64 * kColsumLanes) void k_colsum(const float* __restrict__ part, int64_t slabs, int64_t N,
                                                               T* __restrict__ out) {
  __shared__ float sh[kColsumLanes][64];
  colsum_partials_block<T>(part, slabs, N, out, sh);
}

// out [C, R] = in [R, C]^T for 16-bit elements: 64 x 64 tiles through LDS (ushort rows padded to 66 so the
// column reads spread over banks), 16-byte loads along input rows and 16-byte stores along output rows.
// Used for the weight transposes of the GEMM data gradients (dX = dY . W needs W^T as the [N, K] operand).
__global__ __launch_bounds__(256) void k_transpose16(const uint16_t* __restrict__ in, int64_t R, int64_t C,
                                                      uint16_t* __restrict__ out) {
  __shared__ uint16_t t[64][66];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + i * 256, rr = q >> 3, cc = (q & 7) * 8;
    const int64_t r = r0 + rr, c = c0 + cc;
    uint16_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < R && c + 8 <= C) {
      const uint4 u = *reinterpret_cast<const uint4*>(in + r * C + c);
      __builtin_memcpy(v, &u, 16);
    } else if (r < R) {
      for (int j = 0; j < 8; ++j) if (c + j < C) v[j] = in[r * C + c + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) t[rr][cc + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + i * 256, cc = q >> 3, rr = (q & 7) * 8;  // output row c0 + cc, columns r0 + rr ..
    const int64_t c = c0 + cc, r = r0 + rr;
    if (c >= C) continue;
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[rr + j][cc];
    if (r + 8 <= R) {
      uint4 u;
      __builtin_memcpy(&u, v, 16);
      *reinterpret_cast<uint4*>(out + c * R + r) = u;
    } else {
      for (int j = 0; j < 8; ++j) if (r + j < R) out[c * R + r + j] = v[j];
    }
  }
}

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace

bool gemm_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const void* A,
                    const void* B, const void* C) {
  return M > 0 && N > 0 && K >= 8 && K % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
         lda >= K && ldb >= K && ldc >= N && al16(A) && al16(B) && al16(C) && M < (1ll << 31) && N < (1ll << 31) &&
         K < (1ll << 31);
}

int64_t gemm_bgrad_slabs(int64_t M) { return (M + 63) / 64; }

namespace {
template <typename T>
void launch_pp(const Args& a0, hipStream_t st) {
  Args a = a0;
  a.tiles_m = (a.M + kPPTile - 1) / kPPTile;
  a.tiles_n = (a.N + kPPTile - 1) / kPPTile;
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg >= (1ll << 31)) throw std::runtime_error("gemm_nt: grid too large");
  if (a.epi.bn_stats == 1) {  // statistics epilogue: plain output (no bias / activation / aux)
    hipLaunchKernelGGL((k_gemm_pp<T, kActNone, false, 1>), dim3((unsigned)nwg), dim3(kPPThreads), 0, st, a);
    return;
  }
  if (a.epi.bn_stats == 2) {  // backward-sums epilogue: plain output
    hipLaunchKernelGGL((k_gemm_pp<T, kActNone, false, 2>), dim3((unsigned)nwg), dim3(kPPThreads), 0, st, a);
    return;
  }
  auto go = [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
    if (a.epi.bwd_act) hipLaunchKernelGGL((k_gemm_pp<T, ACT, true>), dim3((unsigned)nwg), dim3(kPPThreads), 0, st, a);
    else hipLaunchKernelGGL((k_gemm_pp<T, ACT, false>), dim3((unsigned)nwg), dim3(kPPThreads), 0, st, a);
  };
  switch (a.epi.act) {
    case kActRelu: go(std::integral_constant<int, kActRelu>{}); break;
    case kActSigmoid: go(std::integral_constant<int, kActSigmoid>{}); break;
    case kActGelu: go(std::integral_constant<int, kActGelu>{}); break;
    case kActGeluTanh: go(std::integral_constant<int, kActGeluTanh>{}); break;
    default: go(std::integral_constant<int, kActNone>{}); break;
  }
}

template <typename C, typename T>
void launch(const Args& a0, bool glds, hipStream_t st) {
  Args a = a0;
  a.tiles_m = (a.M + C::BM - 1) / C::BM;
  a.tiles_n = (a.N + C::BN - 1) / C::BN;
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg >= (1ll << 31)) throw std::runtime_error("gemm_nt: grid too large");
  if (glds) hipLaunchKernelGGL((k_gemm_nt<C, T, true>), dim3((unsigned)nwg), dim3(C::kThreads), 0, st, a);
  else hipLaunchKernelGGL((k_gemm_nt<CfgSmall, T, false>), dim3((unsigned)nwg), dim3(CfgSmall::kThreads), 0, st, a);
}

}  // namespace

namespace {
int g_tile_mode = -1;
}
int gemm_tile_mode() {
  if (g_tile_mode < 0) g_tile_mode = knob("gemm_tile", 0);
  return g_tile_mode;
}
void gemm_set_tile_mode(int mode) { g_tile_mode = mode; }

void gemm_nt(int dt, const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
             int64_t N, int64_t K, const GemmEpilogue& epi, hipStream_t st) {
  if (!gemm_supported(M, N, K, lda, ldb, ldc, A, B, C))
    throw std::runtime_error("gemm_nt: unsupported shape/layout (need K%8==0, N%8==0, ld%8==0, 16B-aligned)");
  if ((epi.pre_out || epi.aux_in) && (epi.ld_aux % 8 != 0 || epi.ld_aux < N))
    throw std::runtime_error("gemm_nt: aux leading dimension must be >= N and a multiple of 8");
  Args a;
  a.A = A; a.B = B; a.C = C;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.epi = epi;
  // tile mode (Config.gemm_tile / gemm_set_tile_mode): 1 small / 2 big / 3 mid / 4 ping-pong / 0 auto
  const int tile_mode = gemm_tile_mode();
  const bool glds = (K % BK) == 0;
  const int64_t big_wgs = ((M + CfgBig::BM - 1) / CfgBig::BM) * ((N + CfgBig::BN - 1) / CfgBig::BN);
  // the ping-pong kernel keeps row offsets of a 256-row tile in 32 bits
  const bool pp_ok = glds && lda < (1 << 22) && ldb < (1 << 22);
  // the ping-pong kernel's BatchNorm epilogues (statistics, backward sums) come with a plain output
  const bool pp_epi = epi.bn_stats == 0 || (!epi.bias && epi.act == kActNone && !epi.pre_out && !epi.bwd_act);
  // auto: the ping-pong kernel from 160 of its 256x256 tiles on (it beats the 128x128 kernel there,
  // benchmarks/bench_resnet_gemms.py), never for outputs of at most 128 columns (half its tile idle:
  // 132 vs ~60 us for the 200704 x 128 x 512 BatchNorm-backward GEMM in the ResNet-50 step)
  const bool pp_auto = N > 128 && big_wgs >= 160;
  const bool pp = pp_ok && pp_epi && (tile_mode == 4 || epi.resid || (tile_mode == 0 && pp_auto));
  if (epi.resid && epi.bwd_act) throw std::runtime_error("gemm_nt: a residual input needs a forward epilogue");
  if (epi.resid && !pp) throw std::runtime_error("gemm_nt: a residual input needs the ping-pong kernel (K % 64 == 0)");
  // (the one-barrier 256x256 kernel only where the ping-pong one is not allowed, never for N <= 128:
  // 108 vs 62 us for the 200704 x 128 x 512 statistics GEMM of the ResNet-50 step)
  const bool big = glds && !pp && (tile_mode == 2 || (tile_mode == 0 && big_wgs >= 256 && N > 128));
  const bool mid = glds && tile_mode == 3;
  const bool log_shapes = knob("gemm_log", 0) != 0;  // debugging: which kernel per shape
  if (log_shapes)
    fprintf(stderr, "[gemm_nt] M %lld N %lld K %lld epi %d resid %d -> %s\n", (long long)M, (long long)N,
            (long long)K, epi.bn_stats, epi.resid != nullptr,
            pp ? "pingpong" : mid ? "256x128" : big ? "256x256" : glds ? "128x128" : "128x128-regs");
  switch (dt) {
    case kF16:
      if (pp) launch_pp<f16>(a, st);
      else if (mid) launch<CfgMid, f16>(a, true, st);
      else if (big) launch<CfgBig, f16>(a, true, st);
      else launch<CfgSmall, f16>(a, glds, st);
      break;
    case kBF16:
      if (pp) launch_pp<bf16>(a, st);
      else if (mid) launch<CfgMid, bf16>(a, true, st);
      else if (big) launch<CfgBig, bf16>(a, true, st);
      else launch<CfgSmall, bf16>(a, glds, st);
      break;
    default: throw std::runtime_error("gemm_nt: fp16 / bf16 only");
  }
  check_launch("gemm_nt");
}

void transpose16(const void* in, int64_t R, int64_t C, void* out, hipStream_t st) {
  if (R <= 0 || C <= 0) return;
  const bool vec = R % 8 == 0 && C % 8 == 0 && al16(in) && al16(out);
  if (!vec) throw std::runtime_error("transpose16: rows / columns must be multiples of 8 and 16-byte aligned");
  const dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  hipLaunchKernelGGL(k_transpose16, grid, dim3(256), 0, st, reinterpret_cast<const uint16_t*>(in), R, C,
                     reinterpret_cast<uint16_t*>(out));
  check_launch("transpose16");
}

void gemm_colsum_finalize(int dt, const float* part, int64_t slabs, int64_t N, void* out, hipStream_t st) {
  const unsigned blocks = (unsigned)((N + 63) / 64);
  switch (dt) {
    case kF16: hipLaunchKernelGGL(k_colsum<f16>, dim3(blocks), dim3(64 * kColsumLanes), 0, st, part, slabs, N, (f16*)out); break;
    case kBF16: hipLaunchKernelGGL(k_colsum<bf16>, dim3(blocks), dim3(64 * kColsumLanes), 0, st, part, slabs, N, (bf16*)out); break;
    default: throw std::runtime_error("gemm_colsum_finalize: fp16 / bf16 only");
  }
  check_launch("gemm_colsum_finalize");
}

}  // namespace bh
