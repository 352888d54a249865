// Transposed-operand MFMA GEMM for gfx950 (see bh/gemm_api.h gemm_tn): C [M, N] = At^T . Bt with At [K, M]
// and Bt [K, N] both contiguous along M / N -- a dense layer's weight gradient dW = dY^T X with the token
// axis as the reduction (csrc/fused_dense_cuda.cu:223-294 and csrc/megatron/fused_weight_gradient_dense.cu
// in the reference run it as a cuBLAS GEMM with both operands transposed).
//
// The 256x256 ping-pong schedule of kernels/gemm.hip (k_gemm_pp: 8 waves as 2 x 4, each 128 x 64 of 16x16
// accumulators, K-step 64 in four barrier-delimited phases with the two wave groups staggered by one
// barrier so one wave of every SIMD multiplies while the other reads LDS and issues the next K-step's
// LDS-DMA) with the operands staged K-major: a K-step's A tile is four 8-KiB sub-images [64 k][64 m] (one
// per 64-column quarter, the units the groups load) and its B tile eight 4-KiB sub-images [64 k][32 n]
// (per wave and column half). The MFMA fragments (8 consecutive k of one m or n per lane) come out of the
// K-major images through ds_read_b64_tr_b16 (16 lanes name a 4 x 16 block and each receives one column of
// 4 rows), two reads per fragment. The 16-byte chunks of every image row are XOR-swizzled by a function of
// the row (fa_sw / fb_sw) so the 32 lanes of one transposed read hit 64 distinct banks; the LDS-DMA writes
// lane-linear 1-KiB pieces, so the swizzle is applied to the SOURCE chunk each lane fetches.
//
// Split-K: the token axis of a weight gradient is long (8k-16k) and its output small (1-16 tiles of 256 x
// 256 per 1024 x 1024), so the grid is tiles x splits; each split writes its fp32 partial tile in the
// accumulator layout (tile-major: every store instruction is 1 KiB of consecutive bytes) and k_tn_reduce
// sums the splits in a fixed order into the row-major 16-bit result (deterministic, no atomics).
#include "bh/api.h"
#include "bh/device.h"
#include "bh/gemm_api.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <typename T> struct Mfma16;
template <> struct Mfma16<f16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma16<bf16> {
  static BH_DEVICE f4v run(i4v a, i4v b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 512;
constexpr int kTile = 256;
constexpr int kBK = 64;
constexpr int kBuf = 65536;   // A 32 KiB (4 sub-images) + B 32 KiB (8 sub-images) per K-step
constexpr int kBOff = 32768;
constexpr unsigned kRsrcWord3 = 0x00020000u;

// chunk swizzles: A rows are 128 B (8 chunks), B rows 64 B (4 chunks); see the header comment
BH_DEVICE int fa_sw(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
BH_DEVICE int fb_sw(int r) { return ((r >> 3) & 1) << 1; }

template <int N> BH_DEVICE void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
BH_DEVICE void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
BH_DEVICE i2v tr4(const char* p) {
  return __builtin_bit_cast(i2v, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)p));
}

struct TnArgs {
  const void* A;  // At [K, lda]
  const void* B;  // Bt [K, ldb]
  void* C;        // [M, N] 16-bit (PART == false)
  float* ws;      // [splits, M, N] fp32 partials (PART)
  int64_t lda, ldb;
  int M, N, K;
  int tiles_m, tiles_n, splits;
};

// the row-major A image of the NN layout (k_gemm_pp's): 256 rows x 128 B, chunk XOR-swizzled by (row >> 1) & 7
BH_DEVICE int swz(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

// AK: A is row-major [M, K] (K-contiguous: the NN layout, C = A . Bt, a data gradient dY . W) and staged as
// k_gemm_pp stages it (256 rows x 128 B per K-step, ds_read_b128 fragments); else K-major At [K, M] (TN).
template <typename T, bool PART, bool AK>
__global__ __launch_bounds__(kThreads, 1) void k_gemm_tn(TnArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-aware bijective remap (as k_gemm_pp); consecutive logical ids share an A column panel and K range
  const int nwg = p.tiles_m * p.tiles_n * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tn = wgid % p.tiles_n, rest = wgid / p.tiles_n;
  const int tm = rest % p.tiles_m, split = rest / p.tiles_m;
  const int brow = tm * kTile, bcol = tn * kTile;
  const int nk = p.K / kBK;
  const int kt0 = (int)((int64_t)split * nk / p.splits), kt1 = (int)((int64_t)(split + 1) * nk / p.splits);

  // whole-tensor resources (the host checks K * ld * 2 < 2^32 and M, N % 256 == 0)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.A), (short)0, (int)((int64_t)(AK ? p.M : p.K) * p.lda * 2), (int)kRsrcWord3);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.B), (short)0, (int)((int64_t)p.K * p.ldb * 2), (int)kRsrcWord3);
  const int lda2 = (int)p.lda * 2, ldb2 = (int)p.ldb * 2;
  // per-lane source offsets of this wave's two pieces of a unit (K-step 0; the K-step rides in soffset):
  // A piece pc = 2 wc + i of sub-image u = 2 wr (+1 for unit 3): rows 8 pc + lane / 8, chunk lane % 8;
  // B piece pc of the unit's two sub-images (waves 2 wr, 2 wr + 1): rows 16 (pc % 4) + lane / 4, chunk lane % 4
  int voffA[2], voffB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pc = 2 * wc + i;
    if constexpr (AK) {
      // piece rows wr * 128 + 8 pc + lane / 8 (unit 3: + 64); chunk lane % 8 holds logical chunk
      // (lane % 8) ^ ((row >> 1) & 7) = (lane % 8) ^ ((i << 2) | (prow >> 1)) (the piece parity is i)
      const int prow = lane >> 3;
      voffA[i] = (brow + wr * 128 + 8 * pc + prow) * lda2 + (((lane & 7) ^ ((i << 2) | (prow >> 1))) << 4);
    } else {
      const int ra = 8 * pc + (lane >> 3);
      voffA[i] = ra * lda2 + (brow + 2 * wr * 64 + ((lane & 7) ^ fa_sw(ra)) * 8) * 2;
    }
    const int rb = 16 * (pc & 3) + (lane >> 2);
    const int wcb = 2 * wr + (pc >> 2);
    voffB[i] = rb * ldb2 + (bcol + wcb * 64 + ((lane & 3) ^ fb_sw(rb)) * 8) * 2;
  }

  f4v acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f4v{0.f, 0.f, 0.f, 0.f};

  // unit j of group wr for K-step kt into buffer dst: j0 / j3 A sub-image 2 wr / 2 wr + 1, j1 / j2 the B
  // sub-images of waves 2 wr, 2 wr + 1 for column half 0 / 1
  auto issue = [&](auto jc, char* dst, int kt) {
    constexpr int j = decltype(jc)::value;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pc = 2 * wc + i;
      if constexpr ((j == 0 || j == 3) && AK) {
        const int rb = wr * 128 + (j == 3 ? 64 : 0) + pc * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(dst + rb * 128), 16,
                                                 voffA[i] + (j == 3 ? 64 * lda2 : 0), kt * kBK * 2, 0, 0);
      } else if constexpr (j == 0 || j == 3) {
        const int u = 2 * wr + (j == 3 ? 1 : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(dst + u * 8192 + pc * 1024), 16,
                                                 voffA[i] + (j == 3 ? 128 : 0), kt * kBK * lda2, 0, 0);
      } else {
        const int ni = j == 2 ? 1 : 0;
        const int sub = ni * 4 + 2 * wr + (pc >> 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(dst + kBOff + sub * 4096 + (pc & 3) * 1024), 16,
                                                 voffB[i] + ni * 64, kt * kBK * ldb2, 0, 0);
      }
    }
  };

  // fragment of lane (fr, fq): 8 consecutive k (rows 8 fq .. 8 fq + 7 of k-substep s) of column fr of a
  // 16-column tile, two transposed 4-row reads
  const int fq = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  auto frag = [&](const char* img, int rowb, int s, int col16, bool is_a) -> i4v {
    const int r0 = s * 32 + 8 * fq + q, r1 = r0 + 4;
    const int lch = 2 * col16 + (pq >> 1);
    const int sw0 = is_a ? fa_sw(r0) : fb_sw(r0), sw1 = is_a ? fa_sw(r1) : fb_sw(r1);
    const i2v lo = tr4(img + r0 * rowb + ((lch ^ sw0) << 4) + (pq & 1) * 8);
    const i2v hi = tr4(img + r1 * rowb + ((lch ^ sw1) << 4) + (pq & 1) * 8);
    return i4v{lo[0], lo[1], hi[0], hi[1]};
  };
  i4v af[2][4], b0[2][2], b1[2][2];
  auto read_a = [&](const char* buf, int mi) {
    if constexpr (AK) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int m = 0; m < 4; ++m)
          af[s][m] = *reinterpret_cast<const i4v*>(buf + swz(wr * 128 + mi * 64 + m * 16 + (lane & 15), s * 4 + fq));
    } else {
      const char* img = buf + (2 * wr + mi) * 8192;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int m = 0; m < 4; ++m) af[s][m] = frag(img, 128, s, m, true);
    }
  };
  auto read_b = [&](const char* buf, int ni, i4v (&bf)[2][2]) {
    const char* img = buf + kBOff + (ni * 4 + wc) * 4096;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int n = 0; n < 2; ++n) bf[s][n] = frag(img, 64, s, n, false);
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
          acc[mi * 4 + m][ni * 2 + n] = Mfma16<T>::run(bf[s][n], af[s][m], acc[mi * 4 + m][ni * 2 + n]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // one K-step from buffer cur; unless LAST, stage K-step kt into nxt (the k_gemm_pp phase order and counts)
  auto step = [&](auto last, const char* cur, char* nxt, int kt) {
    constexpr bool LAST = decltype(last)::value;
    read_a(cur, 0);
    read_b(cur, 0, b0);
    if constexpr (!LAST) issue(std::integral_constant<int, 0>{}, nxt, kt);
    if constexpr (LAST) wait_vmcnt<2>(); else wait_vmcnt<4>();
    raw_barrier();
    mfma_q(0, 0, b0);
    raw_barrier();
    read_b(cur, 1, b1);
    if constexpr (!LAST) issue(std::integral_constant<int, 1>{}, nxt, kt);
    if constexpr (LAST) wait_vmcnt<0>(); else wait_vmcnt<4>();
    raw_barrier();
    mfma_q(0, 1, b1);
    raw_barrier();
    read_a(cur, 1);
    if constexpr (!LAST) issue(std::integral_constant<int, 2>{}, nxt, kt);
    if constexpr (!LAST) wait_vmcnt<4>();
    raw_barrier();
    mfma_q(1, 1, b1);
    raw_barrier();
    if constexpr (!LAST) issue(std::integral_constant<int, 3>{}, nxt, kt);
    if constexpr (!LAST) wait_vmcnt<4>();
    raw_barrier();
    mfma_q(1, 0, b0);
    raw_barrier();
  };

  issue(std::integral_constant<int, 0>{}, smem, kt0);
  issue(std::integral_constant<int, 1>{}, smem, kt0);
  issue(std::integral_constant<int, 2>{}, smem, kt0);
  issue(std::integral_constant<int, 3>{}, smem, kt0);
  wait_vmcnt<0>();
  raw_barrier();
  if (wr == 1) raw_barrier();
  for (int kt = kt0; kt + 1 < kt1; ++kt)
    step(std::false_type{}, smem + ((kt - kt0) & 1) * kBuf, smem + ((kt + 1 - kt0) & 1) * kBuf, kt + 1);
  step(std::true_type{}, smem + ((kt1 - 1 - kt0) & 1) * kBuf, nullptr, 0);
  if (wr == 0) raw_barrier();

  // acc[mt][nt][j] = C[row fr of 16-row tile mt][column 4 fq + j of 16-column tile nt] (B ran first)
  const int fr = lane & 15;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int64_t row = brow + wr * 128 + mt * 16 + fr;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = bcol + wc * 64 + nt * 16 + 4 * fq;
      if constexpr (PART) {
        // tile-major partials: every lane's 16 bytes are consecutive (1 KiB per store instruction)
        const int64_t idx = (((((int64_t)split * p.tiles_m * p.tiles_n + tm * p.tiles_n + tn) * 8 + wave) * 8 + mt) * 4 +
                             nt) * 64 + lane;
        *reinterpret_cast<f4v*>(p.ws + idx * 4) = acc[mt][nt];
      } else {
        typedef T t4 __attribute__((ext_vector_type(4)));
        t4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = from_f<T>(acc[mt][nt][j]);
        *reinterpret_cast<t4*>(reinterpret_cast<T*>(p.C) + row * p.N + col) = o;
      }
    }
  }
}

// sum of the splits' tile-major partials in split order (deterministic) into the row-major C: ACC 0 stores it
// rounded to T, 1 adds it to an fp32 C, 2 adds it to a 16-bit C (in fp32, rounded once)
template <typename T, int ACC>
__global__ __launch_bounds__(256) void k_tn_reduce(const float* __restrict__ ws, void* __restrict__ Cv, int N,
                                                  int tiles_n, int64_t per_split, int splits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= per_split) return;
  f4v acc = *reinterpret_cast<const f4v*>(ws + i * 4);
  for (int s = 1; s < splits; ++s) acc += *reinterpret_cast<const f4v*>(ws + ((int64_t)s * per_split + i) * 4);
  const int lane = (int)(i & 63), nt = (int)((i >> 6) & 3), mt = (int)((i >> 8) & 7), wave = (int)((i >> 11) & 7);
  const int64_t tile = i >> 14;
  const int tm = (int)(tile / tiles_n), tn = (int)(tile % tiles_n);
  const int64_t row = (int64_t)tm * kTile + (wave >> 2) * 128 + mt * 16 + (lane & 15);
  const int col = tn * kTile + (wave & 3) * 64 + nt * 16 + 4 * (lane >> 4);
  typedef T t4 __attribute__((ext_vector_type(4)));
  if constexpr (ACC == 1) {
    f4v* dst = reinterpret_cast<f4v*>(reinterpret_cast<float*>(Cv) + row * N + col);
    *dst = *dst + acc;
  } else {
    t4* dst = reinterpret_cast<t4*>(reinterpret_cast<T*>(Cv) + row * N + col);
    t4 o;
    if constexpr (ACC == 2) {
      const t4 old = *dst;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<T>(to_f<T>(old[j]) + acc[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<T>(acc[j]);
    }
    *dst = o;
  }
}

}  // namespace

bool gemm_tn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* At, const void* Bt,
                       const void* C) {
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return M > 0 && N > 0 && K > 0 && M % kTile == 0 && N % kTile == 0 && K % kBK == 0 && lda >= M && ldb >= N &&
         lda % 8 == 0 && ldb % 8 == 0 && al(At) && al(Bt) && al(C) && K * lda * 2 < 0x7fffffffll &&
         K * ldb * 2 < 0x7fffffffll && M * N < (1ll << 31);
}

bool gemm_nn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A, const void* Bt,
                       const void* C) {
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return M > 0 && N > 0 && K > 0 && M % kTile == 0 && N % kTile == 0 && K % kBK == 0 && lda >= K && ldb >= N &&
         lda % 8 == 0 && ldb % 8 == 0 && al(A) && al(Bt) && al(C) && M * lda * 2 < 0x7fffffffll &&
         K * ldb * 2 < 0x7fffffffll && M * N < (1ll << 31);
}

int gemm_tn_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = (M / kTile) * (N / kTile), nk = K / kBK;
  // about one round of workgroups (one per CU), at least 8 K-steps per split
  int64_t s = std::max<int64_t>(1, 256 / std::max<int64_t>(1, tiles));
  s = std::min<int64_t>(s, std::max<int64_t>(1, nk / 8));
  return (int)s;
}

namespace {
void run_tn(bool ak, int dt, const void* At, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
            int64_t K, float* ws, int splits, hipStream_t st, int accum);
}

void gemm_tn(int dt, const void* At, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
             int64_t K, float* ws, int splits, hipStream_t st, int accum) {
  if (!gemm_tn_supported(M, N, K, lda, ldb, At, Bt, C))
    throw std::runtime_error("gemm_tn: needs M, N % 256 == 0, K % 64 == 0, ld % 8 == 0, 16-byte alignment");
  run_tn(false, dt, At, lda, Bt, ldb, C, M, N, K, ws, splits, st, accum);
}

void gemm_nn(int dt, const void* A, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
             int64_t K, float* ws, int splits, hipStream_t st) {
  if (!gemm_nn_supported(M, N, K, lda, ldb, A, Bt, C))
    throw std::runtime_error("gemm_nn: needs M, N % 256 == 0, K % 64 == 0, ld % 8 == 0, 16-byte alignment");
  run_tn(true, dt, A, lda, Bt, ldb, C, M, N, K, ws, splits, st, 0);
}

namespace {
void run_tn(bool ak, int dt, const void* At, int64_t lda, const void* Bt, int64_t ldb, void* C, int64_t M, int64_t N,
            int64_t K, float* ws, int splits, hipStream_t st, int accum) {
  if (splits < 1 || splits > K / kBK || ((splits > 1 || accum) && !ws)) throw std::runtime_error("gemm_tn: bad split count");
  const bool part = splits > 1 || accum != 0;  // accumulation always goes through the partials
  TnArgs a;
  a.A = At;
  a.B = Bt;
  a.C = C;
  a.ws = ws;
  a.lda = lda;
  a.ldb = ldb;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.tiles_m = (int)(M / kTile);
  a.tiles_n = (int)(N / kTile);
  a.splits = splits;
  const unsigned grid = (unsigned)((int64_t)a.tiles_m * a.tiles_n * splits);
  auto go = [&](auto tt) {
    using T = decltype(tt);
    if (ak) {
      if (part) hipLaunchKernelGGL((k_gemm_tn<T, true, true>), dim3(grid), dim3(kThreads), 0, st, a);
      else hipLaunchKernelGGL((k_gemm_tn<T, false, true>), dim3(grid), dim3(kThreads), 0, st, a);
    } else {
      if (part) hipLaunchKernelGGL((k_gemm_tn<T, true, false>), dim3(grid), dim3(kThreads), 0, st, a);
      else hipLaunchKernelGGL((k_gemm_tn<T, false, false>), dim3(grid), dim3(kThreads), 0, st, a);
    }
  };
  switch (dt) {
    case kF16: go(f16{}); break;
    case kBF16: go(bf16{}); break;
    default: throw std::runtime_error("gemm_tn: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("gemm_tn: ") + hipGetErrorString(e));
  if (part) {
    const int64_t per_split = M * N / 4;  // f4v groups of one split
    const unsigned rg = (unsigned)((per_split + 255) / 256);
    auto red = [&](auto tt, auto accc) {
      using T = decltype(tt);
      constexpr int ACC = decltype(accc)::value;
      hipLaunchKernelGGL((k_tn_reduce<T, ACC>), dim3(rg), dim3(256), 0, st, ws, C, (int)N, a.tiles_n, per_split, splits);
    };
    auto by_acc = [&](auto tt) {
      if (accum == 1) red(tt, std::integral_constant<int, 1>{});
      else if (accum == 2) red(tt, std::integral_constant<int, 2>{});
      else red(tt, std::integral_constant<int, 0>{});
    };
    if (dt == kF16) by_acc(f16{});
    else by_acc(bf16{});
    e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("gemm_tn reduce: ") + hipGetErrorString(e));
  }
}
}  // namespace

}  // namespace bh
