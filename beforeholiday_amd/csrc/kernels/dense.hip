// Dense-layer epilogue kernels (gfx950): activation forward, fused activation-backward + bias-grad.
//
// Reference behaviour: csrc/fused_dense_cuda.cu (hipBLASLt epilogues BIAS / BGRADB / GELU_AUX_BIAS /
// DGELU_BGRAD, :223-294) and csrc/mlp_cuda.cu (bias+ReLU/sigmoid kernels, bias-grad reductions).
// The reference's linear_gelu_linear_backward never applies dGELU; here it does.
//
// MI355X design: the GEMMs run on hipBLASLt (bias folded into its epilogue by at::addmm); these
// kernels are the memory-bound halves, each a single pass over the activation:
//  * act_fwd:   y = act(x (+ bias)), 16-byte vectors, in place allowed.
//  * act_bwd:   dx = dy * act'(aux) AND the bias gradient sum_m dx in the same pass. Columns are
//    owned by lanes (8 columns per lane, 32 lanes = 256 columns per workgroup, 8 row lanes), each
//    workgroup reduces a row-chunk into an fp32 partial [split][N]; a second tiny kernel sums the
//    splits in a fixed order (deterministic, no atomics).
#include "bh/api.h"
#include "bh/dense_api.h"
#include "bh/device.h"
#include "bh/act.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kColLanes = 32;
constexpr int kRowLanes = 8;
constexpr int kCols = kColLanes * 8;  // columns per workgroup

#define DN_DISPATCH(code, T, ...)                                          \
  switch (code) {                                                          \
    case kF32: { using T = float; __VA_ARGS__; } break;                    \
    case kF16: { using T = f16; __VA_ARGS__; } break;                      \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("dense: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
__global__ __launch_bounds__(256) void k_act_fwd(const T* __restrict__ x, const T* __restrict__ bias,
                                                 T* __restrict__ y, int64_t M, int N, int act, bool vec) {
  const int64_t total = M * (int64_t)N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < total; i += stride) {
    float v[8];
    if (vec && i + 8 <= total) {
      VecIO<T>::load(x + i, v);
      if (bias) {
        float b[8];
        VecIO<T>::load(bias + (i % N), b);  // N % 8 == 0 on the vector path: 8 columns of one row
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += b[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_f(v[k], act);
      VecIO<T>::store(y + i, v);
    } else {
      for (int k = 0; k < 8 && i + k < total; ++k) {
        float a = to_f<T>(x[i + k]);
        if (bias) a += to_f<T>(bias[(i + k) % N]);
        y[i + k] = from_f<T>(act_f(a, act));
      }
    }
  }
}

BH_DEVICE uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

// counter-based dropout bits: one 32-bit keyed hash per element index, keep iff u >= p. The seed is
// mixed into a key first and enters both rounds non-linearly, so two seeds give unrelated streams
// (XOR-ing a raw seed into the index would make every seed's mask a permutation of the same bits).
BH_DEVICE uint32_t bda_hash(uint32_t seed, uint64_t i) {
  const uint32_t k = fmix32(seed * 0x9E3779B9u + 0x632BE5ABu);
  const uint32_t h = fmix32((uint32_t)i ^ k);
  return fmix32(h + k * 0x85EBCA6Bu + (uint32_t)(i >> 32) * 0xC2B2AE35u);
}

// out = residual + dropout(x + bias) with the keep bits stored 1 per element (uint8 [M*N/8]).
// Vector path only (N % 8 == 0, 16-byte aligned): each lane owns 8 consecutive elements = 1 mask byte.
template <typename T>
__global__ __launch_bounds__(256) void k_bias_dropout_add(const T* __restrict__ x, const T* __restrict__ bias,
                                                          const T* __restrict__ res, T* __restrict__ out,
                                                          uint8_t* __restrict__ keep, int64_t total, int N,
                                                          uint32_t thresh, float scale, uint32_t seed,
                                                          const int64_t* __restrict__ seed_dev) {
  // a device step seed (graph replay) keys the host seed; read once (scalar load)
  if (seed_dev) seed ^= (uint32_t)(((uint64_t)*seed_dev * 0x9E3779B97F4A7C15ull) >> 32);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < total; i += stride) {
    float v[8], r[8];
    VecIO<T>::load(x + i, v);
    VecIO<T>::load(res + i, r);
    if (bias) {
      float b[8];
      VecIO<T>::load(bias + (i % N), b);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k];
    }
    if (keep) {
      uint32_t bits = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool kp = bda_hash(seed, (uint64_t)(i + k)) >= thresh;
        bits |= (uint32_t)kp << k;
        v[k] = kp ? v[k] * scale : 0.f;
      }
      keep[i >> 3] = (uint8_t)bits;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += r[k];
    VecIO<T>::store(out + i, v);
  }
}

// grid (ceil(N / kCols), splits); block (kColLanes, kRowLanes)
template <typename T>
__global__ __launch_bounds__(256) void k_act_bwd(const T* __restrict__ dy, const T* __restrict__ aux,
                                                 T* __restrict__ dx, float* __restrict__ part, int64_t M, int N,
                                                 int64_t rows_per_split, int act, bool vec,
                                                 const uint8_t* __restrict__ keep, float keep_scale) {
  // keep (vec path only): dropout keep bits, byte (off / 8) holds columns col0..col0+7 of a row
  __shared__ float red[kRowLanes][kCols + 4];
  const int col0 = blockIdx.x * kCols + threadIdx.x * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < M ? r0 + rows_per_split : M;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col0 < N) {
    int64_t r = r0 + threadIdx.y;
    if (vec && col0 + 8 <= N && !keep && act == kActNone) {
      // bias gradient only (the common transformer case): four rows of 16-byte loads in flight per lane
      for (; r + 3 * kRowLanes < r1; r += 4 * kRowLanes) {
        float g[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) VecIO<T>::load(dy + (r + u * kRowLanes) * N + col0, g[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += g[u][k];
          if (dx) VecIO<T>::store(dx + (r + u * kRowLanes) * N + col0, g[u]);
        }
      }
    } else if (vec && col0 + 8 <= N && keep && act == kActNone) {
      // dropout backward + bias gradient (Megatron's bias-dropout-add): the same four rows in flight,
      // with their keep bytes (same per-row order of the sums as the one-row loop below)
      for (; r + 3 * kRowLanes < r1; r += 4 * kRowLanes) {
        float g[4][8];
        uint32_t bits[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t off = (r + u * kRowLanes) * N + col0;
          VecIO<T>::load(dy + off, g[u]);
          bits[u] = keep[off >> 3];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            g[u][k] = ((bits[u] >> k) & 1u) ? g[u][k] * keep_scale : 0.f;
            acc[k] += g[u][k];
          }
          if (dx) VecIO<T>::store(dx + (r + u * kRowLanes) * N + col0, g[u]);
        }
      }
    }
    for (; r < r1; r += kRowLanes) {
      const int64_t off = r * N + col0;
      float g[8], a[8];
      if (vec && col0 + 8 <= N) {
        VecIO<T>::load(dy + off, g);
        if (act != kActNone) VecIO<T>::load(aux + off, a);
        if (keep) {
          const uint32_t bits = keep[off >> 3];
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = ((bits >> k) & 1u) ? g[k] * keep_scale : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (act != kActNone) g[k] *= act_d(a[k], act);
          acc[k] += g[k];
        }
        if (dx) VecIO<T>::store(dx + off, g);
      } else {
        for (int k = 0; k < 8 && col0 + k < N; ++k) {
          float gv = to_f<T>(dy[off + k]);
          if (act != kActNone) gv *= act_d(to_f<T>(aux[off + k]), act);
          acc[k] += gv;
          if (dx) dx[off + k] = from_f<T>(gv);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[threadIdx.y][threadIdx.x * 8 + k] = acc[k];
  __syncthreads();
  const int t = threadIdx.y * kColLanes + threadIdx.x;  // 256 threads -> 256 columns
  const int c = blockIdx.x * kCols + t;
  if (c < N) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kRowLanes; ++j) s += red[j][t];
    part[(int64_t)blockIdx.y * N + c] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(64 * kColsumLanes) void k_colsum_finalize(const float* __restrict__ part, int splits, int N,
                                                                        T* __restrict__ out) {
  __shared__ float sh[kColsumLanes][64];
  colsum_partials_block<T>(part, splits, N, out, sh);
}


// ---- embedding weight gradient: deterministic, no host synchronisation (torch's embedding backward
// reads its segment count back to the host every call). Token ids come sorted (stable) with their
// permutation; sorted positions are cut into chunks of kEmbChunk. Pass 1: one workgroup per (chunk,
// column slab) sums each run-piece of equal ids inside its chunk in order and stores the fp32 sum at
// the piece's first position. Pass 2: the first position of every run adds its pieces (the run start,
// then each chunk boundary the run crosses) in order and writes the weight-gradient row. Rows of ids
// that never occur keep the zero fill; padding_idx rows stay zero.
constexpr int kEmbChunk = 32;
constexpr int kEmbCols = 512;  // columns per workgroup: 256 threads x 2

template <typename T>
__global__ __launch_bounds__(256) void k_embed_pieces(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                                                      const T* __restrict__ dy, float* __restrict__ piece, int64_t n,
                                                      int H) {
  const int64_t p0 = (int64_t)blockIdx.x * kEmbChunk;
  const int c = blockIdx.y * kEmbCols + threadIdx.x * 2;
  if (c >= H) return;
  const int64_t pe = min(n, p0 + kEmbChunk);
  float a0 = 0.f, a1 = 0.f;
  int64_t start = p0;
  for (int64_t p = p0; p < pe; ++p) {
    const T* r = dy + perm[p] * (int64_t)H + c;
    a0 += to_f<T>(r[0]);
    if (c + 1 < H) a1 += to_f<T>(r[1]);
    if (p + 1 == pe || sorted[p + 1] != sorted[p]) {
      float* o = piece + start * (int64_t)H + c;
      o[0] = a0;
      if (c + 1 < H) o[1] = a1;
      a0 = a1 = 0.f;
      start = p + 1;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_embed_runs(const int64_t* __restrict__ sorted, const float* __restrict__ piece,
                                                    T* __restrict__ dw, int64_t n, int H, int64_t pad) {
  const int64_t i = blockIdx.x;
  const int64_t id = sorted[i];
  if ((i > 0 && sorted[i - 1] == id) || id == pad) return;
  const int c = blockIdx.y * kEmbCols + threadIdx.x * 2;
  if (c >= H) return;
  float a0 = piece[i * H + c], a1 = c + 1 < H ? piece[i * H + c + 1] : 0.f;
  for (int64_t j = (i / kEmbChunk + 1) * kEmbChunk; j < n && sorted[j] == id; j += kEmbChunk) {
    a0 += piece[j * H + c];
    if (c + 1 < H) a1 += piece[j * H + c + 1];
  }
  dw[id * H + c] = from_f<T>(a0);
  if (c + 1 < H) dw[id * H + c + 1] = from_f<T>(a1);
}

}  // namespace

void dense_act_forward(int dt, const void* x, const void* bias, void* y, int64_t M, int N, int act, bool vec,
                       hipStream_t st) {
  const int64_t total = M * (int64_t)N;
  if (total == 0) return;
  int64_t blocks = (total / 8 + 255) / 256 + 1;
  if (blocks > 8192) blocks = 8192;
  DN_DISPATCH(dt, T, hipLaunchKernelGGL((k_act_fwd<T>), dim3((unsigned)blocks), dim3(256), 0, st, (const T*)x,
                                        (const T*)bias, (T*)y, M, N, act, vec));
  check_launch("dense_act_forward");
}

int dense_bgrad_splits(int64_t M, int N) {
  const int64_t col_blocks = (N + kCols - 1) / kCols;
  int64_t splits = (2048 + col_blocks - 1) / col_blocks;       // aim for ~2048 workgroups
  // >= 64 rows per split (the 4-row unrolled loops need 32 rows per pass of the 8 row lanes)
  const int64_t max_splits = (M + 63) / 64;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  if (splits > 1024) splits = 1024;
  return (int)splits;
}

void dense_act_backward(int dt, const void* dy, const void* aux, void* dx, void* bgrad, float* part, int splits,
                        int64_t M, int N, int act, bool vec, hipStream_t st) {
  if (N == 0) return;
  const int64_t rps = M > 0 ? (M + splits - 1) / splits : 1;
  dim3 grid((unsigned)((N + kCols - 1) / kCols), (unsigned)splits);
  DN_DISPATCH(dt, T,
      hipLaunchKernelGGL((k_act_bwd<T>), grid, dim3(kColLanes, kRowLanes), 0, st, (const T*)dy, (const T*)aux,
                         (T*)dx, part, M, N, rps, act, vec, (const uint8_t*)nullptr, 1.f);
      check_launch("dense_act_backward");
      if (bgrad) {
        hipLaunchKernelGGL((k_colsum_finalize<T>), dim3((unsigned)((N + 63) / 64)), dim3(64 * kColsumLanes), 0, st,
                           part, splits, N, (T*)bgrad);
        check_launch("dense_bgrad_finalize");
      });
}

void dense_bias_dropout_add(int dt, const void* x, const void* bias, const void* residual, void* out, uint8_t* keep,
                            int64_t M, int N, float p, uint32_t seed, hipStream_t st, const int64_t* seed_dev) {
  const int64_t total = M * (int64_t)N;
  if (total == 0) return;
  if (N % 8 != 0) throw std::runtime_error("dense_bias_dropout_add: N % 8 != 0");
  int64_t blocks = (total / 8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  // keep iff hash >= p * 2^32 (p < 1 is checked by the caller)
  const uint32_t thresh = (uint32_t)((double)p * 4294967296.0);
  const float scale = keep ? 1.f / (1.f - p) : 1.f;
  DN_DISPATCH(dt, T, hipLaunchKernelGGL((k_bias_dropout_add<T>), dim3((unsigned)blocks), dim3(256), 0, st,
                                        (const T*)x, (const T*)bias, (const T*)residual, (T*)out, keep, total, N,
                                        thresh, scale, seed, seed_dev));
  check_launch("dense_bias_dropout_add");
}

void dense_dropout_backward(int dt, const void* dy, const uint8_t* keep, float keep_scale, void* dx, void* bgrad,
                            float* part, int splits, int64_t M, int N, hipStream_t st) {
  if (N == 0) return;
  if (N % 8 != 0) throw std::runtime_error("dense_dropout_backward: N % 8 != 0");
  const int64_t rps = M > 0 ? (M + splits - 1) / splits : 1;
  dim3 grid((unsigned)((N + kCols - 1) / kCols), (unsigned)splits);
  DN_DISPATCH(dt, T,
      hipLaunchKernelGGL((k_act_bwd<T>), grid, dim3(kColLanes, kRowLanes), 0, st, (const T*)dy, (const T*)nullptr,
                         (T*)dx, part, M, N, rps, (int)kActNone, true, keep, keep_scale);
      check_launch("dense_dropout_backward");
      if (bgrad) {
        hipLaunchKernelGGL((k_colsum_finalize<T>), dim3((unsigned)((N + 63) / 64)), dim3(64 * kColsumLanes), 0, st,
                           part, splits, N, (T*)bgrad);
        check_launch("dense_dropout_bgrad_finalize");
      });
}

void embedding_backward(int dt, const int64_t* sorted, const int64_t* perm, const void* dy, float* piece, void* dw,
                        int64_t n, int H, int64_t padding_idx, hipStream_t st) {
  if (n <= 0) return;
  const unsigned slabs = (unsigned)((H + kEmbCols - 1) / kEmbCols);
  DN_DISPATCH(dt, T, {
    hipLaunchKernelGGL((k_embed_pieces<T>), dim3((unsigned)((n + kEmbChunk - 1) / kEmbChunk), slabs), dim3(256), 0,
                       st, sorted, perm, (const T*)dy, piece, n, H);
    hipLaunchKernelGGL((k_embed_runs<T>), dim3((unsigned)n, slabs), dim3(256), 0, st, sorted, piece, (T*)dw, n, H,
                       padding_idx);
  });
  check_launch("embedding_backward");
}

}  // namespace bh
