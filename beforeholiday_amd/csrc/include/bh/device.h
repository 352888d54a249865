// Device foundation for every beforeholiday_amd HIP kernel (gfx950 / CDNA4 only).
//
// What lives here (replacing the reference's csrc/type_shim.h reductions and the
// per-kernel ILP load/store helpers):
//   * element types: f32, f16 (_Float16), bf16 (__bf16), f64 with float conversion
//   * 16-byte vector load/store of 8 (16-bit) / 4 (fp32) elements into float registers
//   * wave64 reductions (sum / max / Welford) and block reductions staged through LDS
//   * Philox4x32-10 counter RNG for dropout-style kernels
//
// Everything is written for a 64-lane wavefront. No CUDA/hipify compatibility paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define BH_DEVICE __device__ __forceinline__
#define BH_HD __host__ __device__ __forceinline__

namespace bh {

constexpr int kWave = 64;

// ----------------------------------------------------------------------------------
// element types
// ----------------------------------------------------------------------------------
using f16 = _Float16;
using bf16 = __bf16;

template <typename T> BH_DEVICE float to_f(T x) { return static_cast<float>(x); }
template <> BH_DEVICE float to_f<float>(float x) { return x; }
template <> BH_DEVICE float to_f<double>(double x) { return static_cast<float>(x); }

template <typename T> BH_DEVICE T from_f(float x) { return static_cast<T>(x); }
template <> BH_DEVICE float from_f<float>(float x) { return x; }

// "accumulate" type: double for double, float otherwise
template <typename T> struct Acc { using type = float; };
template <> struct Acc<double> { using type = double; };

// ----------------------------------------------------------------------------------
// 16-byte vector I/O. kVec<T> elements move in one 16B access for 16-bit types and
// two 16B accesses for fp32 (8 elements per thread either way keeps the per-thread
// loop shape identical across dtypes).
// ----------------------------------------------------------------------------------
constexpr int kVec = 8;

template <typename T> struct VecIO;

template <> struct VecIO<float> {
  static BH_DEVICE void load(const float* p, float (&r)[kVec]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
    r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  }
  static BH_DEVICE void store(float* p, const float (&r)[kVec]) {
    *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(r[4], r[5], r[6], r[7]);
  }
};

template <typename H> struct VecIO16 {
  typedef H h8 __attribute__((ext_vector_type(8)));
  static BH_DEVICE void load(const H* p, float (&r)[kVec]) {
    const h8 v = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < kVec; ++i) r[i] = static_cast<float>(v[i]);
  }
  static BH_DEVICE void store(H* p, const float (&r)[kVec]) {
    h8 v;
#pragma unroll
    for (int i = 0; i < kVec; ++i) v[i] = static_cast<H>(r[i]);
    *reinterpret_cast<h8*>(p) = v;
  }
};
template <> struct VecIO<f16> : VecIO16<f16> {};
template <> struct VecIO<bf16> : VecIO16<bf16> {};

template <> struct VecIO<double> {
  static BH_DEVICE void load(const double* p, float (&r)[kVec]) {
#pragma unroll
    for (int i = 0; i < kVec; i += 2) {
      const double2 v = *reinterpret_cast<const double2*>(p + i);
      r[i] = static_cast<float>(v.x);
      r[i + 1] = static_cast<float>(v.y);
    }
  }
  static BH_DEVICE void store(double* p, const float (&r)[kVec]) {
#pragma unroll
    for (int i = 0; i < kVec; i += 2)
      *reinterpret_cast<double2*>(p + i) = make_double2(r[i], r[i + 1]);
  }
};

// Load kVec elements starting at element i of a tensor of n elements. The vector path
// is taken when `aligned` (all base pointers 16-byte aligned, chunk offsets are multiples
// of kVec) and the whole vector is in range; otherwise a guarded scalar path.
template <typename T>
BH_DEVICE void load_vec(const T* p, int64_t i, int64_t n, bool aligned, float (&r)[kVec]) {
  if (aligned && i + kVec <= n) {
    VecIO<T>::load(p + i, r);
  } else {
#pragma unroll
    for (int k = 0; k < kVec; ++k) r[k] = (i + k < n) ? to_f<T>(p[i + k]) : 0.f;
  }
}
template <typename T>
BH_DEVICE void store_vec(T* p, int64_t i, int64_t n, bool aligned, const float (&r)[kVec]) {
  if (aligned && i + kVec <= n) {
    VecIO<T>::store(p + i, r);
  } else {
#pragma unroll
    for (int k = 0; k < kVec; ++k)
      if (i + k < n) p[i + k] = from_f<T>(r[k]);
  }
}

// ----------------------------------------------------------------------------------
// wave64 / block reductions
// ----------------------------------------------------------------------------------
BH_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
BH_DEVICE double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
BH_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
// Reduction over the low `width` lanes-groups (width a power of two <= 64): every group
// of `width` consecutive lanes reduces independently.
template <int W> BH_DEVICE float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
template <int W> BH_DEVICE float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum; `smem` needs blockDim.x/64 floats. Result is valid in every thread.
BH_DEVICE float block_sum(float v, float* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  v = wave_sum(v);
  __syncthreads();  // protect smem reuse across consecutive calls
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < nw; ++w) r += smem[w];
  return r;
}
BH_DEVICE double block_sum(double v, double* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  double r = 0.0;
  for (int w = 0; w < nw; ++w) r += smem[w];
  return r;
}
BH_DEVICE float block_max(float v, float* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int w = 0; w < nw; ++w) r = fmaxf(r, smem[w]);
  return r;
}

// ----------------------------------------------------------------------------------
// Welford (count, mean, M2) merge — Chan et al. parallel combination.
// ----------------------------------------------------------------------------------
struct Welford {
  float n, mean, m2;
};
BH_DEVICE Welford welford_merge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.mean - a.mean;
  const float wb = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * wb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * wb;
  return r;
}
BH_DEVICE Welford wave_welford(Welford w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Welford b;
    b.n = __shfl_xor(w.n, o, kWave);
    b.mean = __shfl_xor(w.mean, o, kWave);
    b.m2 = __shfl_xor(w.m2, o, kWave);
    w = welford_merge(w, b);
  }
  return w;
}
// smem: 3 * (blockDim.x / 64) floats
BH_DEVICE Welford block_welford(Welford w, float* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  w = wave_welford(w);
  __syncthreads();
  if (lane == 0) {
    smem[wid] = w.n;
    smem[nw + wid] = w.mean;
    smem[2 * nw + wid] = w.m2;
  }
  __syncthreads();
  Welford r{0.f, 0.f, 0.f};
  for (int k = 0; k < nw; ++k) r = welford_merge(r, Welford{smem[k], smem[nw + k], smem[2 * nw + k]});
  return r;
}

// ----------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011), counter-based: (seed, offset, subsequence).
// ----------------------------------------------------------------------------------
struct Philox {
  uint4 ctr;
  uint2 key;
  BH_DEVICE Philox(uint64_t seed, uint64_t subseq, uint64_t offset) {
    key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    ctr = make_uint4((uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)subseq,
                     (uint32_t)(subseq >> 32));
  }
  static BH_DEVICE uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }
  BH_DEVICE uint4 next() {
    uint4 c = ctr;
    uint2 k = key;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint32_t hi0 = mulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
      const uint32_t hi1 = mulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
      c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    // advance the 128-bit counter
    if (++ctr.x == 0) if (++ctr.y == 0) if (++ctr.z == 0) ++ctr.w;
    return c;
  }
  // 4 uniforms in (0, 1]
  BH_DEVICE float4 uniform4() {
    const uint4 r = next();
    constexpr float s = 2.3283064365386963e-10f;  // 2^-32
    return make_float4((r.x + 1.0f) * s, (r.y + 1.0f) * s, (r.z + 1.0f) * s, (r.w + 1.0f) * s);
  }
};

BH_DEVICE bool is_finite(float x) { return __builtin_isfinite(x); }


// Column sums of fp32 split partials part[slabs][N] -> out[N] (optionally scaled), for a block of
// 64 columns x kColsumLanes split-lanes (blockDim 64 * kColsumLanes, grid ceil(N / 64)). Each lane
// keeps 8 independent loads in flight; lanes merge through LDS. Replaces one-thread-per-column loops
// that walk all slabs serially (latency-bound: 20-40 us for a 2 MB partial buffer).
constexpr int kColsumLanes = 16;
template <typename T>
BH_DEVICE void colsum_partials_block(const float* __restrict__ part, int64_t slabs, int64_t N, T* __restrict__ out,
                                     float (&sh)[kColsumLanes][64]) {
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  float acc = 0.f;
  if (c < N) {
    int64_t s = lane;
    for (; s + 7 * kColsumLanes < slabs; s += 8 * kColsumLanes) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(s + u * kColsumLanes) * N + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < slabs; s += kColsumLanes) acc += part[s * N + c];
  }
  sh[lane][cl] = acc;
  __syncthreads();
  if (lane == 0 && c < N && out) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < kColsumLanes; ++l) t += sh[l][cl];
    out[c] = from_f<T>(t);
  }
  __syncthreads();
}

}  // namespace bh
