// Peer-memory 1-D halo exchange for gfx950 (the `peer_memory_cuda` push/pull kernel).
//
// Reference behaviour: apex/contrib/csrc/peer_memory/peer_memory_cuda.cu:359-408 (push_pull_halos_1d,
// a cooperative kernel with magic-value flags that it clears after every use) and :653-741.
//
// MI355X design:
//  * no grid-wide barrier and no cooperative launch: workgroup b of the sender and workgroup b of the
//    receiver own the same element range, so each receiver workgroup waits only for ITS sender
//    workgroup's flag (one flag per workgroup per direction);
//  * monotonically increasing epochs instead of magic values + clearing (no clear/set race), and the
//    transfer buffers are double-buffered by epoch parity, so a rank may start the next exchange
//    while its neighbour is still pulling the previous one;
//  * flag publication is a system-scope release store into the neighbour's memory (xGMI), polling is a
//    system-scope acquire load with s_sleep back-off; every wait is bounded (*err reports a timeout),
//    so no workgroup can spin forever if a peer never arrives;
//  * all stores are ordinary vector stores / vector atomics.
#include "bh/device.h"
#include "bh/peer_api.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

BH_DEVICE int64_t view_offset(const HaloView& v, int64_t i) {
  // views arrive with mergeable dimensions collapsed on the host (an NHWC row halo is [1, 1, N, W*C]),
  // so the leading divisions usually see size-1 dimensions
  const int64_t i3 = i % v.size[3];
  int64_t r = i / v.size[3];
  int64_t o = i3 * v.stride[3];
  if (v.size[2] > 1) {
    o += (r % v.size[2]) * v.stride[2];
    r /= v.size[2];
  }
  if (v.size[1] > 1) {
    o += (r % v.size[1]) * v.stride[1];
    r /= v.size[1];
  }
  return o + r * v.stride[0];
}

// copy elements [lo, hi) of a halo; with a.vec16 every view is innermost-contiguous, its innermost
// size and all strides are multiples of 16 bytes and the range bounds are too, so whole 16-byte
// pieces move (one offset computation per 8 fp16 elements instead of per element)
template <typename E>
BH_DEVICE void copy_range(E* dst, const HaloView* dview, const E* src, const HaloView* sview, int64_t lo, int64_t hi,
                          bool vec16) {
  if (vec16) {
    constexpr int V = 16 / sizeof(E);
    for (int64_t i = lo + (int64_t)threadIdx.x * V; i < hi; i += (int64_t)kBlock * V) {
      const uint4 x = *reinterpret_cast<const uint4*>(sview ? src + view_offset(*sview, i) : src + i);
      *reinterpret_cast<uint4*>(dview ? dst + view_offset(*dview, i) : dst + i) = x;
    }
    return;
  }
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const E x = sview ? src[view_offset(*sview, i)] : src[i];
    if (dview) dst[view_offset(*dview, i)] = x;
    else dst[i] = x;
  }
}

// a timed-out pull leaves NaN (all bits set: NaN in fp16, bf16 and fp32) instead of stale data, so a
// missing neighbour poisons the result visibly (the device loss scaler then skips the step)
template <typename E>
BH_DEVICE void poison_range(E* dst, const HaloView& v, int64_t lo, int64_t hi) {
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) dst[view_offset(v, i)] = static_cast<E>(~E(0));
}

BH_DEVICE bool wait_epoch(int* flag, int epoch, int max_spins) {
  for (int s = 0; s < max_spins; ++s) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) return true;
    __builtin_amdgcn_s_sleep(8);
  }
  return false;
}

template <typename E>
__global__ __launch_bounds__(kBlock) void k_halo_1d(HaloArgs a) {
  const int b = blockIdx.x;
  // per-workgroup ranges are multiples of 16 bytes when the vector path is on
  const int64_t gran = a.vec16 ? 16 / sizeof(E) : 1;
  const int64_t per = ((a.numel + gridDim.x - 1) / gridDim.x + gran - 1) / gran * gran;
  const int64_t lo = min(a.numel, (int64_t)b * per), hi = min(a.numel, lo + per);
  const int slot = a.epoch & 1;
  E* tx_lo = reinterpret_cast<E*>(a.tx_lo_self) + slot * a.numel;
  E* tx_hi = reinterpret_cast<E*>(a.tx_hi_self) + slot * a.numel;
  // 1. stage the outgoing halos in this rank's transfer slots (local memory)
  if (!a.lo_zero) copy_range<E>(tx_lo, nullptr, reinterpret_cast<const E*>(a.out_lo.ptr), &a.out_lo, lo, hi, a.vec16);
  if (!a.hi_zero) copy_range<E>(tx_hi, nullptr, reinterpret_cast<const E*>(a.out_hi.ptr), &a.out_hi, lo, hi, a.vec16);
  __syncthreads();
  // 2. publish: my low halo is what the low neighbour pulls as its HIGH input (its flag row 1)
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // staged data visible before the flag
    if (!a.lo_zero)
      __hip_atomic_store(a.flags_peer_lo + kPeerMaxBlocks + b, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!a.hi_zero) __hip_atomic_store(a.flags_peer_hi + b, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for the neighbours' slots of this epoch, then pull them
  __shared__ int ok[2];
  if (threadIdx.x == 0) {
    ok[0] = a.lo_zero ? 1 : (int)wait_epoch(a.flags_self + b, a.epoch, a.max_spins);
    ok[1] = a.hi_zero ? 1 : (int)wait_epoch(a.flags_self + kPeerMaxBlocks + b, a.epoch, a.max_spins);
    if (!ok[0] || !ok[1]) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  E* in_lo = reinterpret_cast<E*>(a.in_lo.ptr);
  E* in_hi = reinterpret_cast<E*>(a.in_hi.ptr);
  if (a.lo_zero) {
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) in_lo[view_offset(a.in_lo, i)] = E(0);
  } else if (ok[0]) {
    copy_range<E>(in_lo, &a.in_lo, reinterpret_cast<const E*>(a.tx_peer_lo) + slot * a.numel, nullptr, lo, hi, a.vec16);
  } else {
    poison_range<E>(in_lo, a.in_lo, lo, hi);
  }
  if (a.hi_zero) {
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) in_hi[view_offset(a.in_hi, i)] = E(0);
  } else if (ok[1]) {
    copy_range<E>(in_hi, &a.in_hi, reinterpret_cast<const E*>(a.tx_peer_hi) + slot * a.numel, nullptr, lo, hi, a.vec16);
  } else {
    poison_range<E>(in_hi, a.in_hi, lo, hi);
  }
}

constexpr int kReduceBlock = 512;

__global__ __launch_bounds__(kReduceBlock) void k_peer_allreduce(PeerReduceArgs a) {
  __shared__ int ep;
  if (threadIdx.x == 0) ep = a.epoch_dev ? a.epoch_dev[0] + 1 : a.epoch;
  __syncthreads();
  const int epoch = ep;
  const int parity = epoch & 1;
  // 1. push: my payload into row `me` of every rank's slot array (vector stores over xGMI)
  for (int q = 0; q < a.G; ++q) {
    float* dst = a.slots[q] + ((int64_t)parity * a.G + a.me) * a.L;
    for (int i = threadIdx.x; i < a.L; i += kReduceBlock) dst[i] = a.in[i];
  }
  __syncthreads();
  // 2. publish: the rows are visible system-wide before any flag is
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    for (int q = 0; q < a.G; ++q)
      if (q != a.me) __hip_atomic_store(a.flags[q] + a.me, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. one lane per peer waits (bounded) for that peer's rows of this epoch
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  const int q = threadIdx.x;
  if (q < a.G && q != a.me && !wait_epoch(a.flags[a.me] + q, epoch, a.max_spins)) {
    ok = 0;
    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  // 4. sum the G rows in rank order (identical on every rank). A timed-out exchange writes NaN: never
  //    rank-local statistics that silently differ between ranks (the host also raises on *err)
  const float* rows = a.slots[a.me] + (int64_t)parity * a.G * a.L;
  for (int i = threadIdx.x; i < a.L; i += kReduceBlock) {
    float s = __builtin_nanf("");
    if (ok) {
      s = 0.f;
      for (int r = 0; r < a.G; ++r) s += rows[(int64_t)r * a.L + i];
    }
    a.out[i] = s;
  }
  if (a.epoch_dev && threadIdx.x == 0) a.epoch_dev[0] = epoch;  // (read above, before the barrier)
}

}  // namespace

void peer_allreduce(const PeerReduceArgs& a, hipStream_t st) {
  if (a.L <= 0) return;
  if (a.G < 1 || a.G > kPeerMaxRanks || a.me < 0 || a.me >= a.G)
    throw std::runtime_error("peer_allreduce: bad group geometry");
  hipLaunchKernelGGL(k_peer_allreduce, dim3(1), dim3(kReduceBlock), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("peer_allreduce: ") + hipGetErrorString(e));
}

void push_pull_halos_1d(const HaloArgs& a, hipStream_t st) {
  if (a.numel == 0) return;
  const int64_t want = (a.numel + 4 * kBlock - 1) / (4 * kBlock);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, kPeerMaxBlocks));
  if (a.elem_bytes == 2) {
    hipLaunchKernelGGL((k_halo_1d<uint16_t>), dim3(grid), dim3(kBlock), 0, st, a);
  } else if (a.elem_bytes == 4) {
    hipLaunchKernelGGL((k_halo_1d<uint32_t>), dim3(grid), dim3(kBlock), 0, st, a);
  } else {
    throw std::runtime_error("push_pull_halos_1d: element size must be 2 or 4 bytes");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("push_pull_halos_1d: ") + hipGetErrorString(e));
}

}  // namespace bh
