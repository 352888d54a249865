// Peer-memory halo exchange launcher (kernels/peer_memory.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

constexpr int kPeerMaxBlocks = 64;  // flag slots per direction

// A strided 4-D view (elements) of a halo slice.
struct HaloView {
  void* ptr;
  int64_t size[4];
  int64_t stride[4];
};

// One 1-D halo exchange step between this rank and its low / high neighbours (pull protocol):
//   every workgroup b copies its part of the outgoing halos into this rank's transfer buffers
//   (slot epoch % 2), publishes `epoch` in the neighbour's flag array (release, system scope), waits
//   (acquire, bounded) until the neighbour published the same epoch in ours, then pulls the
//   neighbour's transfer slot into the incoming halo. lo_zero / hi_zero: no neighbour on that side
//   -> the incoming halo is zero-filled. Flags: int32 [2][kPeerMaxBlocks], row 0 written by the low
//   neighbour, row 1 by the high neighbour. A wait that exceeds `max_spins` polls sets *err = 1 and
//   skips the copy (no workgroup can hang).
struct HaloArgs {
  HaloView out_lo, out_hi, in_lo, in_hi;
  void* tx_lo_self;   // [2][numel] this rank's low-side transfer slots
  void* tx_hi_self;
  const void* tx_peer_lo;  // low neighbour's HIGH transfer slots (peer pointer)
  const void* tx_peer_hi;  // high neighbour's LOW transfer slots (peer pointer)
  int* flags_self;         // [2][kPeerMaxBlocks]
  int* flags_peer_lo;      // low neighbour's flag array (peer pointer)
  int* flags_peer_hi;      // high neighbour's flag array (peer pointer)
  bool lo_zero, hi_zero;
  int epoch;
  int64_t numel;           // elements of one halo
  int elem_bytes;          // 2 or 4
  int max_spins;
  bool vec16;              // every view copies in 16-byte pieces (set by the host, see k_halo_1d)
  int* err;
};
void push_pull_halos_1d(const HaloArgs& a, hipStream_t st);

// One-shot SUM all-reduce of a small fp32 vector over the G ranks of a peer-memory pool (the IPC path
// of group batch norm; reference: apex/contrib/csrc/groupbn/ipc.cu:22-129 + the peer exchange inside
// nhwc_batch_norm_kernel.h). Every rank pushes its payload into row `me` of every peer's slot array
// (parity epoch % 2: [2][G][L] floats in each rank's pool), publishes `epoch` in each peer's flag
// array (flags[me], release, system scope), waits (bounded) until all G-1 peers published the same
// epoch in its own flags, then sums its G local rows in rank order -- the same order on every rank,
// so all ranks get bitwise-identical results. out may alias in.
constexpr int kPeerMaxRanks = 8;
struct PeerReduceArgs {
  const float* in;
  float* out;
  float* slots[kPeerMaxRanks];  // slot array of each rank (peer pointers; own at index me)
  int* flags[kPeerMaxRanks];    // int32 [G] flag array of each rank
  int G, me, L, epoch, max_spins;
  int* err;
  // device-resident epoch counter (int32 [1]); when set, the kernel takes epoch = *epoch_dev + 1 and stores it
  // back, so a captured HIP graph replays with a fresh epoch each time (the host epoch is ignored)
  int* epoch_dev = nullptr;
};
void peer_allreduce(const PeerReduceArgs& a, hipStream_t st);

}  // namespace bh
