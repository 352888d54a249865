// `peer_memory_cuda` front-end: a raw device pool shared with the other ranks of the node through HIP
// IPC handles (dmabuf-backed on this driver), strided tensor views over pool addresses, and the 1-D
// halo exchange kernel (kernels/peer_memory.hip). Reference API:
// apex/contrib/csrc/peer_memory/peer_memory.cpp:20-28.
#include "common.h"

#include <cstring>
#include <mutex>
#include <set>

#include "bh/peer_api.h"

namespace bhb {
namespace {

std::mutex g_peer_mu;
auto& g_opened = *new std::set<int64_t>();  // peer mappings opened by this process (never destroyed at exit)

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

int64_t allocate_raw(int64_t size) {
  TORCH_CHECK(size > 0, "allocate_raw: size must be positive");
  void* p = nullptr;
  hip_check(hipMalloc(&p, (size_t)size), "allocate_raw (hipMalloc)");
  hip_check(hipMemset(p, 0, (size_t)size), "allocate_raw (hipMemset)");
  return reinterpret_cast<int64_t>(p);
}

void free_raw(int64_t raw) {
  hip_check(hipDeviceSynchronize(), "free_raw (synchronize)");
  hip_check(hipFree(reinterpret_cast<void*>(raw)), "free_raw (hipFree)");
}

void zero(int64_t raw, int64_t size) {
  hip_check(hipMemsetAsync(reinterpret_cast<void*>(raw), 0, (size_t)size,
                           c10::hip::getCurrentHIPStream().stream()), "zero (hipMemsetAsync)");
}

at::Tensor get_raw_ipc_address(int64_t raw) {
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(raw)), "get_raw_ipc_address (hipIpcGetMemHandle)");
  auto t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr<uint8_t>(), &h, sizeof(h));
  return t;
}

// ipc_addresses: uint8 [n, sizeof(handle)] (CPU) of the peer group; returns one device address per peer
// (this rank's own raw pointer at peer_rank, opened IPC mappings elsewhere)
std::vector<int64_t> get_raw_peers(at::Tensor ipc_addresses, int64_t peer_rank, int64_t raw) {
  ipc_addresses = ipc_addresses.to(at::kCPU).contiguous();
  TORCH_CHECK(ipc_addresses.dim() == 2 && ipc_addresses.scalar_type() == at::kByte &&
                  ipc_addresses.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "get_raw_peers: expected uint8 [n, ", sizeof(hipIpcMemHandle_t), "] handles");
  const int64_t n = ipc_addresses.size(0);
  std::vector<int64_t> out(n);
  for (int64_t i = 0; i < n; ++i) {
    if (i == peer_rank) {
      out[i] = raw;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, ipc_addresses.data_ptr<uint8_t>() + i * sizeof(h), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "get_raw_peers (hipIpcOpenMemHandle)");
    out[i] = reinterpret_cast<int64_t>(p);
    std::lock_guard<std::mutex> lock(g_peer_mu);
    g_opened.insert(out[i]);
  }
  return out;
}

void close_raw_peers(std::vector<int64_t> peers) {
  hip_check(hipDeviceSynchronize(), "close_raw_peers (synchronize)");
  std::lock_guard<std::mutex> lock(g_peer_mu);
  for (int64_t p : peers) {
    if (g_opened.erase(p)) hip_check(hipIpcCloseMemHandle(reinterpret_cast<void*>(p)), "hipIpcCloseMemHandle");
  }
}

at::Tensor blob_view(int64_t raw, std::vector<int64_t> shape, bool channels_last, at::ScalarType dt) {
  auto opts = at::TensorOptions().dtype(dt).device(at::kCUDA, c10::hip::current_device());
  std::vector<int64_t> strides(shape.size());
  if (channels_last && shape.size() == 4) {
    const int64_t C = shape[1], H = shape[2], W = shape[3];
    strides = {H * W * C, 1, W * C, C};
  } else {
    int64_t s = 1;
    for (int64_t d = (int64_t)shape.size() - 1; d >= 0; --d) {
      strides[d] = s;
      s *= shape[d];
    }
  }
  return at::from_blob(reinterpret_cast<void*>(raw), shape, strides, [](void*) {}, opts);
}

// 4-D view with mergeable dimensions collapsed (row-major order kept): [N, 1, W, C] rows of an NHWC
// tensor become [1, 1, N, W*C], so the kernel's offset math mostly sees size-1 dimensions
bh::HaloView halo_view(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, "halo tensors must be 4-D GPU tensors");
  int64_t sz[4], st[4];
  int n = 0;
  for (int d = 0; d < 4; ++d) {
    if (t.size(d) == 1) continue;
    if (n > 0 && st[n - 1] == t.size(d) * t.stride(d)) {
      sz[n - 1] *= t.size(d);
      st[n - 1] = t.stride(d);
    } else {
      sz[n] = t.size(d);
      st[n] = t.stride(d);
      ++n;
    }
  }
  bh::HaloView v{};
  v.ptr = t.data_ptr();
  for (int d = 0; d < 4; ++d) {
    const int k = d - (4 - n);  // right-aligned, leading size-1 dimensions
    v.size[d] = k >= 0 ? sz[k] : 1;
    v.stride[d] = k >= 0 ? st[k] : 0;
  }
  return v;
}

bool view_vec16(const bh::HaloView& v, int eb) {
  const int64_t V = 16 / eb;
  if ((reinterpret_cast<uintptr_t>(v.ptr) & 15) != 0 || v.size[3] % V != 0 || (v.size[3] > 1 && v.stride[3] != 1))
    return false;
  for (int d = 0; d < 3; ++d)
    if (v.size[d] > 1 && v.stride[d] % V != 0) return false;
  return true;
}

// Halo exchange step (see bh/peer_api.h). tx_* are [2, numel] transfer-slot tensors in the pool;
// flags are int32 [2, 64] pool tensors. Returns nothing; err (GPU int32 [1]) is set on a timeout.
void push_pull_halos_1d(at::Tensor out_lo, at::Tensor out_hi, at::Tensor in_lo, at::Tensor in_hi, at::Tensor tx_lo_self,
                        at::Tensor tx_hi_self, at::Tensor tx_peer_lo, at::Tensor tx_peer_hi, at::Tensor flags_self,
                        at::Tensor flags_peer_lo, at::Tensor flags_peer_hi, bool lo_zero, bool hi_zero, int64_t epoch,
                        at::Tensor err, int64_t max_spins) {
  TORCH_CHECK(out_lo.sizes() == out_hi.sizes() && out_lo.sizes() == in_lo.sizes() && in_lo.sizes() == in_hi.sizes(),
              "push_pull_halos_1d: all halo views must have the same shape");
  const int64_t n = out_lo.numel();
  const int eb = (int)out_lo.element_size();
  for (const at::Tensor* t : {&tx_lo_self, &tx_hi_self, &tx_peer_lo, &tx_peer_hi})
    TORCH_CHECK(t->numel() >= 2 * n && t->element_size() == eb, "push_pull_halos_1d: transfer slots must be [2, numel]");
  for (const at::Tensor* t : {&flags_self, &flags_peer_lo, &flags_peer_hi})
    TORCH_CHECK(t->scalar_type() == at::kInt && t->numel() >= 2 * bh::kPeerMaxBlocks, "flags must be int32 [2, 64]");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "err must be a GPU int32 tensor");
  TORCH_CHECK(epoch > 0 && epoch < (1ll << 30), "epoch must be in [1, 2^30)");
  bh::HaloArgs a{};
  a.out_lo = halo_view(out_lo);
  a.out_hi = halo_view(out_hi);
  a.in_lo = halo_view(in_lo);
  a.in_hi = halo_view(in_hi);
  a.tx_lo_self = tx_lo_self.data_ptr();
  a.tx_hi_self = tx_hi_self.data_ptr();
  a.tx_peer_lo = tx_peer_lo.data_ptr();
  a.tx_peer_hi = tx_peer_hi.data_ptr();
  a.flags_self = flags_self.data_ptr<int>();
  a.flags_peer_lo = flags_peer_lo.data_ptr<int>();
  a.flags_peer_hi = flags_peer_hi.data_ptr<int>();
  a.lo_zero = lo_zero;
  a.hi_zero = hi_zero;
  a.epoch = (int)epoch;
  a.numel = n;
  a.elem_bytes = eb;
  a.max_spins = (int)max_spins;
  a.err = err.data_ptr<int>();
  a.vec16 = view_vec16(a.out_lo, eb) && view_vec16(a.out_hi, eb) && view_vec16(a.in_lo, eb) &&
            view_vec16(a.in_hi, eb);
  for (const at::Tensor* t : {&tx_lo_self, &tx_hi_self, &tx_peer_lo, &tx_peer_hi})
    a.vec16 = a.vec16 && (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0;
  bh::push_pull_halos_1d(a, stream_for(out_lo));
}

// SUM all-reduce of the fp32 vector `in` (into `out`, may alias) over the pool's ranks: slots[q] /
// flags[q] are the device addresses of rank q's [2, G, capacity] slot array and int32 [G] flags.
void peer_allreduce(at::Tensor in, at::Tensor out, std::vector<int64_t> slots, std::vector<int64_t> flags,
                    int64_t capacity, int64_t me, int64_t epoch, at::Tensor err, int64_t max_spins,
                    c10::optional<at::Tensor> epoch_dev) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kFloat && in.is_contiguous(), "in must be contiguous fp32 GPU");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == in.numel(),
              "out must match in");
  TORCH_CHECK(slots.size() == flags.size() && !slots.empty() && slots.size() <= (size_t)bh::kPeerMaxRanks,
              "peer_allreduce: 1..8 ranks");
  TORCH_CHECK(in.numel() <= capacity, "peer_allreduce: payload of ", in.numel(), " floats exceeds the slot capacity ",
              capacity);
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "err must be a GPU int32 tensor");
  TORCH_CHECK(epoch > 0 && epoch < (1ll << 30), "epoch must be in [1, 2^30)");
  bh::PeerReduceArgs a{};
  a.in = in.data_ptr<float>();
  a.out = out.data_ptr<float>();
  a.G = (int)slots.size();
  for (int q = 0; q < a.G; ++q) {
    a.slots[q] = reinterpret_cast<float*>(slots[q]);
    a.flags[q] = reinterpret_cast<int*>(flags[q]);
  }
  a.me = (int)me;
  a.L = (int)in.numel();
  a.epoch = (int)epoch;
  a.max_spins = (int)max_spins;
  a.err = err.data_ptr<int>();
  if (epoch_dev.has_value() && epoch_dev->defined()) {
    TORCH_CHECK(epoch_dev->is_cuda() && epoch_dev->scalar_type() == at::kInt && epoch_dev->numel() == 1,
                "epoch_dev must be a GPU int32 [1] tensor");
    a.epoch_dev = epoch_dev->data_ptr<int>();
  }
  bh::peer_allreduce(a, stream_for(in));
}

}  // namespace

void register_peer_memory(pybind11::module_& root) {
  auto m = root.def_submodule("peer_memory_cuda", "IPC peer memory pool + 1-D halo exchange (gfx950)");
  m.def("allocate_raw", &allocate_raw);
  m.def("free_raw", &free_raw);
  m.def("zero", &zero);
  m.def("get_raw_ipc_address", &get_raw_ipc_address);
  m.def("get_raw_peers", &get_raw_peers);
  m.def("close_raw_peers", &close_raw_peers);
  m.def("blob_view_half", [](int64_t raw, std::vector<int64_t> shape, bool cl) { return blob_view(raw, shape, cl, at::kHalf); });
  m.def("blob_view_bfloat16", [](int64_t raw, std::vector<int64_t> shape, bool cl) { return blob_view(raw, shape, cl, at::kBFloat16); });
  m.def("blob_view_float", [](int64_t raw, std::vector<int64_t> shape, bool cl) { return blob_view(raw, shape, cl, at::kFloat); });
  m.def("blob_view_int", [](int64_t raw, std::vector<int64_t> shape, bool cl) { return blob_view(raw, shape, cl, at::kInt); });
  m.def("push_pull_halos_1d", &push_pull_halos_1d);
  m.def("peer_allreduce", &peer_allreduce, py::arg("in"), py::arg("out"), py::arg("slots"), py::arg("flags"),
        py::arg("capacity"), py::arg("me"), py::arg("epoch"), py::arg("err"), py::arg("max_spins"),
        py::arg("epoch_dev") = py::none(),
        "one-shot IPC SUM all-reduce of a small fp32 vector (group BN statistics); epoch_dev: device epoch counter");
}

}  // namespace bhb
