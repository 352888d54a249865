// Shared helpers for the ATen/pybind front-end of beforeholiday_amd._C.
#pragma once

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "bh/api.h"

namespace bhb {

inline int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return bh::kF32;
    case at::kHalf: return bh::kF16;
    case at::kBFloat16: return bh::kBF16;
    case at::kDouble: return bh::kF64;
    case at::kByte: return bh::kU8;
    case at::kInt: return bh::kI32;
    case at::kLong: return bh::kI64;
    case at::kBool: return bh::kBool;
    default: TORCH_CHECK(false, "beforeholiday_amd: unsupported dtype ", t);
  }
  return -1;
}

inline hipStream_t stream_for(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

inline void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU (HIP) tensor");
}

inline bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &st);
  return st != hipStreamCaptureStatusNone;
}

template <typename T> inline T* ptr_or_null(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<T>() : nullptr;
}

// Multi-tensor plan (device-resident (tensor, chunk) schedule), cached per signature.
struct MTAPlan {
  bh::MTAView view;
  at::Tensor dev;   // keeps the device buffer alive
  at::Tensor host;  // pinned staging (kept alive: a captured graph may replay the H2D copy)
  bool pinned = false;  // used inside a HIP graph capture: never evicted (the graph holds its pointers)
};

// Builds or fetches the plan for `lists` (all lists same length; list i shares dtype).
const MTAPlan& get_plan(const std::vector<std::vector<at::Tensor>>& lists, int64_t chunk);

// dtype of list i (checks uniformity and contiguity, device)
int list_dtype(const std::vector<at::Tensor>& l, const char* op);

void register_amp_C(pybind11::module_& m);
void register_norms(pybind11::module_& m);
void register_syncbn(pybind11::module_& m);
void register_legacy_optim(pybind11::module_& m);
void register_peer_memory(pybind11::module_& m);
void register_softmax(pybind11::module_& m);
void register_dense(pybind11::module_& m);
void register_contrib(pybind11::module_& m);
void register_misc(pybind11::module_& m);
void register_conv(pybind11::module_& m);
void register_conv_bn(pybind11::module_& m);
void register_bn_fold(pybind11::module_& m);

}  // namespace bhb
