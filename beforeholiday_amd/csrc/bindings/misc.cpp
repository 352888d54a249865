// `apex_C` front-end: flatten / unflatten of dense tensor lists (reference: csrc/flatten_unflatten.cpp:5-17).
// One cat into a contiguous flat buffer / views of it; used by DDP-style bucketing and Reducer.
#include "common.h"

#include <torch/csrc/utils/tensor_flatten.h>

namespace bhb {
namespace {

at::Tensor flatten(std::vector<at::Tensor> tensors) { return torch::utils::flatten_dense_tensors(tensors); }

std::vector<at::Tensor> unflatten(at::Tensor flat, std::vector<at::Tensor> tensors) {
  return torch::utils::unflatten_dense_tensors(flat, tensors);
}

}  // namespace

void register_misc(pybind11::module_& root) {
  auto m = root.def_submodule("apex_C", "flatten / unflatten");
  m.def("flatten", &flatten, "Flatten dense tensors");
  m.def("unflatten", &unflatten, "Unflatten dense tensors");
}

}  // namespace bhb
