// `apex_C` front-end: flatten / unflatten of dense tensor lists (reference: csrc/flatten_unflatten.cpp:5-17).
// One cat into a contiguous flat buffer / views of it; used by DDP-style bucketing and Reducer.
// Also the native knob registry (bh/knobs.h) that beforeholiday_amd/config.py fills at import.
#include "common.h"
#include "bh/knobs.h"

#include <map>
#include <mutex>
#include <string>

#include <torch/csrc/utils/tensor_flatten.h>

namespace bh {
namespace {
std::mutex g_knob_mu;
std::map<std::string, int>& knob_map() {
  static auto* m = new std::map<std::string, int>();
  return *m;
}
}  // namespace
int knob(const char* name, int dflt) {
  std::lock_guard<std::mutex> lock(g_knob_mu);
  auto it = knob_map().find(name);
  return it == knob_map().end() ? dflt : it->second;
}
void set_knob(const char* name, int value) {
  std::lock_guard<std::mutex> lock(g_knob_mu);
  knob_map()[name] = value;
}
}  // namespace bh

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
  root.def("set_knobs", [](std::map<std::string, int> kv) {
    for (auto& e : kv) bh::set_knob(e.first.c_str(), e.second);
  }, "native run-time switches from beforeholiday_amd.config (dense_mfma, dense_tune, gemm_tile, gemm_log)");
  root.def("get_knob", [](const std::string& name, int dflt) { return bh::knob(name.c_str(), dflt); });
}

}  // namespace bhb
