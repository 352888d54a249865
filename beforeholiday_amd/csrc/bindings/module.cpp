// pybind11 module beforeholiday_amd._C: one shared object, one submodule per reference
// extension (amp_C, syncbn, fused_layer_norm_cuda, ...), so the python layer can expose
// the reference's module names without a second build system.
#include "common.h"

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "beforeholiday_amd native kernels (HIP, gfx950)";
  m.attr("arch") = "gfx950";
  bhb::register_amp_C(m);
  bhb::register_syncbn(m);
  bhb::register_norms(m);
  bhb::register_softmax(m);
  bhb::register_dense(m);
  bhb::register_contrib(m);
  bhb::register_misc(m);
  bhb::register_legacy_optim(m);
  bhb::register_peer_memory(m);
  bhb::register_conv(m);
  bhb::register_conv_bn(m);
  bhb::register_bn_fold(m);
}
