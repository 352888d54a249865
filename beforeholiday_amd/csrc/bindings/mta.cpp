// amp_C front-end: python signatures match the reference's csrc/amp_C_frontend.cpp:165-194
// (chunk_size, noop_flag, tensor_lists, ...), kernels are bh::mta_* (kernels/multi_tensor.hip).
#include "common.h"

#include <cmath>
#include <map>
#include <mutex>
#include <unordered_map>

namespace bhb {

namespace {

struct KeyHash {
  size_t operator()(const std::vector<int64_t>& k) const noexcept {
    uint64_t h = 1469598103934665603ull;
    for (int64_t x : k) {
      h ^= static_cast<uint64_t>(x) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    }
    return static_cast<size_t>(h);
  }
};

std::mutex g_plan_mu;
// Heap-allocated and never destroyed: the cached plans own device / pinned tensors, and a static
// destructor running at process exit would free them into PyTorch's caching allocators after those
// were torn down (an exit-time segfault). clear_plan_cache() releases them while torch is alive.
auto& g_plans = *new std::unordered_map<std::vector<int64_t>, MTAPlan, KeyHash>();
constexpr size_t kMaxPlans = 4096;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

int list_dtype(const std::vector<at::Tensor>& l, const char* op) {
  TORCH_CHECK(!l.empty(), op, ": empty tensor list");
  const auto st = l[0].scalar_type();
  for (const auto& t : l) {
    TORCH_CHECK(t.scalar_type() == st, op, ": all tensors of a list must share a dtype");
    TORCH_CHECK(t.is_cuda(), op, ": tensors must be on the GPU");
    TORCH_CHECK(t.is_contiguous() || t.is_contiguous(at::MemoryFormat::ChannelsLast) ||
                    t.is_contiguous(at::MemoryFormat::ChannelsLast3d),
                op, ": tensors must be dense (contiguous or channels_last)");
  }
  return dtype_code(st);
}

const MTAPlan& get_plan(const std::vector<std::vector<at::Tensor>>& lists, int64_t chunk) {
  TORCH_CHECK(!lists.empty(), "multi_tensor: no tensor lists");
  const int depth = static_cast<int>(lists.size());
  const int T = static_cast<int>(lists[0].size());
  for (const auto& l : lists)
    TORCH_CHECK(static_cast<int>(l.size()) == T, "multi_tensor: tensor lists must have equal length");
  TORCH_CHECK(chunk > 0 && chunk % 8 == 0, "multi_tensor: chunk_size must be a positive multiple of 8");
  const auto dev = lists[0][0].device();

  std::vector<int64_t> key;
  key.reserve(4 + (size_t)T * (depth + 1));
  key.push_back(dev.index());
  key.push_back(depth);
  key.push_back(chunk);
  key.push_back(T);
  for (int t = 0; t < T; ++t) {
    const int64_t n = lists[0][t].numel();
    key.push_back(n);
    for (int d = 0; d < depth; ++d) {
      const auto& x = lists[d][t];
      TORCH_CHECK(x.numel() == n, "multi_tensor: size mismatch between lists at index ", t);
      TORCH_CHECK(x.device() == dev, "multi_tensor: all tensors must be on one device");
      key.push_back(reinterpret_cast<int64_t>(x.data_ptr()));
    }
  }

  std::lock_guard<std::mutex> lock(g_plan_mu);
  hipStream_t stream = stream_for(lists[0][0]);
  const bool in_capture = capturing(stream);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    it->second.pinned = it->second.pinned || in_capture;
    return it->second;
  }

  // a plan recorded into a HIP graph must outlive the graph: eviction (a full cache, e.g. eager work
  // whose tensor pointers keep changing) drops only the plans no capture has used
  if (g_plans.size() >= kMaxPlans) {
    for (auto e = g_plans.begin(); e != g_plans.end();) e = e->second.pinned ? std::next(e) : g_plans.erase(e);
  }

  // chunk schedule
  std::vector<int> chunk0(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    const int64_t n = lists[0][t].numel();
    const int64_t c = (n + chunk - 1) / chunk;
    TORCH_CHECK(chunk0[t] + c < (int64_t)INT32_MAX, "multi_tensor: too many chunks");
    chunk0[t + 1] = chunk0[t] + static_cast<int>(c);
  }
  const int C = chunk0[T];

  const size_t o_ptrs = 0;
  const size_t o_numel = align_up(o_ptrs + sizeof(uint64_t) * depth * T, 16);
  const size_t o_al = align_up(o_numel + sizeof(int64_t) * T, 16);
  const size_t o_c0 = align_up(o_al + sizeof(int) * T, 16);
  const size_t o_ct = align_up(o_c0 + sizeof(int) * (T + 1), 16);
  const size_t o_cl = align_up(o_ct + sizeof(int) * C, 16);
  const size_t bytes = align_up(o_cl + sizeof(int) * C, 16) + 16;

  // pinned staging + async copy normally; while capturing (pinned allocation is not allowed then) a
  // pageable table uploaded through kernel arguments
  at::Tensor host = at::empty({(int64_t)bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(!in_capture));
  uint8_t* h = host.data_ptr<uint8_t>();
  auto* hp = reinterpret_cast<uint64_t*>(h + o_ptrs);
  auto* hn = reinterpret_cast<int64_t*>(h + o_numel);
  auto* ha = reinterpret_cast<int*>(h + o_al);
  auto* hc0 = reinterpret_cast<int*>(h + o_c0);
  auto* hct = reinterpret_cast<int*>(h + o_ct);
  auto* hcl = reinterpret_cast<int*>(h + o_cl);
  for (int t = 0; t < T; ++t) {
    bool al = true;
    for (int d = 0; d < depth; ++d) {
      const uint64_t p = reinterpret_cast<uint64_t>(lists[d][t].data_ptr());
      hp[(size_t)d * T + t] = p;
      al = al && (p % 16 == 0);
    }
    hn[t] = lists[0][t].numel();
    ha[t] = al ? 1 : 0;
  }
  for (int t = 0; t <= T; ++t) hc0[t] = chunk0[t];
  for (int t = 0; t < T; ++t)
    for (int c = chunk0[t]; c < chunk0[t + 1]; ++c) {
      hct[c] = t;
      hcl[c] = c - chunk0[t];
    }

  at::Tensor devbuf = at::empty({(int64_t)bytes}, lists[0][0].options().dtype(at::kByte));
  if (in_capture) bh::upload_bytes(devbuf.data_ptr(), host.data_ptr(), bytes, stream);
  else devbuf.copy_(host, /*non_blocking=*/true);

  MTAPlan plan;
  plan.dev = devbuf;
  plan.host = host;
  uint8_t* d = devbuf.data_ptr<uint8_t>();
  plan.view.ptrs = reinterpret_cast<const uint64_t*>(d + o_ptrs);
  plan.view.numel = reinterpret_cast<const int64_t*>(d + o_numel);
  plan.view.aligned = reinterpret_cast<const int*>(d + o_al);
  plan.view.chunk0 = reinterpret_cast<const int*>(d + o_c0);
  plan.view.chunk_tensor = reinterpret_cast<const int*>(d + o_ct);
  plan.view.chunk_local = reinterpret_cast<const int*>(d + o_cl);
  plan.view.T = T;
  plan.view.C = C;
  plan.view.depth = depth;
  plan.view.chunk = static_cast<int>(chunk);
  plan.pinned = in_capture;
  auto res = g_plans.emplace(std::move(key), std::move(plan));
  return res.first->second;
}

namespace {

using Lists = std::vector<std::vector<at::Tensor>>;

void check_noop(const at::Tensor& noop) {
  TORCH_CHECK(noop.is_cuda() && noop.scalar_type() == at::kInt && noop.numel() >= 1,
              "noop_flag must be a GPU int32 tensor");
}

bool lists_empty(const Lists& l) { return l.empty() || l[0].empty(); }

void multi_tensor_scale(int64_t chunk, at::Tensor noop, Lists lists, double scale) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 2, "multi_tensor_scale expects 2 lists");
  check_noop(noop);
  const auto& p = get_plan(lists, chunk);
  bh::mta_scale(p.view, list_dtype(lists[0], "scale"), list_dtype(lists[1], "scale"), (float)scale,
                noop.data_ptr<int>(), stream_for(noop));
}

// scale given as a 1-element fp32 GPU tensor (read on device: no host synchronisation)
void multi_tensor_scale_tensor(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor scale) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 2, "multi_tensor_scale expects 2 lists");
  check_noop(noop);
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == 1,
              "scale must be a 1-element fp32 GPU tensor");
  const auto& p = get_plan(lists, chunk);
  bh::mta_scale(p.view, list_dtype(lists[0], "scale"), list_dtype(lists[1], "scale"), 1.f, noop.data_ptr<int>(),
                stream_for(noop), scale.data_ptr<float>());
}

void multi_tensor_axpby(int64_t chunk, at::Tensor noop, Lists lists, double a, double b, int64_t arg) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 3, "multi_tensor_axpby expects 3 lists");
  check_noop(noop);
  const auto& p = get_plan(lists, chunk);
  bh::mta_axpby(p.view, list_dtype(lists[0], "axpby"), list_dtype(lists[1], "axpby"),
                list_dtype(lists[2], "axpby"), (float)a, (float)b, (int)arg, noop.data_ptr<int>(),
                stream_for(noop));
}

std::tuple<at::Tensor, at::Tensor> norm_impl(int64_t chunk, at::Tensor noop, Lists lists,
                                             bool per_tensor, int norm_type, bool mp,
                                             double scale, bool with_scale) {
  check_noop(noop);
  auto fopt = noop.options().dtype(at::kFloat);
  if (lists_empty(lists)) {
    return {at::zeros({1}, fopt), per_tensor ? at::zeros({0}, fopt) : at::empty({0}, fopt)};
  }
  const auto& p = get_plan(lists, chunk);
  const int T = p.view.T;
  auto total = mp ? at::zeros({1}, fopt) : at::empty({1}, fopt);
  auto per = per_tensor ? at::zeros({T}, fopt) : at::empty({0}, fopt);
  auto partials = at::empty({std::max(p.view.C, 1)}, fopt);
  hipStream_t s = stream_for(noop);
  const int dt_in = list_dtype(lists[0], "l2norm");
  const int dt_out = with_scale ? list_dtype(lists[1], "l2norm_scale") : -1;
  bh::mta_norm_partials(p.view, dt_in, dt_out, norm_type, (float)scale, partials.data_ptr<float>(),
                        noop.data_ptr<int>(), mp, s);
  bh::mta_norm_finalize(p.view, partials.data_ptr<float>(), 1, norm_type,
                        per_tensor ? per.data_ptr<float>() : nullptr, total.data_ptr<float>(), false,
                        0.f, 0.f, noop.data_ptr<int>(), mp, s);
  return {total, per};
}

std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm(int64_t chunk, at::Tensor noop, Lists lists,
                                                       c10::optional<bool> per_tensor) {
  TORCH_CHECK(lists_empty(lists) || lists.size() == 1, "multi_tensor_l2norm expects 1 list");
  return norm_impl(chunk, noop, lists, per_tensor.value_or(false), 2, false, 1.0, false);
}
std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm_mp(int64_t chunk, at::Tensor noop, Lists lists,
                                                          c10::optional<bool> per_tensor) {
  TORCH_CHECK(lists_empty(lists) || lists.size() == 1, "multi_tensor_l2norm_mp expects 1 list");
  return norm_impl(chunk, noop, lists, per_tensor.value_or(false), 2, true, 1.0, false);
}
std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm_scale(int64_t chunk, at::Tensor noop, Lists lists,
                                                             double scale, c10::optional<bool> per_tensor) {
  TORCH_CHECK(lists_empty(lists) || lists.size() == 2, "multi_tensor_l2norm_scale expects 2 lists");
  return norm_impl(chunk, noop, lists, per_tensor.value_or(false), 2, false, scale, true);
}

// out[t] = blend(out[t], norm(list0[t]))  (L2: sqrt(a*o^2+b*n^2), Linf: a*o+b*n)
void multi_tensor_norm_out(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor out, double alpha,
                           double beta, int64_t norm_type) {
  if (lists_empty(lists)) return;
  check_noop(noop);
  const auto& p = get_plan({lists[0]}, chunk);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() == p.view.T,
              "multi_tensor_norm_out: out must be fp32 with one entry per tensor");
  auto partials = at::empty({std::max(p.view.C, 1)}, noop.options().dtype(at::kFloat));
  hipStream_t s = stream_for(noop);
  const int nt = norm_type == 0 ? 0 : 2;
  bh::mta_norm_partials(p.view, list_dtype(lists[0], "norm_out"), -1, nt, 1.f,
                        partials.data_ptr<float>(), noop.data_ptr<int>(), false, s);
  bh::mta_norm_finalize(p.view, partials.data_ptr<float>(), 1, nt, out.data_ptr<float>(), nullptr, true,
                        (float)alpha, (float)beta, noop.data_ptr<int>(), false, s);
}

int copy_dtype(const Lists& lists, size_t idx) {
  return lists.size() > idx ? list_dtype(lists[idx], "copy-out") : -1;
}

void multi_tensor_adam(int64_t chunk, at::Tensor noop, Lists lists, double lr, double beta1,
                       double beta2, double eps, int64_t step, int64_t mode, int64_t bias_correction,
                       double weight_decay) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "multi_tensor_adam expects 4 (or 5) lists");
  const auto& p = get_plan(lists, chunk);
  bh::AdamArgs a{};
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.bc1 = bias_correction ? 1.f - (float)std::pow(beta1, (double)step) : 1.f;
  a.bc2 = bias_correction ? 1.f - (float)std::pow(beta2, (double)step) : 1.f;
  a.decay = (float)weight_decay;
  a.mode = (int)mode;
  a.bias_correction = (int)bias_correction;
  bh::mta_adam(p.view, list_dtype(lists[0], "adam"), list_dtype(lists[1], "adam"),
               list_dtype(lists[2], "adam"), copy_dtype(lists, 4), a, stream_for(noop));
}

// capturable Adam: device lr/step, optional unscale + found_inf skip (GradScaler integration)
void multi_tensor_adam_capturable(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor lr,
                                  double beta1, double beta2, double eps, at::Tensor step, int64_t mode,
                                  int64_t bias_correction, double weight_decay,
                                  c10::optional<at::Tensor> inv_scale,
                                  c10::optional<at::Tensor> found_inf) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "multi_tensor_adam_capturable expects 4 (or 5) lists");
  const auto& p = get_plan(lists, chunk);
  bh::AdamArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.bc1 = a.bc2 = 1.f;
  a.decay = (float)weight_decay;
  a.mode = (int)mode;
  a.bias_correction = (int)bias_correction;
  TORCH_CHECK(lr.scalar_type() == at::kFloat && step.scalar_type() == at::kInt, "lr must be fp32, step int32");
  a.lr_ptr = lr.data_ptr<float>();
  a.step_ptr = step.data_ptr<int>();
  a.inv_scale = ptr_or_null<float>(inv_scale);
  a.found_inf = ptr_or_null<float>(found_inf);
  bh::mta_adam(p.view, list_dtype(lists[0], "adam"), list_dtype(lists[1], "adam"),
               list_dtype(lists[2], "adam"), copy_dtype(lists, 4), a, stream_for(noop));
}

void multi_tensor_sgd(int64_t chunk, at::Tensor noop, Lists lists, double wd, double momentum,
                      double dampening, double lr, bool nesterov, bool first_run, bool wd_after_momentum,
                      double scale) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 3 || lists.size() == 4, "multi_tensor_sgd expects 3 or 4 lists");
  check_noop(noop);
  const auto& p = get_plan(lists, chunk);
  bh::SGDArgs a{};
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.lr = (float)lr;
  a.scale = (float)scale;
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  const int dtg = list_dtype(lists[0], "sgd"), dtp = list_dtype(lists[1], "sgd");
  TORCH_CHECK(list_dtype(lists[2], "sgd") == dtp, "multi_tensor_sgd: momentum dtype must match params");
  bh::mta_sgd(p.view, dtg, dtp, copy_dtype(lists, 3), a, noop.data_ptr<int>(), stream_for(noop));
}

bh::LambArgs lamb_args(double lr, double beta1, double beta2, double eps, int64_t step,
                       int64_t bias_correction, double weight_decay, int64_t grad_averaging, int64_t mode,
                       double max_grad_norm, bool nvlamb) {
  bh::LambArgs a{};
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.beta3 = grad_averaging ? 1.f - (float)beta1 : 1.f;
  a.bc1 = bias_correction ? 1.f - (float)std::pow(beta1, (double)step) : 1.f;
  a.bc2 = bias_correction ? 1.f - (float)std::pow(beta2, (double)step) : 1.f;
  a.eps = (float)eps;
  a.decay = (float)weight_decay;
  a.max_grad_norm = (float)max_grad_norm;
  a.mode = (int)mode;
  a.use_nvlamb = nvlamb;
  a.bias_correction = (int)bias_correction;
  return a;
}

void lamb_run(const Lists& lists, int64_t chunk, const at::Tensor& noop, const bh::LambArgs& a) {
  const auto& p = get_plan(lists, chunk);
  auto fopt = noop.options().dtype(at::kFloat);
  auto partials = at::empty({2 * std::max(p.view.C, 1)}, fopt);
  // k_norm_finalize writes every per-tensor entry when there is at least one chunk
  auto norms = p.view.C > 0 ? at::empty({2 * std::max(p.view.T, 1)}, fopt) : at::zeros({2 * std::max(p.view.T, 1)}, fopt);
  hipStream_t s = stream_for(noop);
  const int dtg = list_dtype(lists[0], "lamb"), dtp = list_dtype(lists[1], "lamb");
  const int dts = list_dtype(lists[2], "lamb");
  TORCH_CHECK(list_dtype(lists[3], "lamb") == dts, "multi_tensor_lamb: exp_avg/exp_avg_sq dtype mismatch");
  bh::mta_lamb_stage1(p.view, dtg, dtp, dts, a, partials.data_ptr<float>(), s);
  bh::mta_norm_finalize(p.view, partials.data_ptr<float>(), 2, 2, norms.data_ptr<float>(), nullptr, false,
                        0.f, 0.f, nullptr, false, s);
  bh::mta_lamb_stage2(p.view, dtp, dts, copy_dtype(lists, 4), a, norms.data_ptr<float>(), s);
}

void multi_tensor_lamb(int64_t chunk, at::Tensor noop, Lists lists, double lr, double beta1, double beta2,
                       double eps, int64_t step, int64_t bias_correction, double weight_decay,
                       int64_t grad_averaging, int64_t mode, at::Tensor global_grad_norm,
                       double max_grad_norm, c10::optional<bool> use_nvlamb) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "multi_tensor_lamb expects 4 (or 5) lists");
  auto a = lamb_args(lr, beta1, beta2, eps, step, bias_correction, weight_decay, grad_averaging, mode,
                     max_grad_norm, use_nvlamb.value_or(false));
  TORCH_CHECK(global_grad_norm.is_cuda() && global_grad_norm.scalar_type() == at::kFloat,
              "global_grad_norm must be a GPU fp32 tensor");
  a.grad_norm = global_grad_norm.data_ptr<float>();
  a.noop = noop.data_ptr<int>();
  lamb_run(lists, chunk, noop, a);
}

void multi_tensor_lamb_mp(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor lr, double beta1,
                          double beta2, double eps, at::Tensor step, int64_t bias_correction,
                          double weight_decay, int64_t grad_averaging, int64_t mode,
                          at::Tensor global_grad_norm, at::Tensor max_grad_norm,
                          c10::optional<bool> use_nvlamb, at::Tensor found_inf, at::Tensor inv_scale) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 4 || lists.size() == 5, "multi_tensor_lamb_mp expects 4 or 5 lists");
  check_noop(noop);
  auto a = lamb_args(0.0, beta1, beta2, eps, 1, bias_correction, weight_decay, grad_averaging, mode, 0.0,
                     use_nvlamb.value_or(false));
  a.lr_ptr = lr.data_ptr<float>();
  TORCH_CHECK(step.scalar_type() == at::kInt, "step must be int32");
  a.step_ptr = step.data_ptr<int>();
  a.grad_norm = global_grad_norm.data_ptr<float>();
  a.max_norm_ptr = max_grad_norm.data_ptr<float>();
  a.found_inf = found_inf.data_ptr<float>();
  a.inv_scale = inv_scale.data_ptr<float>();
  a.noop = noop.data_ptr<int>();
  lamb_run(lists, chunk, noop, a);
}

void multi_tensor_lamb_stage1_cuda(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor per_tensor_decay,
                                   int64_t step, double beta1, double beta2, double eps,
                                   at::Tensor global_grad_norm, double max_global_grad_norm) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 5, "multi_tensor_lamb_stage1_cuda expects 5 lists");
  const auto& p = get_plan(lists, chunk);
  // the reference reads the (host-synchronised) norm value here as well
  const float gn = global_grad_norm.item<float>();
  const float clipped = gn > max_global_grad_norm ? gn / (float)max_global_grad_norm : 1.f;
  const float bc1 = 1.f - (float)std::pow(beta1, (double)step);
  const float bc2 = 1.f - (float)std::pow(beta2, (double)step);
  TORCH_CHECK(list_dtype(lists[2], "lamb_stage1") == list_dtype(lists[1], "lamb_stage1"),
              "lamb_stage1: moments must match param dtype");
  bh::mta_lamb_stage1_standalone(p.view, list_dtype(lists[0], "lamb_stage1"), list_dtype(lists[1], "lamb_stage1"),
                                 list_dtype(lists[4], "lamb_stage1"), per_tensor_decay.data_ptr<float>(),
                                 (float)beta1, (float)beta2, bc1, bc2, (float)eps, clipped, stream_for(noop));
}

void multi_tensor_lamb_stage2_cuda(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor pnorm,
                                   at::Tensor unorm, double lr, double weight_decay,
                                   c10::optional<bool> use_nvlamb) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 2, "multi_tensor_lamb_stage2_cuda expects 2 lists");
  const auto& p = get_plan(lists, chunk);
  bh::mta_lamb_stage2_standalone(p.view, list_dtype(lists[0], "lamb_stage2"), list_dtype(lists[1], "lamb_stage2"),
                                 pnorm.data_ptr<float>(), unorm.data_ptr<float>(), (float)lr,
                                 (float)weight_decay, use_nvlamb.value_or(false), stream_for(noop));
}

void multi_tensor_novograd(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor grad_norms, double lr,
                           double beta1, double beta2, double eps, int64_t step, int64_t bias_correction,
                           double weight_decay, int64_t grad_averaging, int64_t mode, int64_t norm_type) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 3, "multi_tensor_novograd expects 3 lists");
  float bc1 = 1.f, bc2 = 1.f;
  if (bias_correction) {
    bc1 = 1.f - (float)std::pow(beta1, (double)step);
    bc2 = std::sqrt(1.f - (float)std::pow(beta2, (double)step));
  }
  const float beta3 = grad_averaging ? 1.f - (float)beta1 : 1.f;
  multi_tensor_norm_out(chunk, noop, {lists[0]}, grad_norms, beta2, 1.0 - beta2, norm_type);
  const auto& p = get_plan(lists, chunk);
  const int dt = list_dtype(lists[0], "novograd");
  TORCH_CHECK(list_dtype(lists[1], "novograd") == dt && list_dtype(lists[2], "novograd") == dt,
              "multi_tensor_novograd: all lists must share a dtype");
  bh::mta_novograd(p.view, dt, (float)lr, (float)beta1, beta3, bc1, bc2, (float)eps, (int)mode,
                   (float)weight_decay, grad_norms.data_ptr<float>(), stream_for(noop));
}

void multi_tensor_adagrad(int64_t chunk, at::Tensor noop, Lists lists, double lr, double eps, int64_t mode,
                          double weight_decay) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 3, "multi_tensor_adagrad expects 3 lists");
  const auto& p = get_plan(lists, chunk);
  const int dt = list_dtype(lists[0], "adagrad");
  TORCH_CHECK(list_dtype(lists[1], "adagrad") == dt && list_dtype(lists[2], "adagrad") == dt,
              "multi_tensor_adagrad: all lists must share a dtype");
  bh::mta_adagrad(p.view, dt, (float)lr, (float)eps, (int)mode, (float)weight_decay, stream_for(noop));
}

void multi_tensor_lars(int64_t chunk, at::Tensor noop, Lists lists, at::Tensor grad_norms,
                       at::Tensor param_norms, double lr, double trust_coefficient, double eps,
                       double weight_decay, double momentum, double dampening, bool nesterov,
                       bool first_run, bool wd_after_momentum, double scale, bool is_skipped) {
  if (lists_empty(lists)) return;
  TORCH_CHECK(lists.size() == 3 || lists.size() == 4, "multi_tensor_lars expects 3 or 4 lists");
  check_noop(noop);
  const auto& p = get_plan(lists, chunk);
  bh::LarsArgs a{};
  a.lr = (float)lr;
  a.trust_coefficient = (float)trust_coefficient;
  a.eps = (float)eps;
  a.wd = (float)weight_decay;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.scale = (float)scale;
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  a.is_skipped = is_skipped;
  const int dtp = list_dtype(lists[1], "lars");
  TORCH_CHECK(list_dtype(lists[2], "lars") == dtp, "multi_tensor_lars: momentum dtype must match params");
  bh::mta_lars(p.view, list_dtype(lists[0], "lars"), dtp, copy_dtype(lists, 3), a, grad_norms.data_ptr<float>(),
               param_norms.data_ptr<float>(), noop.data_ptr<int>(), stream_for(noop));
}

size_t plan_cache_size() {
  std::lock_guard<std::mutex> lock(g_plan_mu);
  return g_plans.size();
}
void plan_cache_clear() {
  std::lock_guard<std::mutex> lock(g_plan_mu);
  g_plans.clear();
}

}  // namespace

// ---- ParamTable: the fused optimizers' host fast path ------------------------------------------
// The Python step of a fused optimizer walked every parameter twice and marshalled 4-5 tensor lists
// (hundreds of tensors) through pybind per launch: ~0.2 ms of host time for ResNet-50's 161 tensors,
// more than the GPU time of the whole LAMB update. A ParamTable holds each param group's parameters
// and optimizer-state tensors once; a step reads the current gradients through at::Tensor::grad() in
// C++, buckets them by dtype, and launches the same multi-tensor kernels (plans cached by pointer as
// before). Python passes only per-group hyper-parameters. A parameter whose gradient is set but
// whose state does not exist yet makes the step return false before any launch; the optimizer then
// creates the state and rebuilds the table.
class ParamTable {
 public:
  void add_group(std::vector<at::Tensor> params, std::vector<c10::optional<at::Tensor>> s0,
                 std::vector<c10::optional<at::Tensor>> s1, std::vector<c10::optional<at::Tensor>> master) {
    TORCH_CHECK(s0.size() == params.size() && s1.size() == params.size() &&
                    (master.empty() || master.size() == params.size()),
                "ParamTable.add_group: state lists must match the parameter list");
    Group g;
    g.p = std::move(params);
    auto unwrap = [](std::vector<c10::optional<at::Tensor>>& v, size_t n) {
      std::vector<at::Tensor> out(n);
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].has_value()) out[i] = *v[i];
      return out;
    };
    g.s0 = unwrap(s0, g.p.size());
    g.s1 = unwrap(s1, g.p.size());
    g.master = unwrap(master, g.p.size());
    groups_.push_back(std::move(g));
  }
  size_t num_groups() const { return groups_.size(); }

  // hyper[g] = {lr, beta1, beta2, eps, step, bias_correction, weight_decay, grad_averaging}
  // steps (optional): int32 [groups] device step counters (amp's device-resident loss scale): the
  // bias corrections use them, so a step skipped on the device does not advance them.
  // An entry with a master tensor updates the fp32 master from the gradient of its (16-bit) parameter
  // and writes the parameter back in stage 2 (the 5-list mixed-precision launch of
  // csrc/multi_tensor_lamb_mp.cu:41,248,367 in the reference). With ``inv_scale`` those gradients
  // are still loss-scaled: the kernels unscale them on the fly, and the global norm blends
  // ``scaled_norm`` (their norm, computed by amp's overflow check) times inv_scale with the norm of
  // the plain gradients -- no fp32 master gradient is ever materialised.
  bool lamb_step(at::Tensor noop, std::vector<std::vector<double>> hyper, int64_t mode, double max_grad_norm,
                 bool nvlamb, c10::optional<at::Tensor> steps, c10::optional<at::Tensor> inv_scale,
                 c10::optional<at::Tensor> scaled_norm) {
    TORCH_CHECK(hyper.size() == groups_.size(), "ParamTable.lamb_step: one hyper-parameter row per group");
    const bool scaled = inv_scale.has_value();
    // key: (target dtype, grad dtype, copy dtype or -1)
    std::vector<std::map<std::tuple<int, int, int>, Lists>> buckets(groups_.size());
    std::map<int, std::vector<at::Tensor>> plain_gdt, scaled_gdt;
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      const Group& g = groups_[gi];
      for (size_t i = 0; i < g.p.size(); ++i) {
        at::Tensor grad = grad_of(g.p[i], "FusedLAMB");
        if (!grad.defined()) continue;
        if (!g.s0[i].defined() || !g.s1[i].defined()) return false;
        const bool use_master = g.master[i].defined();
        const at::Tensor& target = use_master ? g.master[i] : g.p[i];
        auto& l = buckets[gi][{(int)target.scalar_type(), (int)grad.scalar_type(),
                               use_master ? (int)g.p[i].scalar_type() : -1}];
        if (l.empty()) l.resize(use_master ? 5 : 4);
        l[0].push_back(grad);
        l[1].push_back(target);
        l[2].push_back(g.s0[i]);
        l[3].push_back(g.s1[i]);
        if (use_master) l[4].push_back(g.p[i]);
        ((use_master && scaled) ? scaled_gdt : plain_gdt)[(int)grad.scalar_type()].push_back(grad);
      }
    }
    if (plain_gdt.empty() && scaled_gdt.empty()) return true;
    check_noop(noop);
    if (steps.has_value())
      TORCH_CHECK(steps->is_cuda() && steps->scalar_type() == at::kInt && steps->numel() >= (int64_t)groups_.size(),
                  "ParamTable.lamb_step: steps must be a CUDA int32 tensor with one counter per group");
    if (scaled)
      TORCH_CHECK(inv_scale->is_cuda() && inv_scale->scalar_type() == at::kFloat && inv_scale->numel() == 1,
                  "ParamTable.lamb_step: inv_scale must be a one-element CUDA fp32 tensor");
    // global gradient norm: one deterministic norm per gradient dtype, blended on the device
    auto norm_of = [&](std::vector<at::Tensor> l) {
      return std::get<0>(norm_impl(kNormChunk, noop, {std::move(l)}, false, 2, false, 1.0, false));
    };
    std::vector<at::Tensor> norms;
    for (auto& kv : plain_gdt) norms.push_back(norm_of(kv.second));
    at::Tensor gnorm;
    if (!scaled_gdt.empty()) {
      at::Tensor sn;
      if (scaled_norm.has_value()) {
        sn = scaled_norm->contiguous();
        TORCH_CHECK(sn.is_cuda() && sn.scalar_type() == at::kFloat && sn.numel() == 1,
                    "ParamTable.lamb_step: scaled_norm must be a one-element CUDA fp32 tensor");
      } else {
        std::vector<at::Tensor> sl;
        for (auto& kv : scaled_gdt) sl.push_back(norm_of(kv.second));
        sn = sl.size() == 1 ? sl[0] : norm_of(sl);
      }
      // the usual amp O2 case (one plain dtype at most): one blend launch, no per-step pointer list
      at::Tensor plain = norms.size() == 1 ? norms[0] : norms.empty() ? at::Tensor() : norm_of(norms);
      gnorm = at::empty({1}, sn.options());
      bh::norm_blend(plain.defined() ? plain.data_ptr<float>() : nullptr, sn.data_ptr<float>(),
                     inv_scale->data_ptr<float>(), gnorm.data_ptr<float>(), stream_for(noop));
    } else {
      gnorm = norms.size() == 1 ? norms[0] : norm_of(norms);
    }
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      const auto& h = hyper[gi];
      TORCH_CHECK(h.size() == 8, "ParamTable.lamb_step: 8 hyper-parameters per group");
      for (auto& kv : buckets[gi]) {
        auto a = lamb_args(h[0], h[1], h[2], h[3], (int64_t)h[4], (int64_t)h[5], h[6], (int64_t)h[7], mode,
                           max_grad_norm, nvlamb);
        a.grad_norm = gnorm.data_ptr<float>();
        a.noop = noop.data_ptr<int>();  // a set flag (amp's device-resident overflow) skips the step
        if (steps.has_value()) a.step_ptr = steps->data_ptr<int>() + gi;
        if (scaled && kv.second.size() == 5) a.inv_scale = inv_scale->data_ptr<float>();
        lamb_run(kv.second, kElemChunk, noop, a);
      }
    }
    return true;
  }

  // hyper[g] = {lr, beta1, beta2, eps, step, bias_correction, weight_decay}; a group entry with a
  // master tensor updates the fp32 master and writes the 16-bit parameter in the same launch, reading
  // the parameter's gradient times ``inv_scale`` when given (amp O2 / O5 without master gradients).
  // A set noop flag skips every launch; ``steps`` are device step counters as in lamb_step.
  bool adam_step(at::Tensor noop, std::vector<std::vector<double>> hyper, int64_t mode,
                 c10::optional<at::Tensor> steps, c10::optional<at::Tensor> inv_scale) {
    TORCH_CHECK(hyper.size() == groups_.size(), "ParamTable.adam_step: one hyper-parameter row per group");
    // every group is checked before anything launches: a retry after state creation must not
    // update the groups that were already complete a second time
    std::vector<std::map<std::tuple<int, int, int, int>, Lists>> all(groups_.size());
    bool any = false;
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      const Group& g = groups_[gi];
      auto& buckets = all[gi];
      for (size_t i = 0; i < g.p.size(); ++i) {
        at::Tensor grad = grad_of(g.p[i], "FusedAdam");
        if (!grad.defined()) continue;
        if (!g.s0[i].defined() || !g.s1[i].defined()) return false;
        const bool use_master = g.master[i].defined();
        const at::Tensor& target = use_master ? g.master[i] : g.p[i];
        auto& l = buckets[{(int)target.scalar_type(), (int)g.s0[i].scalar_type(), (int)grad.scalar_type(),
                           use_master ? (int)g.p[i].scalar_type() : -1}];
        if (l.empty()) l.resize(use_master ? 5 : 4);
        l[0].push_back(grad);
        l[1].push_back(target);
        l[2].push_back(g.s0[i]);
        l[3].push_back(g.s1[i]);
        if (use_master) l[4].push_back(g.p[i]);
        any = true;
      }
    }
    if (!any) return true;
    check_noop(noop);
    if (steps.has_value())
      TORCH_CHECK(steps->is_cuda() && steps->scalar_type() == at::kInt && steps->numel() >= (int64_t)groups_.size(),
                  "ParamTable.adam_step: steps must be a CUDA int32 tensor with one counter per group");
    if (inv_scale.has_value())
      TORCH_CHECK(inv_scale->is_cuda() && inv_scale->scalar_type() == at::kFloat && inv_scale->numel() == 1,
                  "ParamTable.adam_step: inv_scale must be a one-element CUDA fp32 tensor");
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      auto& buckets = all[gi];
      if (buckets.empty()) continue;
      const auto& h = hyper[gi];
      TORCH_CHECK(h.size() == 7, "ParamTable.adam_step: 7 hyper-parameters per group");
      for (auto& kv : buckets) {
        const Lists& lists = kv.second;
        bh::AdamArgs a{};
        a.lr = (float)h[0];
        a.beta1 = (float)h[1];
        a.beta2 = (float)h[2];
        a.eps = (float)h[3];
        a.bias_correction = (int)h[5];
        a.bc1 = a.bias_correction ? 1.f - (float)std::pow(h[1], h[4]) : 1.f;
        a.bc2 = a.bias_correction ? 1.f - (float)std::pow(h[2], h[4]) : 1.f;
        a.decay = (float)h[6];
        a.mode = (int)mode;
        a.noop = noop.data_ptr<int>();
        if (steps.has_value()) a.step_ptr = steps->data_ptr<int>() + gi;
        if (inv_scale.has_value() && lists.size() == 5) a.inv_scale = inv_scale->data_ptr<float>();
        const auto& p = get_plan(lists, kElemChunk);
        bh::mta_adam(p.view, list_dtype(lists[0], "adam"), list_dtype(lists[1], "adam"),
                     list_dtype(lists[2], "adam"), copy_dtype(lists, 4), a, stream_for(noop));
      }
    }
    return true;
  }

 private:
  struct Group {
    std::vector<at::Tensor> p, s0, s1, master;
  };
  static constexpr int64_t kElemChunk = 16384;  // multi_tensor_applier.chunk_size
  static constexpr int64_t kNormChunk = 65536;  // multi_tensor_applier_l2norm.chunk_size

  // the gradient laid out like its parameter (the kernels walk raw memory); undefined if none
  static at::Tensor grad_of(const at::Tensor& p, const char* who) {
    const at::Tensor& g = p.grad();
    if (!g.defined()) return g;
    TORCH_CHECK(!g.is_sparse(), who, " does not support sparse gradients");
    const auto st = p.scalar_type();
    TORCH_CHECK(st == at::kFloat || st == at::kHalf || st == at::kBFloat16 || st == at::kDouble, who,
                " only supports fp16, bf16, fp32 and fp64 parameters");
    if (p.numel() <= 1 || same_order(g, p)) return g;
    at::Tensor c = g.contiguous(p.suggest_memory_format());
    TORCH_CHECK(same_order(c, p), who, ": gradient layout differs from the parameter's");
    return c;
  }
  // the same element order in memory: equal strides on every dimension longer than 1 (a [K, C, 1, 1]
  // weight is both contiguous and channels_last, with different strides on the unit dims)
  static bool same_order(const at::Tensor& a, const at::Tensor& b) {
    if (a.sizes() != b.sizes()) return false;
    for (int64_t d = 0; d < a.dim(); ++d)
      if (a.size(d) > 1 && a.stride(d) != b.stride(d)) return false;
    return true;
  }

  std::vector<Group> groups_;
};

void register_amp_C(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("amp_C", "multi-tensor apply kernels (gfx950)");
  m.def("clear_plan_cache", [] {
    std::lock_guard<std::mutex> lock(g_plan_mu);
    g_plans.clear();
  }, "drop the cached device-resident chunk plans (registered with atexit by the python package)");
  m.def("multi_tensor_scale", &multi_tensor_scale, "out = in * scale with overflow flag");
  m.def("update_scale_device", [](at::Tensor scale, at::Tensor unskipped, at::Tensor overflow,
                                  c10::optional<at::Tensor> step_flag, double factor, int64_t window, double min_scale,
                                  double max_scale) {
    TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && unskipped.scalar_type() == at::kInt &&
                    overflow.scalar_type() == at::kInt && (!step_flag || step_flag->scalar_type() == at::kInt),
                "update_scale_device: fp32 scale, int32 counter / flags on the GPU");
    bh::amp_update_scale(scale.data_ptr<float>(), unskipped.data_ptr<int>(), overflow.data_ptr<int>(),
                         step_flag ? step_flag->data_ptr<int>() : nullptr, (float)factor, (int)window, (float)min_scale,
                         (float)max_scale, stream_for(scale));
  }, py::arg("scale"), py::arg("unskipped"), py::arg("overflow"), py::arg("step_flag"), py::arg("factor"),
     py::arg("window"), py::arg("min_scale"), py::arg("max_scale"),
     "amp's device loss-scale bookkeeping of one backward pass in one launch");
  m.def("multi_tensor_scale_tensor", &multi_tensor_scale_tensor, "out = in * scale[0] (device scalar)");
  m.def("multi_tensor_sgd", &multi_tensor_sgd, "fused SGD");
  m.def("multi_tensor_axpby", &multi_tensor_axpby, "out = a*x + b*y with overflow flag");
  m.def("multi_tensor_l2norm", &multi_tensor_l2norm, py::arg("chunk_size"), py::arg("noop_flag"),
        py::arg("tensor_lists"), py::arg("per_tensor") = py::none());
  m.def("multi_tensor_l2norm_mp", &multi_tensor_l2norm_mp, py::arg("chunk_size"), py::arg("noop_flag"),
        py::arg("tensor_lists"), py::arg("per_tensor") = py::none());
  m.def("multi_tensor_l2norm_scale", &multi_tensor_l2norm_scale, py::arg("chunk_size"), py::arg("noop_flag"),
        py::arg("tensor_lists"), py::arg("scale"), py::arg("per_tensor") = py::none());
  m.def("multi_tensor_norm_out", &multi_tensor_norm_out, "blended per-tensor norms");
  m.def("multi_tensor_lamb_stage1_cuda", &multi_tensor_lamb_stage1_cuda);
  m.def("multi_tensor_lamb_stage2_cuda", &multi_tensor_lamb_stage2_cuda);
  m.def("multi_tensor_adam", &multi_tensor_adam, "fused Adam/AdamW (5th list: low-precision param copy)");
  m.def("multi_tensor_adam_capturable", &multi_tensor_adam_capturable, py::arg("chunk_size"),
        py::arg("noop_flag"), py::arg("tensor_lists"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"),
        py::arg("eps"), py::arg("step"), py::arg("mode"), py::arg("bias_correction"),
        py::arg("weight_decay"), py::arg("inv_scale") = py::none(), py::arg("found_inf") = py::none());
  m.def("multi_tensor_adagrad", &multi_tensor_adagrad);
  m.def("multi_tensor_novograd", &multi_tensor_novograd);
  m.def("multi_tensor_lamb", &multi_tensor_lamb, py::arg("chunk_size"), py::arg("noop_flag"),
        py::arg("tensor_lists"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("epsilon"),
        py::arg("step"), py::arg("bias_correction"), py::arg("weight_decay"), py::arg("grad_averaging"),
        py::arg("mode"), py::arg("global_grad_norm"), py::arg("max_grad_norm"),
        py::arg("use_nvlamb_python") = py::none());
  m.def("multi_tensor_lamb_mp", &multi_tensor_lamb_mp);
  m.def("multi_tensor_lars", &multi_tensor_lars);
  m.def("plan_cache_size", &plan_cache_size);
  py::class_<ParamTable>(m, "ParamTable", "per-optimizer parameter / state table for the fused host fast path")
      .def(py::init<>())
      .def("add_group", &ParamTable::add_group, py::arg("params"), py::arg("state0"), py::arg("state1"),
           py::arg("master") = std::vector<c10::optional<at::Tensor>>())
      .def("num_groups", &ParamTable::num_groups)
      .def("lamb_step", &ParamTable::lamb_step, py::arg("noop_flag"), py::arg("hyper"), py::arg("mode"),
           py::arg("max_grad_norm"), py::arg("use_nvlamb"), py::arg("steps") = py::none(),
           py::arg("inv_scale") = py::none(), py::arg("scaled_norm") = py::none())
      .def("adam_step", &ParamTable::adam_step, py::arg("noop_flag"), py::arg("hyper"), py::arg("mode"),
           py::arg("steps") = py::none(), py::arg("inv_scale") = py::none());
  m.def("plan_cache_clear", &plan_cache_clear);
}

}  // namespace bhb
