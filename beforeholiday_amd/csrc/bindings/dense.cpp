// `fused_dense_cuda`, `mlp_cuda`, `fused_weight_gradient_mlp_cuda` front-ends
// (reference APIs: csrc/fused_dense_base.cpp:15-20, csrc/mlp.cpp:46-164,
// csrc/megatron/fused_weight_gradient_dense.cpp).
//
// One implementation behind both the Python layers (ops/fused_dense.py) and the reference-named
// extensions: forward GEMMs with bias / activation epilogues on the MFMA kernel (gemm.hip) where the
// static rule picks it, data gradients through data_grad (MFMA dActivation + bias-gradient epilogue,
// hipBLASLt for a plain dY . W where the library measured faster), weight gradients through
// weight_grad (gemm_tn.hip for large weights, the 1x1 weight-gradient kernel for smaller ones, the
// library GEMM otherwise). Activation, dActivation and bias-gradient passes are kernels/dense.hip.
#include "common.h"
#include "bh/knobs.h"

#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "bh/dense_api.h"
#include "bh/gemm_api.h"

#include <cstdlib>

namespace bhb {
namespace {

bool al16(const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

at::Tensor as2d(const at::Tensor& t) { return t.dim() == 2 ? t : t.reshape({-1, t.size(-1)}); }

// y = act(x (+ bias)) in place on x
void act_inplace(at::Tensor& x, const at::Tensor& bias, int act) {
  if (act == bh::kActNone && !bias.defined()) return;
  const int64_t N = x.size(-1), M = x.numel() / std::max<int64_t>(N, 1);
  const bool vec = (N % 8 == 0) && al16(x) && (!bias.defined() || al16(bias));
  bh::dense_act_forward(dtype_code(x.scalar_type()), x.data_ptr(), bias.defined() ? bias.data_ptr() : nullptr,
                        x.data_ptr(), M, (int)N, act, vec, stream_for(x));
}

// dx = dy * act'(aux) (into dx_out, may be dy itself), returns bias grad if want_bgrad
at::Tensor act_backward(const at::Tensor& dy, const at::Tensor& aux, at::Tensor dx_out, int act, bool want_bgrad) {
  const int64_t N = dy.size(-1), M = dy.numel() / std::max<int64_t>(N, 1);
  at::Tensor bgrad;
  if (want_bgrad) bgrad = at::empty({N}, dy.options());
  if (act == bh::kActNone && !want_bgrad) return bgrad;
  const int splits = bh::dense_bgrad_splits(M, (int)N);
  auto part = at::empty({(int64_t)splits * N}, dy.options().dtype(at::kFloat));
  const bool vec = (N % 8 == 0) && al16(dy) && (!aux.defined() || al16(aux)) && (!dx_out.defined() || al16(dx_out));
  bh::dense_act_backward(dtype_code(dy.scalar_type()), dy.data_ptr(), aux.defined() ? aux.data_ptr() : nullptr,
                         (act != bh::kActNone && dx_out.defined()) ? dx_out.data_ptr() : nullptr,
                         want_bgrad ? bgrad.data_ptr() : nullptr, part.data_ptr<float>(), splits, M, (int)N, act, vec,
                         stream_for(dy));
  return bgrad;
}

at::Tensor bias_grad(const at::Tensor& dy) { return act_backward(dy, at::Tensor(), at::Tensor(), bh::kActNone, true); }

// Megatron bias-dropout-add: out = residual + dropout(x + bias); returns (out, keep bits uint8 [numel/8]).
// p == 0 (or eval) -> keep is an empty tensor and no dropout is applied.
std::vector<at::Tensor> bias_dropout_add(const at::Tensor& x, const c10::optional<at::Tensor>& bias,
                                         const at::Tensor& residual, double p, int64_t seed,
                                         const c10::optional<at::Tensor>& seed_dev) {
  check_cuda(x, "x");
  TORCH_CHECK(residual.sizes() == x.sizes() && residual.scalar_type() == x.scalar_type(),
              "bias_dropout_add: residual must match x in shape and dtype");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "bias_dropout_add: p must be in [0, 1)");
  auto xc = x.contiguous(), rc = residual.contiguous();
  const int64_t N = xc.size(-1), M = xc.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(N % 8 == 0 && al16(xc) && al16(rc), "bias_dropout_add: needs N % 8 == 0 and 16-byte aligned tensors");
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->contiguous();
    TORCH_CHECK(b.numel() == N && b.scalar_type() == x.scalar_type() && al16(b), "bias_dropout_add: bad bias");
  }
  const int64_t* sd = nullptr;  // device step seed (utils/graph_rng.py)
  if (seed_dev.has_value() && seed_dev->defined()) {
    TORCH_CHECK(seed_dev->scalar_type() == at::kLong && seed_dev->numel() == 1 && seed_dev->device() == x.device(),
                "bias_dropout_add: seed_dev must be an int64 [1] tensor on x's device");
    sd = seed_dev->data_ptr<int64_t>();
  }
  auto out = at::empty_like(xc);
  at::Tensor keep = at::empty({p > 0.0 ? xc.numel() / 8 : 0}, xc.options().dtype(at::kByte));
  bh::dense_bias_dropout_add(dtype_code(xc.scalar_type()), xc.data_ptr(), b.defined() ? b.data_ptr() : nullptr,
                             rc.data_ptr(), out.data_ptr(), p > 0.0 ? keep.data_ptr<uint8_t>() : nullptr, M, (int)N,
                             (float)p, (uint32_t)seed, stream_for(xc), sd);
  return {out, keep};
}

// backward of the dropout branch: dx = dy * keep / (1 - p) (dy itself when there is no mask), bias grad = sum dx
std::vector<at::Tensor> dropout_backward(const at::Tensor& dy, const at::Tensor& keep, double p, bool want_bgrad) {
  check_cuda(dy, "dy");
  auto g = dy.contiguous();
  const int64_t N = g.size(-1), M = g.numel() / std::max<int64_t>(N, 1);
  if (keep.numel() == 0) return {g, want_bgrad ? bias_grad(g) : at::Tensor()};
  TORCH_CHECK(keep.numel() * 8 == g.numel() && N % 8 == 0 && al16(g), "dropout_backward: mask / shape mismatch");
  auto dx = at::empty_like(g);
  at::Tensor bgrad;
  if (want_bgrad) bgrad = at::empty({N}, g.options());
  const int splits = bh::dense_bgrad_splits(M, (int)N);
  auto part = at::empty({(int64_t)splits * N}, g.options().dtype(at::kFloat));
  bh::dense_dropout_backward(dtype_code(g.scalar_type()), g.data_ptr(), keep.data_ptr<uint8_t>(),
                             (float)(1.0 / (1.0 - p)), dx.data_ptr(), want_bgrad ? bgrad.data_ptr() : nullptr,
                             part.data_ptr<float>(), splits, M, (int)N, stream_for(g));
  return {dx, bgrad};
}

// ------------------------------------------------------------------------------------------------
// MFMA GEMM with fused epilogue (kernels/gemm.hip). Config.dense_mfma = False routes everything back
// to hipBLASLt + the separate epilogue passes (A/B switch for benchmarks).
// ------------------------------------------------------------------------------------------------
bool mfma_enabled() { return bh::knob("dense_mfma", 1) != 0; }

bool mfma_ok(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c) {
  const auto t = a.scalar_type();
  if (!mfma_enabled() || (t != at::kHalf && t != at::kBFloat16) || b.scalar_type() != t || c.scalar_type() != t)
    return false;
  if (a.stride(1) != 1 || b.stride(1) != 1 || c.stride(1) != 1) return false;
  return bh::gemm_supported(a.size(0), b.size(0), a.size(1), a.stride(0), b.stride(0), c.stride(0), a.data_ptr(),
                            b.data_ptr(), c.data_ptr());
}

// Measured dispatch between the MFMA GEMM with the fused epilogue and hipBLASLt + a separate epilogue
// pass: per (op, dtype, M, N, K, epilogue) both are timed once on the current stream (first call, e.g.
// a warmup step) and the faster is kept. The MFMA kernel wins where the fused epilogue saves a pass
// that matters (K <= 1024: the GPT-2-medium fc1 forward, small MLPs); hipBLASLt's main loop wins the
// large-K shapes (fc2 forward / fc1 backward at K = 4096: 0.12 vs 0.08 ms,
// profiles/gemm_mfma_big_tile_vs_hipblaslt.jsonl). The timing is opt-in (Config.dense_tune): a per-process
// timing pick can differ between ranks (another kernel, other rounding), so by default the static
// K <= 1024 rule decides; during HIP-graph capture the cached choice (or the rule) is used.
bool tune_enabled() { return bh::knob("dense_tune", 0) != 0; }

template <typename F>
float time_ms(hipStream_t st, F&& fn) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fn();
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < 3; ++i) fn();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

// tests / benchmarks pin the MFMA kernel so the measured dispatch cannot route around it
bool g_force_mfma = false;

template <typename FA, typename FB>
bool prefer_mfma(const char* op, const at::Tensor& a, int64_t M, int64_t N, int64_t K, int variant, FA&& mfma,
                 FB&& lib) {
  static std::mutex mu;
  static auto& cache = *new std::map<std::tuple<std::string, int, int64_t, int64_t, int64_t, int>, bool>();
  if (g_force_mfma) return true;
  const auto key = std::make_tuple(std::string(op), (int)a.scalar_type(), M, N, K, variant);
  {
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const bool rule = K <= 1024;
  hipStream_t st = stream_for(a);
  if (!tune_enabled() || capturing(st)) return rule;
  const float tm = time_ms(st, mfma);
  const float tl = time_ms(st, lib);
  const bool pick = tm < tl;
  std::lock_guard<std::mutex> lock(mu);
  cache[key] = pick;
  return pick;
}

// y = act(x . w^T + bias), optionally also the pre-activation. x [M,K], w [N,K].
std::vector<at::Tensor> linear_act(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int act,
                                   bool want_pre) {
  auto y = at::empty({x.size(0), w.size(0)}, x.options());
  at::Tensor pre;
  if (want_pre) pre = at::empty_like(y);
  const bool bias_ok = !bias.defined() || (bias.is_contiguous() && al16(bias) && bias.scalar_type() == x.scalar_type());
  auto run_mfma = [&] {
    bh::GemmEpilogue e;
    e.bias = bias.defined() ? bias.data_ptr() : nullptr;
    e.act = act;
    e.pre_out = want_pre ? pre.data_ptr() : nullptr;
    e.ld_aux = y.size(1);
    bh::gemm_nt(dtype_code(x.scalar_type()), x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(),
                y.stride(0), x.size(0), w.size(0), x.size(1), e, stream_for(x));
  };
  auto run_lib = [&] {
    if (bias.defined()) at::addmm_out(y, bias, x, w.t());
    else at::mm_out(y, x, w.t());
    if (want_pre) pre.copy_(y);
    act_inplace(y, at::Tensor(), act);
  };
  if (bias_ok && mfma_ok(x, w, y) &&
      prefer_mfma("linear_act", x, x.size(0), w.size(0), x.size(1), act * 2 + (want_pre ? 1 : 0), run_mfma, run_lib)) {
    run_mfma();
  } else {
    run_lib();
  }
  return {y, pre};
}

// dx = (dy . wt^T) * act'(aux) and its column sum. dy [M,N], wt [K,N] (the weight transposed).
std::vector<at::Tensor> linear_dact(const at::Tensor& dy, const at::Tensor& wt, const at::Tensor& aux, int act,
                                    bool want_bgrad) {
  auto dx = at::empty({dy.size(0), wt.size(0)}, dy.options());
  const bool aux_ok = act == bh::kActNone ||
                      (aux.defined() && aux.dim() == 2 && aux.stride(1) == 1 && aux.stride(0) % 8 == 0 && al16(aux) &&
                       aux.scalar_type() == dy.scalar_type());
  auto run_lib = [&] {
    at::mm_out(dx, dy, wt.t());
    return act_backward(dx, aux, dx, act, want_bgrad);
  };
  auto run_mfma = [&] {
    at::Tensor part, db;
    bh::GemmEpilogue e;
    e.act = act;
    e.bwd_act = true;
    e.aux_in = act != bh::kActNone ? aux.data_ptr() : nullptr;
    e.ld_aux = act != bh::kActNone ? aux.stride(0) : dx.size(1);
    const int64_t slabs = bh::gemm_bgrad_slabs(dy.size(0));
    if (want_bgrad) {
      part = at::empty({slabs, dx.size(1)}, dy.options().dtype(at::kFloat));
      e.bgrad_part = part.data_ptr<float>();
    }
    bh::gemm_nt(dtype_code(dy.scalar_type()), dy.data_ptr(), dy.stride(0), wt.data_ptr(), wt.stride(0),
                dx.data_ptr(), dx.stride(0), dy.size(0), wt.size(0), dy.size(1), e, stream_for(dy));
    if (want_bgrad) {
      db = at::empty({dx.size(1)}, dy.options());
      bh::gemm_colsum_finalize(dtype_code(dy.scalar_type()), part.data_ptr<float>(), slabs, dx.size(1), db.data_ptr(),
                               stream_for(dy));
    }
    return db;
  };
  // a plain data gradient (no activation derivative, no bias gradient) has no epilogue to fuse: the library
  // GEMM measured 1.0-1.18x faster there (profiles/dgrad_transformer_nt_vs_hipblaslt.jsonl)
  const bool fused_work = act != bh::kActNone || want_bgrad || g_force_mfma;
  if (fused_work && aux_ok && mfma_ok(dy, wt, dx) &&
      prefer_mfma("linear_dact", dy, dy.size(0), wt.size(0), dy.size(1), act * 2 + (want_bgrad ? 1 : 0), run_mfma,
                  run_lib)) {
    return {dx, run_mfma()};
  }
  return {dx, run_lib()};
}

// dx = (dy . w) * act'(aux) and its column sum, w [N, K] as the layer stores it. The MFMA kernel needs the
// weight transposed ([K, N] rows), so the transpose runs only when that kernel takes the call.
std::vector<at::Tensor> data_grad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& aux, int act,
                                  bool want_bgrad) {
  const bool fused_work = act != bh::kActNone || want_bgrad || g_force_mfma;
  const bool t16 = w.dim() == 2 && w.is_contiguous() && w.element_size() == 2 && w.size(0) % 8 == 0 &&
                   w.size(1) % 8 == 0 && w.scalar_type() == dy.scalar_type();
  if (!fused_work || !t16 || !mfma_enabled()) {
    auto dx = at::mm(dy, w);
    at::Tensor db;
    if (act != bh::kActNone || want_bgrad) db = act_backward(dx, aux, dx, act, want_bgrad);
    return {dx, db};
  }
  auto wt = at::empty({w.size(1), w.size(0)}, w.options());
  bh::transpose16(w.data_ptr(), w.size(0), w.size(1), wt.data_ptr(), stream_for(w));
  return linear_dact(dy, wt, aux, act, want_bgrad);
}

}  // namespace

bool dense_wgrad_conv(const at::Tensor& dy, const at::Tensor& x, at::Tensor& out);  // bindings/conv.cpp

namespace {

// The static weight-gradient rules (identical on every rank): the transposed-operand MFMA GEMM
// (kernels/gemm_tn.hip) from 1.5M-element weights on (1.12-1.28x hipBLASLt at 8192 tokens,
// profiles/wgrad_tn_vs_hipblaslt.jsonl), the 1x1 weight-gradient kernel up to ~2.4M elements
// (1.05-2.4x the library at 512^2 .. 3072 x 768), both from 4096 tokens; the library GEMM otherwise.
constexpr int64_t kWgradMinTokens = 4096, kWgradTnMinElems = 1536 * 1024, kWgradConvMaxElems = 3072 * 800;

at::Tensor weight_grad(const at::Tensor& dy_in, const at::Tensor& x_in) {
  const at::Tensor dy = as2d(dy_in), x = as2d(x_in);
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  const bool mfma = bh::knob("dense_wgrad", 1) != 0 && dy.scalar_type() == x.scalar_type() &&
                    (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16) && T >= kWgradMinTokens &&
                    dy.stride(-1) == 1 && x.stride(-1) == 1;
  if (mfma && N * K >= kWgradTnMinElems &&
      bh::gemm_tn_supported(N, K, T, dy.stride(0), x.stride(0), dy.data_ptr(), x.data_ptr(), dy.data_ptr())) {
    auto out = at::empty({N, K}, dy.options());
    const int s = bh::gemm_tn_splits(N, K, T);
    at::Tensor ws;
    if (s > 1) ws = at::empty({(int64_t)s, N, K}, dy.options().dtype(at::kFloat));
    bh::gemm_tn(dtype_code(dy.scalar_type()), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
                N, K, T, s > 1 ? ws.data_ptr<float>() : nullptr, s, stream_for(dy));
    return out;
  }
  at::Tensor out;
  if (mfma && N * K <= kWgradConvMaxElems && dense_wgrad_conv(dy, x, out)) return out;
  return at::mm(dy.t(), x);
}

// ------------------------------------------------------------------------------------------------
// fused_dense_cuda
// ------------------------------------------------------------------------------------------------
at::Tensor linear_bias_forward(at::Tensor input, at::Tensor weight, at::Tensor bias) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  // the MFMA GEMM with the bias in its epilogue where the static rule picks it (linear_act), else addmm
  auto y = linear_act(x, weight.contiguous(), bias.defined() ? bias.contiguous() : bias, bh::kActNone, false)[0];
  auto shape = input.sizes().vec();
  shape.back() = weight.size(0);
  return y.view(shape);
}

std::vector<at::Tensor> linear_bias_backward(at::Tensor input, at::Tensor weight, at::Tensor d_output) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output.contiguous());
  auto d_input = data_grad(dy, weight.contiguous(), at::Tensor(), bh::kActNone, false)[0].view(input.sizes());
  return {d_input, weight_grad(dy, x), bias_grad(dy)};
}

std::vector<at::Tensor> linear_gelu_linear_forward(at::Tensor input, at::Tensor weight1, at::Tensor bias1,
                                                   at::Tensor weight2, at::Tensor bias2) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto h = linear_act(x, weight1.contiguous(), bias1.contiguous(), bh::kActGelu, true);
  auto gelu_in = h[1], out1 = h[0];
  auto out2 = linear_act(out1, weight2.contiguous(), bias2.contiguous(), bh::kActNone, false)[0];
  return {gelu_in, out1, out2};
}

// returns {d_input, d_weight1, d_bias1, d_weight2, d_bias2}
std::vector<at::Tensor> linear_gelu_linear_backward(at::Tensor input, at::Tensor gelu_in, at::Tensor output1,
                                                    at::Tensor weight1, at::Tensor weight2, at::Tensor d_output2) {
  check_cuda(input, "input");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output2.contiguous());
  auto h = as2d(output1.contiguous());
  auto d_weight2 = weight_grad(dy, h);
  auto d_bias2 = bias_grad(dy);
  auto dh = data_grad(dy, weight2.contiguous(), as2d(gelu_in.contiguous()), bh::kActGelu, true);
  auto d_h = dh[0], d_bias1 = dh[1];
  auto d_weight1 = weight_grad(d_h, x);
  auto d_input = data_grad(d_h, weight1.contiguous(), at::Tensor(), bh::kActNone, false)[0].view(input.sizes());
  return {d_input, d_weight1, d_bias1, d_weight2, d_bias2};
}

// ------------------------------------------------------------------------------------------------
// mlp_cuda: inputs = (x, W_0..W_{n-1}[, b_0..b_{n-1}]); activation 0 none, 1 relu, 2 sigmoid after
// every layer. forward returns the n layer outputs (last = result); backward returns grads for inputs.
// ------------------------------------------------------------------------------------------------
int mlp_act(int activation) {
  switch (activation) {
    case 0: return bh::kActNone;
    case 1: return bh::kActRelu;
    case 2: return bh::kActSigmoid;
    default: TORCH_CHECK(false, "mlp: activation must be 0 (none), 1 (relu) or 2 (sigmoid)");
  }
  return 0;
}

std::vector<at::Tensor> mlp_forward(int use_bias, int activation, std::vector<at::Tensor> inputs) {
  TORCH_CHECK(!inputs.empty(), "mlp: no inputs");
  check_cuda(inputs[0], "input");
  const int64_t n = use_bias ? (int64_t)(inputs.size() - 1) / 2 : (int64_t)inputs.size() - 1;
  const int act = mlp_act(activation);
  std::vector<at::Tensor> outs;
  at::Tensor h = inputs[0].contiguous();
  for (int64_t i = 0; i < n; ++i) {
    const at::Tensor w = inputs[1 + i].contiguous();
    at::Tensor y = linear_act(h, w, use_bias ? inputs[1 + n + i].contiguous() : at::Tensor(), act, false)[0];
    outs.push_back(y);
    h = y;
  }
  return outs;
}

std::vector<at::Tensor> mlp_backward(int use_bias, int activation, at::Tensor grad_o, std::vector<at::Tensor> outputs,
                                     std::vector<at::Tensor> inputs) {
  const int64_t n = use_bias ? (int64_t)(inputs.size() - 1) / 2 : (int64_t)inputs.size() - 1;
  const int act = mlp_act(activation);
  std::vector<at::Tensor> grads(inputs.size());
  // dpre := dL/d(pre-activation of layer i). The last layer's comes from one dActivation pass over
  // grad_o; every earlier one straight out of the dgrad GEMM's epilogue (dActivation + bias grad).
  at::Tensor g = grad_o.contiguous();
  at::Tensor dpre = (act == bh::kActNone) ? g : at::empty_like(g);
  at::Tensor db = act_backward(g, outputs[n - 1], dpre, act, use_bias != 0);
  if (act == bh::kActNone) dpre = g;
  for (int64_t i = n - 1; i >= 0; --i) {
    const at::Tensor& x = (i == 0) ? inputs[0] : outputs[i - 1];
    grads[1 + i] = weight_grad(dpre, x.contiguous());
    if (use_bias) grads[1 + n + i] = db;
    if (i > 0) {
      auto r = data_grad(dpre, inputs[1 + i].contiguous(), outputs[i - 1].contiguous(), act, use_bias != 0);
      dpre = r[0];
      db = r[1];
    } else {
      g = inputs[0].requires_grad()
              ? data_grad(dpre, inputs[1].contiguous(), at::Tensor(), bh::kActNone, false)[0]
              : at::Tensor();
    }
  }
  grads[0] = inputs[0].requires_grad() ? g : at::zeros_like(inputs[0]);
  return grads;
}

// ------------------------------------------------------------------------------------------------
// fused_weight_gradient_mlp_cuda: main_grad[N,K] += d_output[M,N]^T @ input[M,K]
// ------------------------------------------------------------------------------------------------
// the transposed-operand MFMA GEMM accumulating into main_grad (accum 1: fp32, 2: 16-bit) where it takes the
// shape (a contiguous [N, K] main_grad); false: the caller runs the library GEMM
bool wgrad_accum_tn(const at::Tensor& x, const at::Tensor& dy, at::Tensor& main_grad, int accum) {
  if (!(x.scalar_type() == dy.scalar_type() && (x.scalar_type() == at::kHalf || x.scalar_type() == at::kBFloat16) &&
        main_grad.is_contiguous() && main_grad.dim() == 2 && main_grad.size(0) == dy.size(1) &&
        main_grad.size(1) == x.size(1) && x.size(0) >= 4096 &&
        bh::gemm_tn_supported(dy.size(1), x.size(1), dy.size(0), dy.stride(0), x.stride(0), dy.data_ptr(),
                              x.data_ptr(), main_grad.data_ptr())))
    return false;
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  const int s = bh::gemm_tn_splits(N, K, T);
  auto ws = at::empty({(int64_t)s, N, K}, dy.options().dtype(at::kFloat));
  bh::gemm_tn(dtype_code(dy.scalar_type()), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0),
              main_grad.data_ptr(), N, K, T, ws.data_ptr<float>(), s, stream_for(dy), accum);
  return true;
}

void wgrad_gemm_accum_fp32(at::Tensor input, at::Tensor d_output, at::Tensor main_grad) {
  check_cuda(input, "input");
  TORCH_CHECK(main_grad.scalar_type() == at::kFloat, "wgrad_gemm_accum_fp32: main_grad must be fp32");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output.contiguous());
  if (wgrad_accum_tn(x, dy, main_grad, 1)) return;
  if (x.scalar_type() == at::kFloat) {
    main_grad.addmm_(dy.t(), x);
  } else {
    at::addmm_out(main_grad, main_grad, dy.t(), x, at::kFloat, 1, 1);
  }
}

void wgrad_gemm_accum_fp16(at::Tensor input, at::Tensor d_output, at::Tensor main_grad) {
  check_cuda(input, "input");
  TORCH_CHECK(main_grad.scalar_type() == input.scalar_type(), "wgrad_gemm_accum_fp16: dtype mismatch");
  auto x = as2d(input.contiguous());
  auto dy = as2d(d_output.contiguous());
  if (wgrad_accum_tn(x, dy, main_grad, 2)) return;
  main_grad.addmm_(dy.t(), x);
}

// activation helpers exposed for python modules (bias_gelu etc.)
at::Tensor act_forward_py(at::Tensor x, c10::optional<at::Tensor> bias, int act) {
  check_cuda(x, "x");
  auto y = x.contiguous().clone();
  act_inplace(y, bias.has_value() ? bias->contiguous() : at::Tensor(), act);
  return y;
}

std::vector<at::Tensor> act_backward_py(at::Tensor dy, at::Tensor aux, int act, bool want_bgrad) {
  check_cuda(dy, "dy");
  dy = dy.contiguous();
  aux = aux.contiguous();
  auto dx = at::empty_like(dy);
  auto db = act_backward(dy, aux, dx, act, want_bgrad);
  if (act == bh::kActNone) dx = dy;
  return {dx, db.defined() ? db : at::Tensor()};
}

}  // namespace

namespace {
// embedding weight gradient without torch's host read-back of the segment count (kernels/dense.hip)
at::Tensor embedding_bwd(at::Tensor dy, at::Tensor ids, int64_t num_weights, int64_t padding_idx) {
  check_cuda(dy, "dy");
  check_cuda(ids, "ids");
  const int64_t H = dy.size(-1);
  auto d2 = dy.reshape({-1, H}).contiguous();
  auto flat = ids.reshape({-1}).to(at::kLong);
  TORCH_CHECK(flat.numel() == d2.size(0), "embedding_backward: ", flat.numel(), " ids for ", d2.size(0), " rows");
  TORCH_CHECK(H > 0 && H <= INT32_MAX, "embedding_backward: bad hidden size");
  auto sp = at::sort(flat, /*stable=*/true, 0, false);
  const at::Tensor& sorted = std::get<0>(sp);
  const at::Tensor& perm = std::get<1>(sp);
  auto dw = at::zeros({num_weights, H}, dy.options());
  const int64_t n = d2.size(0);
  if (n == 0) return dw;
  auto piece = at::empty({n, H}, dy.options().dtype(at::kFloat));
  bh::embedding_backward(dtype_code(dy.scalar_type()), sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(),
                         d2.data_ptr(), piece.data_ptr<float>(), dw.data_ptr(), n, (int)H, padding_idx,
                         stream_for(dy));
  return dw;
}
}  // namespace

void register_dense(pybind11::module_& root) {
  namespace py = pybind11;
  auto fd = root.def_submodule("fused_dense_cuda", "GEMM + bias / GELU dense layers");
  fd.def("linear_bias_forward", &linear_bias_forward);
  fd.def("linear_bias_backward", &linear_bias_backward);
  fd.def("linear_gelu_linear_forward", &linear_gelu_linear_forward);
  fd.def("linear_gelu_linear_backward", &linear_gelu_linear_backward);
  fd.def("act_forward", &act_forward_py, py::arg("x"), py::arg("bias"), py::arg("act"));
  fd.def("weight_grad", [](at::Tensor dy, at::Tensor x) {
    check_cuda(dy, "dy");
    return weight_grad(dy, x);
  }, py::arg("dy"), py::arg("x"), "dW = dy^T . x for 2-D [tokens, out] / [tokens, in] (static MFMA / library rule)");
  fd.def("data_grad", [](at::Tensor dy, at::Tensor w, c10::optional<at::Tensor> aux, int act, bool want_bgrad) {
    check_cuda(dy, "dy");
    return data_grad(dy.contiguous(), w.contiguous(), aux.has_value() ? aux->contiguous() : at::Tensor(), act,
                     want_bgrad);
  }, py::arg("dy"), py::arg("w"), py::arg("aux"), py::arg("act"), py::arg("want_bgrad"),
     "(dy . w) * act'(aux) and its column sum; w [out, in] as stored");
  fd.def("act_backward", &act_backward_py, py::arg("dy"), py::arg("aux"), py::arg("act"), py::arg("want_bgrad"));
  fd.def("embedding_backward", &embedding_bwd, py::arg("dy"), py::arg("ids"), py::arg("num_weights"),
         py::arg("padding_idx") = -1, "deterministic embedding weight gradient [num_weights, H], no host sync");
  fd.def("bias_grad", [](at::Tensor dy) {
    check_cuda(dy, "dy");
    return bias_grad(dy.contiguous());
  }, py::arg("dy"), "column sum of dy[..., N] over all leading dims (fp32 accumulation, dy dtype out)");
  fd.def("bias_dropout_add", &bias_dropout_add, py::arg("x"), py::arg("bias"), py::arg("residual"), py::arg("p"),
         py::arg("seed"), py::arg("seed_dev") = py::none(),
         "out = residual + dropout(x + bias) in one pass; returns (out, keep bits)");
  fd.def("dropout_backward", &dropout_backward, py::arg("dy"), py::arg("keep"), py::arg("p"), py::arg("want_bgrad"),
         "dx = dy * keep / (1 - p) with the bias gradient sum(dx) from the same pass; returns (dx, bgrad)");
  auto mlp = root.def_submodule("mlp_cuda", "N-layer MLP");
  mlp.def("forward", &mlp_forward);
  mlp.def("backward", &mlp_backward);
  auto gm = root.def_submodule("gemm", "MFMA GEMM with fused dense epilogues (kernels/gemm.hip)");
  gm.def("linear_act", [](at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, int act, bool want_pre) {
    check_cuda(x, "x");
    return linear_act(x, w, bias.has_value() ? *bias : at::Tensor(), act, want_pre);
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("act"), py::arg("want_pre"));
  gm.def("linear_dact", [](at::Tensor dy, at::Tensor wt, c10::optional<at::Tensor> aux, int act, bool want_bgrad) {
    check_cuda(dy, "dy");
    return linear_dact(dy, wt, aux.has_value() ? *aux : at::Tensor(), act, want_bgrad);
  }, py::arg("dy"), py::arg("wt"), py::arg("aux"), py::arg("act"), py::arg("want_bgrad"));
  gm.def("mm_nt", [](at::Tensor a, at::Tensor b, c10::optional<at::Tensor> bias) {
    // C = a . b^T (+ bias) on the MFMA GEMM, unconditionally (no measured dispatch, no library
    // fallback: a fixed kernel per shape, so every rank computes bitwise the same); unsupported
    // shapes / layouts raise
    check_cuda(a, "a");
    check_cuda(b, "b");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1) && a.scalar_type() == b.scalar_type() &&
                    (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16),
                "gemm.mm_nt: a [M, K] and b [N, K] fp16 / bf16");
    auto c = at::empty({a.size(0), b.size(0)}, a.options());
    const bool bias_ok = !bias.has_value() || !bias->defined() ||
                         (bias->is_contiguous() && al16(*bias) && bias->scalar_type() == a.scalar_type() &&
                          bias->numel() == b.size(0));
    TORCH_CHECK(bias_ok && a.stride(1) == 1 && b.stride(1) == 1 &&
                    bh::gemm_supported(a.size(0), b.size(0), a.size(1), a.stride(0), b.stride(0), c.stride(0),
                                       a.data_ptr(), b.data_ptr(), c.data_ptr()),
                "gemm.mm_nt: unsupported shape / layout (K % 8, N % 8, 16-byte aligned rows)");
    bh::GemmEpilogue e;
    e.bias = (bias.has_value() && bias->defined()) ? bias->data_ptr() : nullptr;
    bh::gemm_nt(dtype_code(a.scalar_type()), a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                c.stride(0), a.size(0), b.size(0), a.size(1), e, stream_for(a));
    return c;
  }, py::arg("a"), py::arg("b"), py::arg("bias") = py::none());
  gm.def("transpose", [](at::Tensor x) {
    check_cuda(x, "x");
    TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.element_size() == 2, "gemm.transpose: contiguous 2-D 16-bit");
    auto y = at::empty({x.size(1), x.size(0)}, x.options());
    bh::transpose16(x.data_ptr(), x.size(0), x.size(1), y.data_ptr(), stream_for(x));
    return y;
  }, py::arg("x"), "x.t().contiguous() for a 2-D 16-bit tensor (64 x 64 LDS tiles, 16-byte accesses)");
  // dW [N, K] = dy[T, N]^T @ x[T, K] on the transposed-operand ping-pong kernel (splits: 0 = automatic)
  gm.def("weight_grad_tn", [](at::Tensor dy, at::Tensor x, int64_t splits) {
    TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0) &&
                    dy.scalar_type() == x.scalar_type() && dy.stride(1) == 1 && x.stride(1) == 1 &&
                    (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16),
                "gemm.weight_grad_tn: dy [T, N] and x [T, K], one 16-bit dtype, unit column stride");
    const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
    auto out = at::empty({N, K}, dy.options());
    TORCH_CHECK(bh::gemm_tn_supported(N, K, T, dy.stride(0), x.stride(0), dy.data_ptr(), x.data_ptr(), out.data_ptr()),
                "gemm.weight_grad_tn: unsupported shape (N, K % 256, T % 64, aligned rows)");
    const int s = splits > 0 ? (int)splits : bh::gemm_tn_splits(N, K, T);
    at::Tensor ws;
    if (s > 1) ws = at::empty({(int64_t)s, N, K}, dy.options().dtype(at::kFloat));
    bh::gemm_tn(dtype_code(dy.scalar_type()), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
                N, K, T, s > 1 ? ws.data_ptr<float>() : nullptr, s, stream_for(dy));
    return out;
  }, py::arg("dy"), py::arg("x"), py::arg("splits") = 0);
  // C [M, N] = a [M, K] @ bt [K, N] (both row-major): the data gradient dY @ W on the MFMA kernel
  gm.def("mm_nn", [](at::Tensor a, at::Tensor bt, int64_t splits) {
    TORCH_CHECK(a.is_cuda() && bt.is_cuda() && a.dim() == 2 && bt.dim() == 2 && a.size(1) == bt.size(0) &&
                    a.scalar_type() == bt.scalar_type() && a.stride(1) == 1 && bt.stride(1) == 1 &&
                    (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16),
                "gemm.mm_nn: a [M, K] and bt [K, N], one 16-bit dtype, unit column stride");
    const int64_t M = a.size(0), K = a.size(1), N = bt.size(1);
    auto out = at::empty({M, N}, a.options());
    TORCH_CHECK(bh::gemm_nn_supported(M, N, K, a.stride(0), bt.stride(0), a.data_ptr(), bt.data_ptr(), out.data_ptr()),
                "gemm.mm_nn: unsupported shape (M, N % 256, K % 64, aligned rows)");
    const int s = splits > 0 ? (int)splits : bh::gemm_tn_splits(M, N, K);
    at::Tensor ws;
    if (s > 1) ws = at::empty({(int64_t)s, M, N}, a.options().dtype(at::kFloat));
    bh::gemm_nn(dtype_code(a.scalar_type()), a.data_ptr(), a.stride(0), bt.data_ptr(), bt.stride(0), out.data_ptr(), M,
                N, K, s > 1 ? ws.data_ptr<float>() : nullptr, s, stream_for(a));
    return out;
  }, py::arg("a"), py::arg("bt"), py::arg("splits") = 0);
  gm.def("mm_nn_supported", [](at::Tensor a, at::Tensor bt) {
    return a.is_cuda() && bt.is_cuda() && a.dim() == 2 && bt.dim() == 2 && a.size(1) == bt.size(0) &&
           a.scalar_type() == bt.scalar_type() && a.stride(1) == 1 && bt.stride(1) == 1 &&
           (a.scalar_type() == at::kHalf || a.scalar_type() == at::kBFloat16) &&
           bh::gemm_nn_supported(a.size(0), bt.size(1), a.size(1), a.stride(0), bt.stride(0), a.data_ptr(),
                                 bt.data_ptr(), a.data_ptr());
  }, py::arg("a"), py::arg("bt"));
  gm.def("weight_grad_tn_supported", [](at::Tensor dy, at::Tensor x) {
    return dy.is_cuda() && x.is_cuda() && dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0) &&
           dy.scalar_type() == x.scalar_type() && dy.stride(1) == 1 && x.stride(1) == 1 &&
           (dy.scalar_type() == at::kHalf || dy.scalar_type() == at::kBFloat16) &&
           bh::gemm_tn_supported(dy.size(1), x.size(1), dy.size(0), dy.stride(0), x.stride(0), dy.data_ptr(),
                                 x.data_ptr(), dy.data_ptr());
  }, py::arg("dy"), py::arg("x"));
  gm.def("mfma_enabled", &mfma_enabled);
  gm.def("set_tile_mode", &bh::gemm_set_tile_mode, "0 auto, 1 128x128, 2 256x256, 3 256x128, 4 ping-pong 256x256");
  gm.def("tile_mode", &bh::gemm_tile_mode);
  gm.def("set_force_mfma", [](bool on) { g_force_mfma = on; },
         "route every supported linear_act / linear_dact call to the MFMA kernel (no measured dispatch)");
  auto wg = root.def_submodule("fused_weight_gradient_mlp_cuda", "weight-gradient GEMM accumulated into main_grad");
  wg.def("wgrad_gemm_accum_fp32", &wgrad_gemm_accum_fp32);
  wg.def("wgrad_gemm_accum_fp16", &wgrad_gemm_accum_fp16);
}

}  // namespace bhb
