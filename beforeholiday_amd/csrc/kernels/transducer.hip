// RNN-T (transducer) loss on gfx950: forward-backward lattice recursions + fused gradient.
//
// Reference behaviour: apex/contrib/csrc/transducer/transducer_loss_kernel.cu (alpha / beta over the
// (t, u) lattice from log-softmax inputs, loss = -log P(y|x), gradient optionally fused with the
// log-softmax backward; packed or padded [B, T, U+1, V] inputs) and the python reference
// apex/contrib/transducer/_transducer_ref.py.
//
// MI355X design:
//  * alpha and beta: one workgroup per sequence walks the lattice by anti-diagonals (t + u = n);
//    the nodes of a diagonal are independent, so the workgroup's lanes take them in parallel and
//    one barrier separates diagonals. Only the blank and label log-probs of each node are read.
//  * gradient: one workgroup per lattice node (row of V log-probs), 16-byte vectors; with
//    fuse_softmax_backward the softmax backward is applied in the same pass, so the [.., V]
//    tensor is read once and written once.
#include "bh/api.h"
#include "bh/device.h"
#include "bh/transducer_api.h"

#include <stdexcept>
#include <string>

namespace bh {
namespace {

constexpr int kBlock = 256;

#define TD_DISPATCH(code, T, ...)                                          \
  switch (code) {                                                          \
    case kF32: { using T = float; __VA_ARGS__; } break;                    \
    case kF16: { using T = f16; __VA_ARGS__; } break;                      \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("transducer: unsupported dtype " + std::to_string(code)); \
  }

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

BH_DEVICE float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + log1pf(__expf(-fabsf(a - b)));
}

struct Geo {
  const int* f_len;
  const int* y_len;
  const int64_t* batch_offset;  // packed: cumulative f_len*(y_len+1); null when padded
  int max_t, max_u1;            // padded geometry (U+1)
};

// row index of lattice node (b, t, u) in the [rows, V] view of x
BH_DEVICE int64_t node_row(const Geo& g, int b, int t, int u) {
  if (g.batch_offset) {
    const int64_t start = b == 0 ? 0 : g.batch_offset[b - 1];
    return start + (int64_t)t * (g.y_len[b] + 1) + u;
  }
  return ((int64_t)b * g.max_t + t) * g.max_u1 + u;
}

// alpha[b][t][u] / beta[b][t][u] stored padded [B, max_t, max_u1]
template <typename T>
__global__ __launch_bounds__(kBlock) void k_alpha_beta(const T* __restrict__ x, const int64_t* __restrict__ label,
                                                       int label_stride, Geo g, int V, int blank,
                                                       float* __restrict__ alpha, float* __restrict__ beta,
                                                       float* __restrict__ loss) {
  const int b = blockIdx.x;
  const bool do_beta = blockIdx.y == 1;
  const int Tb = g.f_len[b], Ub = g.y_len[b];  // nodes t in [0, Tb), u in [0, Ub]
  float* A = (do_beta ? beta : alpha) + (int64_t)b * g.max_t * g.max_u1;
  const int64_t* lab = label + (int64_t)b * label_stride;
  if (Tb <= 0) {
    if (threadIdx.x == 0 && !do_beta) loss[b] = INFINITY;
    return;
  }
  for (int n = 0; n <= Tb - 1 + Ub; ++n) {
    const int d = do_beta ? (Tb - 1 + Ub - n) : n;  // diagonal index t + u
    const int u_lo = max(0, d - (Tb - 1)), u_hi = min(Ub, d);
    for (int u = u_lo + (int)threadIdx.x; u <= u_hi; u += kBlock) {
      const int t = d - u;
      float v;
      if (!do_beta) {
        if (t == 0 && u == 0) {
          v = 0.f;
        } else {
          float a = -INFINITY, c = -INFINITY;
          if (t > 0) a = A[(t - 1) * g.max_u1 + u] + to_f<T>(x[node_row(g, b, t - 1, u) * V + blank]);
          if (u > 0) c = A[t * g.max_u1 + u - 1] + to_f<T>(x[node_row(g, b, t, u - 1) * V + lab[u - 1]]);
          v = lse2(a, c);
        }
      } else {
        const float xb = to_f<T>(x[node_row(g, b, t, u) * V + blank]);
        if (t == Tb - 1 && u == Ub) {
          v = xb;
        } else {
          float a = -INFINITY, c = -INFINITY;
          if (t < Tb - 1) a = A[(t + 1) * g.max_u1 + u] + xb;
          if (u < Ub) c = A[t * g.max_u1 + u + 1] + to_f<T>(x[node_row(g, b, t, u) * V + lab[u]]);
          v = lse2(a, c);
        }
      }
      A[t * g.max_u1 + u] = v;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (do_beta) {
      loss[b] = -A[0];
    }
  }
}

// grad wrt x (log-probs) or, fused, wrt the logits of the log-softmax
template <typename T>
__global__ __launch_bounds__(kBlock) void k_grad(const T* __restrict__ x, const float* __restrict__ loss_grad,
                                                 const float* __restrict__ alpha, const float* __restrict__ beta,
                                                 const int64_t* __restrict__ label, int label_stride, Geo g, int V,
                                                 int blank, bool fuse_softmax, T* __restrict__ dx, int B) {
  // blockIdx.x enumerates padded nodes (b, t, u); padded layouts also zero the invalid rows
  const int64_t node = blockIdx.x;
  const int u = (int)(node % g.max_u1);
  const int t = (int)((node / g.max_u1) % g.max_t);
  const int b = (int)(node / ((int64_t)g.max_u1 * g.max_t));
  const int Tb = g.f_len[b], Ub = g.y_len[b];
  const bool valid = t < Tb && u <= Ub;
  if (!valid) {
    if (g.batch_offset) return;  // packed: the row does not exist
    T* out = dx + node_row(g, b, t, u) * V;
    for (int v = threadIdx.x; v < V; v += kBlock) out[v] = from_f<T>(0.f);
    return;
  }
  const int64_t row = node_row(g, b, t, u);
  const T* xr = x + row * V;
  T* out = dx + row * V;
  const float* Ab = alpha + (int64_t)b * g.max_t * g.max_u1;
  const float* Bb = beta + (int64_t)b * g.max_t * g.max_u1;
  const float ll = Bb[0];  // log P(y | x)
  const float scale = -loss_grad[b];
  const float a = Ab[t * g.max_u1 + u];
  const float occ = __expf(a + Bb[t * g.max_u1 + u] - ll);  // posterior occupancy of the node
  const int lab = u < Ub ? (int)label[(int64_t)b * label_stride + u] : -1;
  float g_blank, g_lab = 0.f;
  {
    const float xb = to_f<T>(xr[blank]);
    if (t == Tb - 1 && u == Ub) g_blank = __expf(a + xb - ll);
    else if (t < Tb - 1) g_blank = __expf(a + Bb[(t + 1) * g.max_u1 + u] + xb - ll);
    else g_blank = 0.f;
    if (lab >= 0) g_lab = __expf(a + Bb[t * g.max_u1 + u + 1] + to_f<T>(xr[lab]) - ll);
  }
  for (int v = threadIdx.x; v < V; v += kBlock) {
    float d = 0.f;
    if (v == blank) d += g_blank;
    if (v == lab) d += g_lab;
    if (fuse_softmax) d -= __expf(to_f<T>(xr[v])) * occ;
    out[v] = from_f<T>(scale * d);
  }
}

}  // namespace

void transducer_loss_forward(int dt, const void* x, const int64_t* label, int label_stride, const int* f_len,
                             const int* y_len, const int64_t* batch_offset, int B, int max_t, int max_u1, int V,
                             int blank, float* alpha, float* beta, float* loss, hipStream_t st) {
  if (B == 0) return;
  Geo g{f_len, y_len, batch_offset, max_t, max_u1};
  TD_DISPATCH(dt, T, hipLaunchKernelGGL((k_alpha_beta<T>), dim3(B, 2), dim3(kBlock), 0, st, (const T*)x, label,
                                        label_stride, g, V, blank, alpha, beta, loss));
  check_launch("transducer_loss_forward");
}

void transducer_loss_backward(int dt, const void* x, const float* loss_grad, const float* alpha, const float* beta,
                              const int64_t* label, int label_stride, const int* f_len, const int* y_len,
                              const int64_t* batch_offset, int B, int max_t, int max_u1, int V, int blank,
                              bool fuse_softmax, void* dx, hipStream_t st) {
  const int64_t nodes = (int64_t)B * max_t * max_u1;
  if (nodes == 0) return;
  Geo g{f_len, y_len, batch_offset, max_t, max_u1};
  TD_DISPATCH(dt, T, hipLaunchKernelGGL((k_grad<T>), dim3((unsigned)nodes), dim3(kBlock), 0, st, (const T*)x,
                                        loss_grad, alpha, beta, label, label_stride, g, V, blank, fuse_softmax, (T*)dx,
                                        B));
  check_launch("transducer_loss_backward");
}

}  // namespace bh

// ==========================================================================================
// RNN-T joint (reference: apex/contrib/csrc/transducer/transducer_joint_kernel.cu:177-845)
//
// MI355X design: a workgroup owns one (b, t) encoder row and a tile of kJointU prediction rows; each
// lane keeps its 8-element slice of f in registers and streams g / out in 16-byte vectors, so f is
// read once per tile and the [B, T, U, H] broadcast is never materialised. ReLU + dropout are fused;
// dropout bits are a keyed counter hash of the element index (no RNG state, no mask tensor), the
// backward regenerates them. The two backward reductions (sum over U for df, over T for dg) are
// separate deterministic passes, one workgroup per output row (no atomics).
// ==========================================================================================
#include "bh/transducer_api.h"

namespace bh {
namespace {

constexpr int kJointU = 4;       // prediction rows per forward workgroup
constexpr int kJointBlock = 256;

BH_DEVICE uint32_t jmix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}
BH_DEVICE uint32_t joint_hash(uint32_t seed, uint64_t i) {
  const uint32_t k = jmix(seed * 0x9E3779B9u + 0x632BE5ABu);
  return jmix(jmix((uint32_t)i ^ k) + k * 0x85EBCA6Bu + (uint32_t)(i >> 32) * 0xC2B2AE35u);
}

BH_DEVICE int64_t joint_row(const JointArgs& a, int b, int t, int u) {
  if (a.batch_offset) return (b ? a.batch_offset[b - 1] : 0) + (int64_t)t * a.g_len[b] + u;
  return ((int64_t)b * a.T + t) * a.U + u;
}

template <typename T>
__global__ __launch_bounds__(kJointBlock) void k_joint_fwd(JointArgs a, const T* __restrict__ f, const T* __restrict__ g,
                                                           T* __restrict__ out, uint8_t* __restrict__ mask) {
  const int bt = blockIdx.x;
  const int b = bt / a.T, t = bt % a.T;
  const int u0 = blockIdx.y * kJointU;
  const int fl = min(a.f_len[b], a.T), gl = min(a.g_len[b], a.U);  // lengths clamped to the tensors
  const bool packed = a.batch_offset != nullptr;
  const bool trow = t < fl;
  if (packed && (!trow || u0 >= gl)) return;  // nothing of this tile exists in the packed output
  const int H8 = a.H / 8;
  for (int c = threadIdx.x; c < H8; c += kJointBlock) {
    float fv[8];
    if (trow) VecIO<T>::load(f + ((int64_t)b * a.T + t) * a.H + c * 8, fv);
#pragma unroll
    for (int j = 0; j < kJointU; ++j) {
      const int u = u0 + j;
      if (u >= a.U || (packed && u >= gl)) break;
      const int64_t row = joint_row(a, b, t, u);
      if (row < 0 || row >= a.rows) continue;  // inconsistent batch_offset: never write out of bounds
      float o[8];
      uint32_t bits = 0u;
      if (trow && u < gl) {
        float gv[8];
        VecIO<T>::load(g + ((int64_t)b * a.U + u) * a.H + c * 8, gv);
        const uint64_t e0 = (((uint64_t)b * a.T + t) * a.U + u) * (uint64_t)a.H + (uint64_t)c * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float h = fv[k] + gv[k];
          bool keep = true;
          if (a.relu && !(h > 0.f)) keep = false;
          if (a.dropout && joint_hash(a.seed, e0 + k) < a.keep_thresh) keep = false;
          o[k] = keep ? (a.dropout ? h * a.scale : h) : 0.f;
          bits |= (uint32_t)keep << k;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = 0.f;  // padded output: invalid rows are zero
      }
      VecIO<T>::store(out + row * a.H + c * 8, o);
      if (mask) {
#pragma unroll
        for (int k = 0; k < 8; ++k) mask[row * a.H + c * 8 + k] = (uint8_t)((bits >> k) & 1u);
      }
    }
  }
}

// gradient factor of element (b, t, u, h) given its output value
template <typename T>
BH_DEVICE void joint_grad_mask(const JointArgs& a, const T* out, int64_t row, int b, int t, int u, int c,
                               float (&gr)[8]) {
  if (a.relu) {
    float ov[8];
    VecIO<T>::load(out + row * a.H + c * 8, ov);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (!(ov[k] > 0.f)) gr[k] = 0.f;  // out > 0  <=>  h > 0 and kept
  } else if (a.dropout) {
    const uint64_t e0 = (((uint64_t)b * a.T + t) * a.U + u) * (uint64_t)a.H + (uint64_t)c * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (joint_hash(a.seed, e0 + k) < a.keep_thresh) gr[k] = 0.f;
  }
  if (a.dropout) {
#pragma unroll
    for (int k = 0; k < 8; ++k) gr[k] *= a.scale;
  }
}

// df(b, t, :) = sum_u grad'(b, t, u, :)
template <typename T>
__global__ __launch_bounds__(kJointBlock) void k_joint_bwd_f(JointArgs a, const T* __restrict__ grad,
                                                             const T* __restrict__ out, T* __restrict__ df) {
  const int bt = blockIdx.x;
  const int b = bt / a.T, t = bt % a.T;
  const int fl = min(a.f_len[b], a.T), gl = min(a.g_len[b], a.U);
  const int H8 = a.H / 8;
  for (int c = threadIdx.x; c < H8; c += kJointBlock) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t < fl) {
      for (int u = 0; u < gl; ++u) {
        const int64_t row = joint_row(a, b, t, u);
        if (row < 0 || row >= a.rows) continue;
        float gr[8];
        VecIO<T>::load(grad + row * a.H + c * 8, gr);
        joint_grad_mask(a, out, row, b, t, u, c, gr);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += gr[k];
      }
    }
    VecIO<T>::store(df + ((int64_t)b * a.T + t) * a.H + c * 8, acc);
  }
}

// dg(b, u, :) = sum_t grad'(b, t, u, :)
template <typename T>
__global__ __launch_bounds__(kJointBlock) void k_joint_bwd_g(JointArgs a, const T* __restrict__ grad,
                                                             const T* __restrict__ out, T* __restrict__ dg) {
  const int bu = blockIdx.x;
  const int b = bu / a.U, u = bu % a.U;
  const int fl = min(a.f_len[b], a.T), gl = min(a.g_len[b], a.U);
  const int H8 = a.H / 8;
  for (int c = threadIdx.x; c < H8; c += kJointBlock) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (u < gl) {
      for (int t = 0; t < fl; ++t) {
        const int64_t row = joint_row(a, b, t, u);
        if (row < 0 || row >= a.rows) continue;
        float gr[8];
        VecIO<T>::load(grad + row * a.H + c * 8, gr);
        joint_grad_mask(a, out, row, b, t, u, c, gr);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += gr[k];
      }
    }
    VecIO<T>::store(dg + ((int64_t)b * a.U + u) * a.H + c * 8, acc);
  }
}

#define JOINT_DISPATCH(code, T, ...)                                      \
  switch (code) {                                                         \
    case kF32: { using T = float; __VA_ARGS__; } break;                   \
    case kF16: { using T = f16; __VA_ARGS__; } break;                     \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;                   \
    default: throw std::runtime_error("transducer_joint: unsupported dtype " + std::to_string(code)); \
  }

}  // namespace

void transducer_joint_forward(const JointArgs& a, int dt, const void* f, const void* g, void* out, uint8_t* mask,
                              hipStream_t st) {
  if (a.B == 0 || a.T == 0 || a.U == 0 || a.H == 0) return;
  if (a.H % 8) throw std::runtime_error("transducer_joint: hidden size must be a multiple of 8");
  const dim3 grid(a.B * a.T, (a.U + kJointU - 1) / kJointU);
  JOINT_DISPATCH(dt, T,
      hipLaunchKernelGGL((k_joint_fwd<T>), grid, dim3(kJointBlock), 0, st, a, (const T*)f, (const T*)g, (T*)out, mask));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("transducer_joint_forward: ") + hipGetErrorString(e));
}

void transducer_joint_backward(const JointArgs& a, int dt, const void* grad, const void* out, void* df, void* dg,
                               hipStream_t st) {
  if (a.B == 0 || a.T == 0 || a.U == 0 || a.H == 0) return;
  if (a.H % 8) throw std::runtime_error("transducer_joint: hidden size must be a multiple of 8");
  JOINT_DISPATCH(dt, T, {
      hipLaunchKernelGGL((k_joint_bwd_f<T>), dim3(a.B * a.T), dim3(kJointBlock), 0, st, a, (const T*)grad,
                         (const T*)out, (T*)df);
      hipLaunchKernelGGL((k_joint_bwd_g<T>), dim3(a.B * a.U), dim3(kJointBlock), 0, st, a, (const T*)grad,
                         (const T*)out, (T*)dg);
  });
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("transducer_joint_backward: ") + hipGetErrorString(e));
}

}  // namespace bh
