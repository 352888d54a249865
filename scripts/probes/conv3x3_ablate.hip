// Ablation probe for the direct 3x3 conv kernel (kernels/conv.hip, plain epilogue, no prologue):
// the same main loop with pieces switched off by a template mask, timed standalone with hipEvents.
// Results are NOT numerically meaningful for the ablated variants -- only the time is.
//   bit 0: epilogue stores skipped     bit 1: halo global loads skipped (LDS gets zeros)
//   bit 2: weight global loads skipped bit 3: per-step barrier skipped (chunk-end barriers kept)
//   bit 4: epilogue stores as 16-byte LDS-staged rows instead of 2-byte scatter
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 conv3x3_ablate.hip -o conv3x3_ablate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16;
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;
#define DEV __device__ __forceinline__

constexpr int kThreads = 256, kTH = 8, kBN = 64, kCK = 64, kPix = 144, kMaxHC = 40;
constexpr int kHaloBytes = (kTH + 2) * kMaxHC * kPix;
constexpr int kWBytes = kBN * 128;
constexpr int kHaloPer = ((kTH + 2) * kMaxHC * 8 + kThreads - 1) / kThreads;

struct Args { const f16* x; const f16* w; f16* y; int N, H, W, C, K; int flag; };
struct Geo { int G, gw, HC, XT, YT, tiles, tpw; };

DEV f16v mfma(i4v a, i4v b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}
DEV int wsw(int row, int ch) { return row * 128 + ((ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4); }

template <int G, int ABL>
__global__ __launch_bounds__(kThreads, 2) void k_conv(Args a, Geo g) {
  constexpr int GW = 32 / G, HC = G * (GW + 2);
  __shared__ __attribute__((aligned(16))) char smem[kHaloBytes + 2 * kWBytes];
  char* halo = smem;
  char* wb = smem + kHaloBytes;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int tile0 = blockIdx.x * g.tpw;
  const int ntile = min(g.tpw, g.tiles - tile0);
  const int k0 = blockIdx.y * kBN;
  const f16* X = a.x;
  const f16* Wt = a.w;
  const int C = a.C, H = a.H, W = a.W, N = a.N;
  const int nch = C / kCK, per_tile = nch * 9, steps = ntile * per_tile;
  constexpr int npieces = (kTH + 2) * HC * 8;
  auto origin = [&](int t, int& n0, int& y0, int& x0) {
    const int xt = t % g.XT; t /= g.XT;
    const int yt = t % g.YT;
    n0 = (t / g.YT) * G; y0 = yt * kTH; x0 = xt * 32;
  };
  i4v hreg[kHaloPer];
  uint32_t hmask = 0;
  auto halo_load = [&](int t, int c0) {
    int n0, y0, x0;
    origin(t, n0, y0, x0);
    hmask = 0;
#pragma unroll
    for (int i = 0; i < kHaloPer; ++i) {
      const int q = tid + i * kThreads, pix = q >> 3, ch = q & 7;
      const int hr = pix / HC, hc = pix - hr * HC;
      const int gi = hc / (GW + 2), jj = hc - gi * (GW + 2);
      const int n = n0 + gi, y = y0 - 1 + hr, x = x0 - 1 + jj;
      const bool ok = q < npieces && n < N && y >= 0 && y < H && x >= 0 && x < W;
      const int off = ok ? ((n * H + y) * W + x) * C + c0 + ch * 8 : 0;
      if constexpr (ABL & 2) hreg[i] = i4v{off, 0, 0, 0};
      else hreg[i] = *reinterpret_cast<const i4v*>(X + off);
      hmask |= (ok ? 1u : 0u) << i;
    }
  };
  auto halo_store = [&]() {
#pragma unroll
    for (int i = 0; i < kHaloPer; ++i) {
      const int q = tid + i * kThreads;
      if (q < npieces) *reinterpret_cast<i4v*>(halo + (q >> 3) * kPix + (q & 7) * 16) = ((hmask >> i) & 1u) ? hreg[i] : i4v{0, 0, 0, 0};
    }
  };
  i4v wr0[2], wr1[2];
  auto w_load = [&](int step, i4v(&wreg)[2]) {
    const int within = step % per_tile, chunk = within / 9, rs = within - chunk * 9;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = tid + i * kThreads, row = p >> 3, ch = p & 7;
      if constexpr (ABL & 4) wreg[i] = i4v{row, ch, rs, chunk};
      else wreg[i] = *reinterpret_cast<const i4v*>(Wt + ((k0 + row) * 9 + rs) * C + chunk * kCK + ch * 8);
    }
  };
  auto w_store = [&](char* buf, const i4v(&wreg)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) { const int p = tid + i * kThreads; *reinterpret_cast<i4v*>(buf + wsw(p >> 3, p & 7)) = wreg[i]; }
  };
  f16v acc[2][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[kb][pb][i] = 0.f;
  };
  const int gi = r32 / GW, jl = r32 - gi * GW;
  const int hcol = gi * (GW + 2) + jl;
  f16* Y = a.y;
  auto epilogue = [&](int t) {
    int n0, y0, x0;
    origin(t, n0, y0, x0);
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
      const int y = y0 + 2 * wave + pb;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int pp = 8 * (v >> 2) + 4 * h + (v & 3);
        const int gp = pp / GW, xp = pp - gp * GW;
        const int n = n0 + gp, x = x0 + xp;
        if (y >= H || n >= N || x >= W) continue;
        const int off = ((n * H + y) * W + x) * a.K + k0 + r32;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          if ((ABL & 1) && !a.flag) continue;
          Y[off + 32 * kb] = (f16)acc[kb][pb][v];
        }
      }
    }
  };
  zero_acc();
  halo_load(tile0, 0);
  w_load(0, wr0);
  halo_store();
  w_store(wb, wr0);
  if (steps > 1) w_load(1, wr1);
  __syncthreads();
  auto step_body = [&](int t, i4v(&nxt2)[2], const i4v(&nxt)[2]) {
    const int it = t / per_tile, within = t - it * per_tile;
    const int chunk = within / 9, rs = within - chunk * 9;
    const bool last_rs = rs == 8;
    const bool more = chunk + 1 < nch || it + 1 < ntile;
    if (t + 2 < steps) w_load(t + 2, nxt2);
    if (rs == 0 && more) {
      if (chunk + 1 < nch) halo_load(tile0 + it, (chunk + 1) * kCK);
      else halo_load(tile0 + it + 1, 0);
    }
    const char* wcur = wb + (t & 1) * kWBytes;
    const int r = rs / 3, s = rs - r * 3;
    const char* hb0 = halo + ((2 * wave + r) * HC + hcol + s) * kPix;
    const char* hb1 = hb0 + HC * kPix;
    auto frags = [&](int kk, i4v (&f)[4]) {
      const int ch = 2 * kk + h;
      f[0] = *reinterpret_cast<const i4v*>(wcur + wsw(r32, ch));
      f[1] = *reinterpret_cast<const i4v*>(wcur + wsw(32 + r32, ch));
      f[2] = *reinterpret_cast<const i4v*>(hb0 + ch * 16);
      f[3] = *reinterpret_cast<const i4v*>(hb1 + ch * 16);
    };
    i4v fa[4], fb[4];
    frags(0, fa);
#pragma unroll
    for (int kk = 0; kk < 4; kk += 2) {
      frags(kk + 1, fb);
      acc[0][0] = mfma(fa[2], fa[0], acc[0][0]);
      acc[0][1] = mfma(fa[3], fa[0], acc[0][1]);
      acc[1][0] = mfma(fa[2], fa[1], acc[1][0]);
      acc[1][1] = mfma(fa[3], fa[1], acc[1][1]);
      if (kk + 2 < 4) frags(kk + 2, fa);
      acc[0][0] = mfma(fb[2], fb[0], acc[0][0]);
      acc[0][1] = mfma(fb[3], fb[0], acc[0][1]);
      acc[1][0] = mfma(fb[2], fb[1], acc[1][0]);
      acc[1][1] = mfma(fb[3], fb[1], acc[1][1]);
    }
    if (t + 1 < steps) w_store(wb + ((t + 1) & 1) * kWBytes, nxt);
    if (last_rs && chunk + 1 == nch) { epilogue(tile0 + it); zero_acc(); }
    if (last_rs && more) { __syncthreads(); halo_store(); }
    if constexpr (ABL & 8) { if (last_rs) __syncthreads(); } else __syncthreads();
  };
  for (int t = 0; t < steps; t += 2) {
    step_body(t, wr0, wr1);
    if (t + 1 < steps) step_body(t + 1, wr1, wr0);
  }
}

Geo make_geo(int H, int W, int N, int K) {
  Geo g; g.G = 1;
  while (g.G < 4 && 32 / (2 * g.G) >= W) g.G *= 2;
  g.gw = 32 / g.G; g.HC = g.G * (g.gw + 2);
  g.XT = g.G == 1 ? (W + 31) / 32 : 1;
  g.YT = (H + kTH - 1) / kTH;
  g.tiles = g.XT * g.YT * ((N + g.G - 1) / g.G);
  const long ktiles = K / kBN;
  g.tpw = (int)std::max<long>(1, (g.tiles * ktiles + 511) / 512);
  return g;
}

template <int G, int ABL> float run(Args a, Geo g, hipStream_t st) {
  dim3 grid((g.tiles + g.tpw - 1) / g.tpw, a.K / kBN);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_conv<G, ABL>), grid, dim3(kThreads), 0, st, a, g);
  hipEventRecord(e0, st);
  const int it = 30;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_conv<G, ABL>), grid, dim3(kThreads), 0, st, a, g);
  hipEventRecord(e1, st); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / it;
}

template <int G> void shape(int C, int HW) {
  const int N = 256, K = C;
  size_t nx = (size_t)N * HW * HW * C, nw = (size_t)K * 9 * C;
  std::vector<f16> hx(nx), hw(nw);
  for (size_t i = 0; i < nx; ++i) hx[i] = (f16)((rand() % 2001 - 1000) * 1e-3f);
  for (size_t i = 0; i < nw; ++i) hw[i] = (f16)((rand() % 2001 - 1000) * 1e-5f);
  f16 *x, *w, *y;
  hipMalloc(&x, nx * 2); hipMalloc(&w, nw * 2); hipMalloc(&y, nx * 2);
  hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice);
  Args a{x, w, y, N, HW, HW, C, K, 0};
  Geo g = make_geo(HW, HW, N, K);
  const double fl = 2.0 * N * HW * HW * C * K * 9;
  auto rep = [&](const char* name, float ms) { printf("C=%d HW=%d G=%d %-22s %.4f ms %.0f TF/s\n", C, HW, G, name, ms, fl / ms / 1e9); };
  rep("base", run<G, 0>(a, g, 0));
  rep("no_store", run<G, 1>(a, g, 0));
  rep("no_halo_load", run<G, 2>(a, g, 0));
  rep("no_w_load", run<G, 4>(a, g, 0));
  rep("no_step_barrier", run<G, 8>(a, g, 0));
  rep("no_loads_no_store", run<G, 7>(a, g, 0));
  rep("all_off", run<G, 15>(a, g, 0));
  hipFree(x); hipFree(w); hipFree(y);
}

int main() {
  shape<1>(64, 56);
  shape<1>(128, 28);
  shape<2>(256, 14);
  shape<4>(512, 7);
  return 0;
}
