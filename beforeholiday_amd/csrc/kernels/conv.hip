// Direct 3x3 / stride 1 / pad 1 NHWC convolution on MFMA 32x32x16 (gfx950): see bh/conv_api.h.
//
// Implicit GEMM with the output channel on the MFMA row and the output pixel on the lane:
//   acc[k_out, pixel] += W[k_out, r, s, c] * X[pixel + (r-1, s-1), c]
// Workgroup = 4 waves = an 8-row x 32-lane window of output pixels x 64 output channels; wave w owns
// window rows 2w, 2w+1 (two 32x32 accumulator tiles per 32 output channels). The 32 lanes of a row
// are 32 consecutive columns of one image (W >= 32: W / 32 column tiles), or G = 2 / 4 images side
// by side with 16 / 8 lanes each (W <= 16 / 8), so a 14x14 or 7x7 layer still fills the lanes.
// Per 64-channel input chunk the window's halo (10 rows x (lanes + 2 per image) pixels, zero outside
// the image) is staged in LDS once -- 144-byte pixel slots keep the 32-pixel fragment reads bank-
// conflict free -- and read at all nine (r, s) offsets (each input pixel leaves HBM / L2 ~1.3 times
// instead of 9); the 64x64 weight slice of each (r, s) streams through a double buffer (register
// prefetch, one barrier per offset), and the next chunk's halo is prefetched into registers while
// the current chunk computes. Loads are issued unconditionally on clamped addresses and zeroed when
// written to LDS, so no select waits on a load in front of the MFMAs.
#include "bh/api.h"
#include "bh/conv_api.h"
#include "bh/knobs.h"
#include "bh/device.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <stdexcept>
#include <string>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;

template <typename T> struct Mfma32;
template <> struct Mfma32<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0,
                                                   0);
  }
};

constexpr int kThreads = 256;
constexpr int kTH = 8;      // output rows per window (2 per wave)
constexpr int kBN = 64;     // output channels per workgroup
constexpr int kCK = 64;     // input channels per chunk
constexpr int kPix = 144;   // LDS bytes per halo pixel: 128 data + 16 pad
constexpr int kMaxHC = 40;  // halo columns G * (lanes per image + 2) <= 40
constexpr int kWBytes = kBN * 128;
constexpr int kMaxProC = 512;                 // input channels the BatchNorm prologue covers
constexpr int kProBytes = 2 * kMaxProC * 4;   // its scale / shift in LDS
constexpr int kOutOfRange = 0x7ff00000;       // a byte offset past every tensor the kernel reads

struct Geo {
  int G, gw, HC, XT, YT, tiles, tpw;  // tpw: consecutive windows per workgroup
};

// 64 x 128-byte weight image, swizzled for the 32-row fragment reads (ds_read_b128) and for the
// 4-row column reads (ds_read_b64_tr_b16) alike
BH_DEVICE int wsw(int row, int ch) { return row * 128 + ((ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4); }

// A operand from a [k rows][m columns] image: lane (m = m0 + (lane & 31), half h) gets image rows
// r0 .. r0 + 7 of its column (r0 already includes 8h), two transposed 4-row reads
BH_DEVICE i4v frag_tr(const char* img, int r0, int m0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = m0 + 16 * (g & 1) + 4 * p;
  const int cb = (col & 7) << 1;
  const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + wsw(r0 + q, col >> 3) + cb));
  const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + wsw(r0 + 4 + q, col >> 3) + cb));
  typedef int i2v __attribute__((ext_vector_type(2)));
  const i2v l = __builtin_bit_cast(i2v, lo), hh = __builtin_bit_cast(i2v, hi);
  return i4v{l[0], l[1], hh[0], hh[1]};
}

// FLIP: the data gradient of conv(x, w): input dY [N, H, W, K_w], weights given as the forward's
// w [K_w][3][3][C_w], computing conv with W'[c][r][s][k] = w[k][2-r][2-s][c]. The slice of each
// step is then a [k_w rows][c_w contiguous] block of w, staged as it lies and read as the MFMA A
// operand through ds_read_b64_tr_b16 -- no transposed weight copy is ever materialised.
template <typename T, bool FLIP, int G, bool PRO, int EPI, int NB_ = 3, bool SW_ = true>
__global__ __launch_bounds__(kThreads, 2) void k_conv3x3(Conv3x3Args a, Geo g) {
  // window geometry as compile-time constants (the halo address math divides by them)
  constexpr int GW = 32 / G, HC = G * (GW + 2);
  // the plain epilogue stores from the transposed accumulator layout (8-byte channel runs per lane); the
  // statistics epilogues keep the pixel-per-register layout (their per-channel sums stay in-lane)
  constexpr bool SW = SW_ && EPI == kConvEpiPlain;
  // weight-slice buffers: 3 where the LDS budget of two workgroups per CU allows (the next step's first
  // fragments are then read BEFORE the barrier that ends a step), 2 for the 40-column G = 4 halo
  constexpr int NB = G == 1 ? NB_ : 2;
  // halo row stride and the byte shift of each image block: with G images side by side the 16-lane
  // groups of ds_read_b128 ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, + 32) span two images, and at the
  // plain 144-byte slot pitch image 1's pixels land on image 0's banks (2-way at G = 2, 3-way at G = 4).
  // Block b = pix / (GW + 2) of the halo (image b % G of row b / G) is shifted by b * kImgShift bytes:
  // 224 B makes every group conflict free at G = 2; at G = 4 that would not fit two workgroups' LDS,
  // 32 B leaves 2-way (exhaustive search over the shifts).
  constexpr int kImgShift = G == 2 ? 224 : G == 4 ? 32 : 0;
  constexpr int RS = HC * kPix + G * kImgShift;
  constexpr int kHaloB = (kTH + 2) * RS;
  __shared__ __attribute__((aligned(16))) char smem[kHaloB + NB * kWBytes + (PRO ? kProBytes : 0)];
  char* halo = smem;
  char* wb = smem + kHaloB;
  float* ss = reinterpret_cast<float*>(smem + kHaloB + NB * kWBytes);  // PRO: scale[C], shift[C]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int tile0 = blockIdx.x * g.tpw;
  const int ntile = min(g.tpw, g.tiles - tile0);
  const int k0 = blockIdx.y * kBN;
  const T* X = reinterpret_cast<const T*>(a.x);
  const T* Wt = reinterpret_cast<const T*>(a.w);
  const int C = a.C, H = a.H, W = a.W, N = a.N;
  const int nch = C / kCK;
  constexpr int npieces = (kTH + 2) * HC * 8;
  constexpr int kHaloPer = (npieces + kThreads - 1) / kThreads;  // 16-byte halo pieces per thread: 11 / 12 / 13
  if constexpr (PRO) {
    for (int c = tid; c < C; c += kThreads) {
      ss[c] = a.pro_scale[c];
      ss[kMaxProC + c] = a.pro_shift[c];
    }
    // the first halo_store below reads channels other threads (other waves) wrote: without this
    // barrier a wave could normalise its first halo with stale LDS (round 3's run-to-run and
    // rank-to-rank differences, tests/test_determinism.py)
    __syncthreads();
  }
  // window origin of tile id t: x-tile fastest, then row window, then image group
  auto origin = [&](int t, int& n0, int& y0, int& x0) __attribute__((always_inline)) {
    const int xt = t % g.XT;
    t /= g.XT;
    const int yt = t % g.YT;
    n0 = (t / g.YT) * G;
    y0 = yt * kTH;
    x0 = xt * 32;
  };

  // ---- halo staging: registers (prefetch) -> LDS ----
  // Buffer loads through a whole-tensor resource: a padding pixel gets an offset past the tensor and
  // comes back as zeros (no select at the LDS store), the per-lane offset is 32-bit.
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X), (short)0, (int)((int64_t)N * H * W * C * 2), 0x00020000);
  i4v hreg[kHaloPer];
  uint32_t hmask = 0;  // PRO: in-image pieces (the prologue must not turn the zero padding into relu(shift))
  int hc0 = 0;  // first input channel of the staged chunk (the prologue's scale / shift)
  auto halo_load = [&](int t, int c0) __attribute__((always_inline)) {
    int n0, y0, x0;
    origin(t, n0, y0, x0);
    hc0 = c0;
    // the piece coordinates below depend on the thread only; hoisted out of the chunk loop they would
    // hold ~2 VGPRs per piece across the whole loop (it spilled them, and every scratch reload is a
    // vmcnt(0)): the empty asm makes them look per-chunk, so they are recomputed (~10 VALU per piece)
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int i = 0; i < kHaloPer; ++i) {
      const int q = tq + i * kThreads, pix = q >> 3, ch = q & 7;
      const int hr = pix / HC, hc = pix - hr * HC;
      const int gi = hc / (GW + 2), jj = hc - gi * (GW + 2);
      const int n = n0 + gi, y = y0 - 1 + hr, x = x0 - 1 + jj;
      const bool ok = q < npieces && n < N && y >= 0 && y < H && x >= 0 && x < W;
      const int off = ok ? (((n * H + y) * W + x) * C + c0 + ch * 8) * 2 : kOutOfRange;
      hreg[i] = __builtin_amdgcn_raw_buffer_load_b128(rsX, off, 0, 0);
      if constexpr (PRO) hmask = (hmask & ~(1u << i)) | ((ok ? 1u : 0u) << i);
    }
  };
  auto halo_store = [&]() __attribute__((always_inline)) {
    float sc[8], sh[8];
    if constexpr (PRO) {
      // BatchNorm + ReLU of the producing layer on the staged input; this thread's pieces all hold
      // channels hc0 + 8 (tid & 7) .. + 7 (kThreads is a multiple of 8). Padding stays zero: it pads
      // the normalised activation, not the raw input.
      const int cb = hc0 + 8 * (tid & 7);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[j] = ss[cb + j];
        sh[j] = ss[kMaxProC + cb + j];
      }
    }
#pragma unroll
    for (int i = 0; i < kHaloPer; ++i) {
      const int q = tid + i * kThreads;
      if (q < npieces) {
        i4v v = hreg[i];
        if constexpr (PRO) {
          typedef T t8 __attribute__((ext_vector_type(8)));
          t8 e = __builtin_bit_cast(t8, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = from_f<T>(fmaxf(fmaf(to_f<T>(e[j]), sc[j], sh[j]), 0.f));
          v = ((hmask >> i) & 1u) ? __builtin_bit_cast(i4v, e) : i4v{0, 0, 0, 0};
        }
        const int pix = q >> 3;
        *reinterpret_cast<i4v*>(halo + pix * kPix + (pix / (GW + 2)) * kImgShift + (q & 7) * 16) = v;
      }
    }
  };
  // ---- weight slice of step (chunk, r * 3 + s): W[k0 .. k0+63][r][s][c0 .. c0+63] ----
  // Three register slots, two steps of lookahead: the slice of step t + 2 is requested at the start of
  // step t and written to LDS at the end of step t + 1, so an L2 round trip (longer than one step's
  // 16 MFMAs per wave) never sits between the barrier of one step and the MFMAs of the next.
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Wt), (short)0, (int)((int64_t)a.K * 9 * C * 2), 0x00020000);
  // per-lane part of the slice offsets (the (chunk, rs) part is uniform)
  int wvoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + i * kThreads, row = p >> 3, ch = p & 7;
    wvoff[i] = FLIP ? (row * 9 * a.K + k0 + ch * 8) * 2 : ((k0 + row) * 9 * C + ch * 8) * 2;
  }
  auto w_load = [&](int chunk, int rs, i4v(&wreg)[2]) __attribute__((always_inline)) {
    // FLIP: image row = input channel c (= w's output channel), 64 contiguous k
    const int so = FLIP ? (chunk * kCK * 9 + (8 - rs)) * a.K * 2 : (rs * C + chunk * kCK) * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wvoff[i] + so, 0, 0);
  };
  auto w_store = [&](char* buf, const i4v(&wreg)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = tid + i * kThreads;
      *reinterpret_cast<i4v*>(buf + wsw(p >> 3, p & 7)) = wreg[i];
    }
  };

  f16v acc[2][2];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[kb][pb][i] = 0.f;
  };
  const int gi = r32 / GW, jl = r32 - gi * GW;
  const int hlane = (gi * (GW + 2) + jl) * kPix + gi * kImgShift;  // this lane's halo pixel at s = 0
  T* Y = reinterpret_cast<T*>(a.y);
  // the pixel-per-register epilogues store through a buffer resource: a 32-bit byte offset per store instead
  // of 64-bit address math (conv3x3_supported keeps N H W K * 2 below kOutOfRange)
  const __amdgpu_buffer_rsrc_t rsY =
      __builtin_amdgcn_make_buffer_rsrc(Y, (short)0, (int)((int64_t)N * H * W * a.K * 2), 0x00020000);
  const T* BY = reinterpret_cast<const T*>(a.by);
  // Output tile of the wave, D[pixel][channel] (the MFMA's A operand is the halo, B the weights):
  // lane (r32, h) holds channel k0 + 32 kb + r32 of pixels 8 (v >> 2) + 4 h + (v & 3) of window row
  // 2 wave + pb in acc[kb][pb][v]. Stores are 64-byte channel runs of one pixel; the per-channel
  // statistics stay in 2 x 2 registers per lane for the whole workgroup.
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, e0[2] = {0.f, 0.f}, e1[2] = {0.f, 0.f}, e2[2] = {0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int ch = k0 + 32 * kb + r32;
    if constexpr (EPI == kConvEpiStats) {
      e0[kb] = a.kshift ? a.kshift[ch] : 0.f;
    } else if constexpr (EPI == kConvEpiAffine) {
      e0[kb] = a.a_scale[ch];
      e1[kb] = a.a_shift[ch];
    } else if constexpr (EPI == kConvEpiBwd) {
      e0[kb] = a.bscale[ch];
      e1[kb] = a.bshift[ch];
      e2[kb] = a.bmean[ch];
    }
  }
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    int n0, y0, x0;
    origin(t, n0, y0, x0);
    if constexpr (SW) {
      // swapped operands: lane (r32, h) holds pixel r32 of window row 2 wave + pb, channels
      // k0 + 32 kb + 8 g + 4 h .. + 3 in acc[kb][pb][4 g .. 4 g + 3]: one 8-byte store per 4 channels
      // (16 stores per wave and window instead of 64 2-byte ones)
      typedef T t4 __attribute__((ext_vector_type(4)));
      const int gp = r32 / GW, xp = r32 - gp * GW;
      const int n = n0 + gp, x = x0 + xp;
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        const int y = y0 + 2 * wave + pb;
        if (y >= H || n >= N || x >= W) continue;
        const int off = ((n * H + y) * W + x) * a.K + k0 + 4 * h;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            t4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = from_f<T>(acc[kb][pb][4 * g + i]);
            *reinterpret_cast<t4*>(Y + off + 32 * kb + 8 * g) = o;
          }
      }
      return;
    }
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
          float xv = acc[kb][pb][v];
          if constexpr (EPI == kConvEpiAffine) {
            // conv + bias / frozen BatchNorm (+ residual) (+ ReLU) (x mask) in the epilogue
            xv = fmaf(xv, e0[kb], e1[kb]);
            const float rv = a.r ? to_f<T>(reinterpret_cast<const T*>(a.r)[off + 32 * kb]) : 0.f;
            if (a.r && !a.r_mul) xv += rv;
            if (a.relu) xv = fmaxf(xv, 0.f);
            if (a.r && a.r_mul) xv *= rv;
          }
          const T o = from_f<T>(xv);
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, o), rsY, (off + 32 * kb) * 2, 0, 0);
          const float f = to_f<T>(o);  // statistics of the value as stored
          if constexpr (EPI == kConvEpiStats) {
            const float d = f - e0[kb];
            s1[kb] += d;
            s2[kb] = fmaf(d, d, s2[kb]);
          } else if constexpr (EPI == kConvEpiBwd) {
            const float yv = to_f<T>(BY[off + 32 * kb]);
            const float dz = (!a.brelu || fmaf(yv, e0[kb], e1[kb]) > 0.f) ? f : 0.f;
            s1[kb] += dz;
            s2[kb] = fmaf(dz, yv - e2[kb], s2[kb]);
          }
        }
      }
    }
  };

  // ---- main loop: one iteration = one 64-channel chunk of one window = the nine (r, s) steps, with
  // rs a compile-time constant, and every global load unconditional (the prefetch of the slice two
  // steps ahead and of the next chunk's halo always target a valid slice / window). The compiler's
  // vmcnt bookkeeping then stays exact: with the conditional loads of the round-5 loop it merged the
  // paths into vmcnt(0) ahead of every weight store, so each step waited for the slice it had just
  // requested two steps ahead (profiles/conv_pmc_r6.md). The slice of step t sits in register slot
  // t % 3 = rs % 3 (a chunk is nine steps), in LDS buffer t & 1.
  i4v wr[3][2];
  const int nchunks = ntile * nch;
  // fragments of k-step kk of step rs from weight buffer wcur (image rows: output channels, or for FLIP
  // the reduction channels read transposed) and the halo at offset (rs / 3, rs % 3)
  auto frags = [&](const char* wcur, int rs, int kk, i4v (&f)[4]) __attribute__((always_inline)) {
    const int r = rs / 3, s = rs - r * 3;
    const char* hb0 = halo + (2 * wave + r) * RS + s * kPix + hlane;  // window row 2w, offset (r, s)
    const char* hb1 = hb0 + RS;                                         // window row 2w + 1
    const int ch = 2 * kk + h;
    if (FLIP) {
      f[0] = frag_tr(wcur, 16 * kk + 8 * h, 0, lane);
      f[1] = frag_tr(wcur, 16 * kk + 8 * h, 32, lane);
    } else {
      f[0] = *reinterpret_cast<const i4v*>(wcur + wsw(r32, ch));
      f[1] = *reinterpret_cast<const i4v*>(wcur + wsw(32 + r32, ch));
    }
    f[2] = *reinterpret_cast<const i4v*>(hb0 + ch * 16);
    f[3] = *reinterpret_cast<const i4v*>(hb1 + ch * 16);
  };
  auto mfma4 = [&](const i4v (&f)[4]) __attribute__((always_inline)) {
    // acc[kb][pb]: SW puts the weights (output channels) on the MFMA rows, the pixels on the lanes
    if constexpr (SW) {
      acc[0][0] = Mfma32<T>::run(f[0], f[2], acc[0][0]);
      acc[0][1] = Mfma32<T>::run(f[0], f[3], acc[0][1]);
      acc[1][0] = Mfma32<T>::run(f[1], f[2], acc[1][0]);
      acc[1][1] = Mfma32<T>::run(f[1], f[3], acc[1][1]);
    } else {
      acc[0][0] = Mfma32<T>::run(f[2], f[0], acc[0][0]);
      acc[0][1] = Mfma32<T>::run(f[3], f[0], acc[0][1]);
      acc[1][0] = Mfma32<T>::run(f[2], f[1], acc[1][0]);
      acc[1][1] = Mfma32<T>::run(f[3], f[1], acc[1][1]);
    }
  };
  // software pipeline over the four k-steps with two fragment sets: the reads of k-step kk + 2 are issued
  // right after the MFMAs of kk (which free that set) and before those of kk + 1, so each read group has
  // four MFMAs (>= 128 cycles) to land; the scheduling barriers keep the compiler from sinking the reads
  // behind the MFMAs and reusing one set (read, lgkmcnt(0), 4 MFMAs, ...). fa / fb hold k-steps 0 / 1.
  i4v fa[4], fb[4];
  auto mfma_step = [&](const char* wcur, int rs) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    mfma4(fa);
    __builtin_amdgcn_sched_barrier(0);
    frags(wcur, rs, 2, fa);
    __builtin_amdgcn_sched_barrier(0);
    mfma4(fb);
    __builtin_amdgcn_sched_barrier(0);
    frags(wcur, rs, 3, fb);
    __builtin_amdgcn_sched_barrier(0);
    mfma4(fa);
    mfma4(fb);
    __builtin_amdgcn_sched_barrier(0);
  };
  zero_acc();
  halo_load(tile0, 0);
  if constexpr (NB == 3) {
    // Three LDS weight buffers (slice t in buffer t % 3 = rs % 3) and register slots (slice t in slot
    // t % 3): slice t + 3 is requested at the start of step t and written to LDS at the end of step t + 1,
    // so each step ends with: store slice t + 2, read the first two k-steps' fragments of step t + 1 (its
    // slice was published by the previous barrier), barrier -- and the MFMAs of step t + 1 start right at
    // the barrier instead of behind an LDS round trip. (Not across a chunk boundary: the halo changes.)
    w_load(0, 0, wr[0]);
    w_load(0, 1, wr[1]);
    halo_store();
    w_store(wb, wr[0]);
    w_store(wb + kWBytes, wr[1]);
    w_load(0, 2, wr[2]);
    __syncthreads();
    for (int cidx = 0; cidx < nchunks; ++cidx) {
      const int it = cidx / nch, chunk = cidx - it * nch;
      const int nchunk = chunk + 1 == nch ? 0 : chunk + 1;  // chunk of the slices after rs = 8
      // the (window, chunk) whose halo is prefetched during this chunk: the next one, or this window's
      // first chunk again after the last (loaded, stored, never read)
      const int htile = (chunk + 1 == nch && it + 1 < ntile) ? tile0 + it + 1 : tile0 + it;
#pragma unroll
      for (int rs = 0; rs < 9; ++rs) {
        if (rs + 3 < 9) w_load(chunk, rs + 3, wr[rs % 3]);
        else w_load(nchunk, rs + 3 - 9, wr[rs % 3]);
        if (rs == 0) halo_load(htile, nchunk * kCK);
        const char* wcur = wb + (rs % 3) * kWBytes;
        if (rs == 0) {
          frags(wcur, 0, 0, fa);
          frags(wcur, 0, 1, fb);
        }
        mfma_step(wcur, rs);
        w_store(wb + ((rs + 2) % 3) * kWBytes, wr[(rs + 2) % 3]);  // slice t + 2 (requested at step t - 1)
        if (rs < 8) {
          const char* wnext = wb + ((rs + 1) % 3) * kWBytes;
          frags(wnext, rs + 1, 0, fa);
          frags(wnext, rs + 1, 1, fb);
        } else {
          __syncthreads();  // every wave is done with this chunk's halo
          halo_store();
          if (chunk + 1 == nch) {  // window done: results out, accumulators reset
            epilogue(tile0 + it);
            zero_acc();
          }
        }
        __syncthreads();
      }
    }
  } else {
    // two LDS weight buffers: slice t + 2 requested at the start of step t (register slot t % 3), slice
    // t + 1 written to buffer (t + 1) & 1 at its end
    w_load(0, 0, wr[0]);
    halo_store();
    w_store(wb, wr[0]);
    w_load(0, 1, wr[1]);
    __syncthreads();
    for (int cidx = 0; cidx < nchunks; ++cidx) {
      const int it = cidx / nch, chunk = cidx - it * nch;
      const int nchunk = chunk + 1 == nch ? 0 : chunk + 1;
      const int htile = (chunk + 1 == nch && it + 1 < ntile) ? tile0 + it + 1 : tile0 + it;
      const char* wbase = wb + (cidx & 1) * kWBytes;  // buffer of rs = 0 (9 is odd: parity flips per chunk)
#pragma unroll
      for (int rs = 0; rs < 9; ++rs) {
        if (rs + 2 < 9) w_load(chunk, rs + 2, wr[(rs + 2) % 3]);
        else w_load(nchunk, rs + 2 - 9, wr[(rs + 2) % 3]);
        if (rs == 0) halo_load(htile, nchunk * kCK);
        const char* wcur = (rs & 1) ? wb + kWBytes - (wbase - wb) : wbase;  // buffer (t & 1)
        frags(wcur, rs, 0, fa);
        frags(wcur, rs, 1, fb);
        mfma_step(wcur, rs);
        // slice t + 1 (requested a step ago) into the other buffer: every wave finished reading it at
        // the barrier that ended step t - 1
        w_store(wb + kWBytes - (wcur - wb), wr[(rs + 1) % 3]);
        if (rs == 8) {
          __syncthreads();  // every wave is done with this chunk's halo
          halo_store();
          if (chunk + 1 == nch) {
            epilogue(tile0 + it);
            zero_acc();
          }
        }
        __syncthreads();
      }
    }
  }
  if constexpr (EPI == kConvEpiStats || EPI == kConvEpiBwd) {
    // per-workgroup partial of each statistic: lane halves, then the 4 waves (LDS, the halo is free)
    float* red = reinterpret_cast<float*>(smem);  // [waves][2][64]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s1[kb] += __shfl_xor(s1[kb], 32);
      s2[kb] += __shfl_xor(s2[kb], 32);
      if (h == 0) {
        red[(wave * 2) * 64 + 32 * kb + r32] = s1[kb];
        red[(wave * 2 + 1) * 64 + 32 * kb + r32] = s2[kb];
      }
    }
    __syncthreads();
    if (tid < 128) {
      const int stat = tid >> 6, c = tid & 63;
      float u = 0.f;
#pragma unroll
      for (int q = 0; q < kThreads / 64; ++q) u += red[(q * 2 + stat) * 64 + c];
      a.part[((int64_t)stat * gridDim.x + blockIdx.x) * a.K + k0 + c] = u;
    }
  }
}

template <typename T> struct Tag { using type = T; };

Geo make_geo(int H, int W) {
  Geo g;
  g.G = 1;
  while (g.G < 4 && 32 / (2 * g.G) >= W) g.G *= 2;  // pack up to 4 narrow images side by side
  g.gw = 32 / g.G;
  g.HC = g.G * (g.gw + 2);
  g.XT = g.G == 1 ? (W + 31) / 32 : 1;
  g.YT = (H + kTH - 1) / kTH;
  g.tiles = 0;
  g.tpw = 1;
  return g;
}

}  // namespace

bool conv3x3_supported(const Conv3x3Args& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int64_t pix = (int64_t)a.N * a.H * a.W;
  if (a.pro_scale && (!a.pro_shift || a.C > kMaxProC)) return false;
  if ((a.epi == kConvEpiStats || a.epi == kConvEpiBwd) && !a.part) return false;
  if (a.epi == kConvEpiBwd && (!a.by || !al(a.by) || !a.bscale || !a.bshift || !a.bmean)) return false;
  if (a.epi == kConvEpiAffine && (!a.a_scale || !a.a_shift || a.pro_scale)) return false;
  return a.N > 0 && a.H > 0 && a.W > 0 && a.C > 0 && a.K > 0 && a.C % kCK == 0 && a.K % kBN == 0 && al(a.x) &&
         al(a.w) && al(a.y) && pix * a.C * 2 + 128 < kOutOfRange && pix * a.K * 2 < kOutOfRange &&
         (int64_t)a.K * 9 * a.C * 2 < kOutOfRange;  // 32-bit byte offsets in the buffer loads
}

namespace {

struct Launch {
  Geo g;
  dim3 grid;
};

Launch plan(const Conv3x3Args& a) {
  const Geo g = make_geo(a.H, a.W);
  if (g.HC > kMaxHC) throw std::runtime_error("conv3x3: halo geometry out of range");
  Launch l;
  l.g = g;
  const int64_t tiles = (int64_t)g.XT * g.YT * ((a.N + g.G - 1) / g.G);
  l.g.tiles = (int)tiles;
  const int64_t ktiles = a.K / kBN;
  // about two resident workgroups per CU over the whole grid: each walks tpw consecutive windows and
  // prefetches the next window's halo while computing the current one. (A one-workgroup-per-CU
  // variant holding all nine weight slices of a chunk in LDS measured 1.2x slower: profiles/
  // conv3x3_direct_vs_miopen.jsonl.)
  l.g.tpw = (int)std::max<int64_t>(1, (tiles * ktiles + 511) / 512);
  l.grid = dim3((unsigned)((tiles + l.g.tpw - 1) / l.g.tpw), (unsigned)ktiles);
  return l;
}

}  // namespace

int conv3x3_parts(const Conv3x3Args& a) { return (int)plan(a).grid.x; }

void conv3x3_run(int dt, const Conv3x3Args& a, bool flip, hipStream_t st) {
  if (!conv3x3_supported(a)) throw std::runtime_error("conv3x3: needs C % 64 == 0, K % 64 == 0, aligned tensors");
  // instantiated: forward (prologue and / or statistics epilogue), data gradient (backward epilogue)
  if (flip && (a.pro_scale || a.epi == kConvEpiStats)) throw std::runtime_error("conv3x3_dgrad: no prologue / stats");
  if (!flip && a.epi == kConvEpiBwd) throw std::runtime_error("conv3x3_forward: no backward epilogue");
  if (flip && a.epi == kConvEpiAffine) throw std::runtime_error("conv3x3_dgrad: no affine epilogue");
  const Launch l = plan(a);
  // pipeline variants (A/B knobs, Config.conv3x3_nb / conv3x3_sw): weight buffers 3 (next step's first
  // fragments read before the barrier) or 2; the plain epilogue from the transposed accumulator layout
  const int nb = knob("conv3x3_nb", 2) == 3 ? 3 : 2;
  const bool sw = knob("conv3x3_sw", 0) != 0;
  auto launch = [&](auto tt, auto gg) {
    using T = typename decltype(tt)::type;
    constexpr int GG = decltype(gg)::value;
    auto L = [&](auto kern) { hipLaunchKernelGGL(kern, l.grid, dim3(kThreads), 0, st, a, l.g); };
    if (flip) {
      if (a.epi == kConvEpiBwd) L(k_conv3x3<T, true, GG, false, kConvEpiBwd>);
      else if (nb == 2 && !sw) L(k_conv3x3<T, true, GG, false, kConvEpiPlain, 2, false>);
      else if (nb == 2) L(k_conv3x3<T, true, GG, false, kConvEpiPlain, 2, true>);
      else if (!sw) L(k_conv3x3<T, true, GG, false, kConvEpiPlain, 3, false>);
      else L(k_conv3x3<T, true, GG, false, kConvEpiPlain>);
    } else if (a.pro_scale) {
      if (a.epi == kConvEpiStats && nb == 2) L(k_conv3x3<T, false, GG, true, kConvEpiStats, 2>);
      else if (a.epi == kConvEpiStats) L(k_conv3x3<T, false, GG, true, kConvEpiStats>);
      else L(k_conv3x3<T, false, GG, true, kConvEpiPlain>);
    } else {
      if (a.epi == kConvEpiStats && nb == 2) L(k_conv3x3<T, false, GG, false, kConvEpiStats, 2>);
      else if (a.epi == kConvEpiStats) L(k_conv3x3<T, false, GG, false, kConvEpiStats>);
      else if (a.epi == kConvEpiAffine) L(k_conv3x3<T, false, GG, false, kConvEpiAffine>);
      else L(k_conv3x3<T, false, GG, false, kConvEpiPlain>);
    }
  };
  auto by_g = [&](auto tt) {
    switch (l.g.G) {
      case 1: launch(tt, std::integral_constant<int, 1>{}); break;
      case 2: launch(tt, std::integral_constant<int, 2>{}); break;
      default: launch(tt, std::integral_constant<int, 4>{}); break;
    }
  };
  switch (dt) {
    case kF16: by_g(Tag<f16>{}); break;
    case kBF16: by_g(Tag<bf16>{}); break;
    default: throw std::runtime_error("conv3x3: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv3x3: ") + hipGetErrorString(e));
}

void conv3x3_forward(int dt, const Conv3x3Args& a, hipStream_t st) { conv3x3_run(dt, a, false, st); }
void conv3x3_dgrad(int dt, const Conv3x3Args& a, hipStream_t st) { conv3x3_run(dt, a, true, st); }

}  // namespace bh
