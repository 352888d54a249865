// Weight gradient of a stride-1 "same" NHWC convolution (R x R, R = 1 or 3) on MFMA 32x32x16 (gfx950):
//   dW[k][r][s][c] = sum over pixels p of dY[p][k] * X[p + (r - P, s - P)][c],   P = (R - 1) / 2
// see bh/conv_api.h.
//
// The reduction runs over pixels, which sit on the strided (row) axis of both NHWC operands, so both
// MFMA operands are read from LDS with ds_read_b64_tr_b16 (the 16-lane hardware transpose: each lane
// names 4 contiguous channels of one pixel row, and gets one channel of 4 pixels). The k-dimension is
// a list of 4-pixel groups along image rows, so a 14- or 7-wide image wastes at most one group column
// instead of padding rows to 32.
//
// Workgroup = 8 waves = a 64 (k) x 64 (c) tile of all R*R offsets, one workgroup per CU: the two
// waves of a SIMD share a 32x32 (k, c) quadrant and split its R*R offsets (5 + 4 accumulators at
// R = 3), so each SIMD runs two waves that cover each other's waits. A window is TH whole image
// rows: its dY (TH x 4*G4 pixels, zero past the image) and the X halo ((TH + 2P) x (4*G4 + 2P)
// pixels, zero outside the image) land in LDS by LDS-DMA (buffer loads through whole-tensor
// resources: an out-of-image pixel gets an out-of-range offset and arrives as zeros), double
// buffered (up to 141 KiB: padded pixel slots, see kSlot). Every k-step reads one dY
// fragment and reuses it for the R*R shifted X fragments; the next k-step's fragments are read
// behind the current MFMAs. Each workgroup walks a contiguous run of windows and writes an fp32
// partial tile; a second kernel sums the splits in a fixed order into the 16-bit weight gradient
// (deterministic, no atomics, no zero-fill). Workgroups that share windows sit on one XCD (shared L2).
#include "bh/api.h"
#include "bh/conv_api.h"
#include "bh/device.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace bh {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4_ptr;

template <typename T> struct MfmaW;
template <> struct MfmaW<f16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
  }
};
template <> struct MfmaW<bf16> {
  static BH_DEVICE f16v run(i4v a, i4v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, a), __builtin_bit_cast(b8v, b), c, 0, 0, 0);
  }
};

constexpr int kThreads = 512;   // 8 waves: two per SIMD
constexpr int kTile = 64;        // k and c per workgroup
// LDS bytes per pixel slot: 64 channels x 2 B + 64 B pad. At a 48-dword stride any four consecutive
// slots start in four distinct 16-dword bank quarters, so the transposed reads (4 pixels x 64 B per
// 32-lane half) are conflict free, and a slot's address is LINEAR in the slot index: the R*R
// shifted X fragments are one base register plus immediate offsets (no per-read swizzle math).
constexpr int kSlot = 192;
constexpr int kMaxHalo = 288;    // X slots per window
constexpr int kMaxD = 128;       // dY slots per window (k-steps x 16)
// dY slots hold 64 * KT channels: 128 + 64 B (KT = 1) or 256 + 64 B (KT = 2, again four distinct
// bank quarters for four consecutive slots)
template <int KT> constexpr int dslot() { return KT == 1 ? 192 : 320; }
constexpr unsigned kRsrcWord3 = 0x00020000u;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One LDS-DMA instruction (16 B per lane, lane-linear at LDS byte address `lds`) through buffer
// resource `rs`, as inline asm: issued through the builtin, the compiler cannot tell the DMA's LDS
// writes from the fragment reads of the OTHER window buffer and puts an s_waitcnt vmcnt(0) in front
// of every following ds_read -- which serialises the prefetch with the compute. Here the kernel
// orders them itself (wait_vmcnt + barrier at the window boundary).
BH_DEVICE void dma16(i4v rs, int voff, unsigned lds) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %2, 0 offen lds" ::"v"(voff),
      "s"(lds), "s"(rs)
      : "memory", "m0");
}
BH_DEVICE i4v make_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  return i4v{(int)(uint32_t)a, (int)((a >> 32) & 0xffff), (int)(uint32_t)bytes, (int)kRsrcWord3};
}
BH_DEVICE unsigned lds_addr(const void* p) {
  typedef const __attribute__((address_space(3))) char* lds_cptr;
  return (unsigned)(uintptr_t)((lds_cptr)p);
}

template <int N> BH_DEVICE void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// workgroup barrier the compiler may not move LDS accesses across (LDS-DMA writes are invisible to it)
BH_DEVICE void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// operand fragment: two transposed 4-pixel reads at byte offsets lo / hi (+ a compile-time shift)
BH_DEVICE i4v frag2(const char* img, int lo, int hi) {
  const s4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + lo));
  const s4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(img + hi));
  const i2v l = __builtin_bit_cast(i2v, a), hh = __builtin_bit_cast(i2v, b);
  return i4v{l[0], l[1], hh[0], hh[1]};
}

// window geometry (G4 four-pixel groups per row, TH rows) as compile-time constants: the staging
// address math divides by them
// PRO: x is the raw input of a BatchNorm + ReLU that was never applied (models/resnet.py folds it into
// the consumers): every lane rewrites the X chunks its own LDS-DMA brought in -- relu(x * scale + shift),
// rounded as the normalisation pass would -- after they land and before the window barrier; chunks of
// pixels outside the image stay zero (they pad the normalised activation).
// WIDE (1x1 only): 256 output channels per workgroup -- the four k quarters of 64 go to the four wave
// pairs and each wave runs every k-step of the window (no split of the k-steps between the two waves of
// a SIMD, no LDS hand-off at the end) -- which cuts the bytes staged per MFMA by a quarter; the dY slot
// grows to 512 + 64 B (144 dwords: again four distinct bank quarters) and the window to 64 pixels.
// S (R = 3 only): the convolution's stride. At S = 2 (the ResNet downsampling 3x3) dY pixel (y, x) of the
// window reads X pixel (2 y + r - 1, 2 x + s - 1): the X halo is (2 TH + 1) x (8 G4 + 1) slots and the
// fragment of shift (r, s) sits at slot 2 (row * HC + x) + r * HC + s -- still one base address plus
// an immediate per shift; only the slot map and the staging addresses change.
template <typename T, int R, int G4, int TH, int KT, int CT = 1, bool PRO = false, bool WIDE = false, int S = 1>
__global__ __launch_bounds__(kThreads, 1) void k_conv_wgrad(ConvWgradArgs a, ConvWgradGeo g, float* __restrict__ ws,
                                                           T* __restrict__ out) {
  static_assert(S == 1 || R == 3, "the strided halo is a 3x3 geometry (1x1 stride 2 uses flat windows)");
  constexpr int P = (R - 1) / 2, RR = R * R;
  constexpr int HC = S * (4 * G4 - 1) + R, KSTEPS = (TH * G4 + 3) / 4;
  constexpr int XS = (S * (TH - 1) + R) * HC, DS = KSTEPS * 16;  // X halo / dY pixel slots per window
  constexpr int KW = WIDE ? 4 : 2;  // k sub-tiles of 32 KT across the waves
  static_assert(!WIDE || (R == 1 && KT == 2), "wide tiles: 1x1, two 32-row sub-tiles per wave");
  constexpr int DSL = WIDE ? 576 : dslot<KT>(), TK = 32 * KT * KW;  // dY slot bytes, output channels per workgroup
  // X slot bytes (CT = 4, the 256 x 256 wide tile: 512 + 64 B, 144 dwords like the wide dY slot), input
  // channels per workgroup
  constexpr int XSL = CT == 4 ? 576 : dslot<CT>(), TC = kTile * CT;
  constexpr int BUFX = (XS * XSL + 1023) / 1024 * 1024, BUF = BUFX + (DS * DSL + 1023) / 1024 * 1024;
  constexpr int XP = BUFX / 1024, DP = (BUF - BUFX) / 1024;  // 1-KiB LDS-DMA pieces
  constexpr int XPW = (XP + 7) / 8, DPW = (DP + 7) / 8;  // pieces per wave
  // offsets per wave: the two waves of a SIMD split the R*R offsets; at R = 1 the slot is the wave's
  // 32-column sub-tile of its 32 * CT input channels instead
  constexpr int NOFF = R == 1 ? CT : (RR + 1) / 2;
  static_assert(XS <= kMaxHalo && DS <= kMaxD, "window does not fit");
  static_assert(2 * BUF + (PRO ? 8 * TC : 0) <= 160 * 1024, "two window buffers must fit in LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + (PRO ? 8 * TC : 0)];
  // XCD-aware placement: hardware deals workgroup ids round-robin over the 8 XCDs; consecutive
  // logical ids (same window run, different tiles) land on one XCD so the run is read from one L2
  const int b = blockIdx.x;
  const int L = (b & 7) * (g.grid / 8) + (b >> 3);
  if (L >= g.tiles * g.splits) return;  // grid padding (before any barrier)
  const int tile = L % g.tiles, split = L / g.tiles;
  const int k0 = (tile / g.ctiles) * TK, c0 = (tile % g.ctiles) * TC;
  const int w_begin = split * g.wpw, w_end = min(g.nwin, w_begin + g.wpw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kw = WIDE ? wave >> 1 : (wave >> 1) & 1, cw = wave & 1, half = WIDE ? 0 : wave >> 2;
  // R = 3: the two waves of a SIMD split the offsets (rs0 .. rs0 + noff - 1); R = 1 (one offset):
  // they split the k-steps instead (half h takes ks = h, h + 2, ...) and write separate partials
  const int rs0 = R == 1 ? 0 : half * NOFF, noff = R == 1 ? NOFF : min(NOFF, RR - rs0);
  const int C = a.C, K = a.K, H = a.H, W = a.W;
  // whole-tensor buffer resources: a pixel outside the image (or a pad chunk) gets an offset past
  // the range and lands in LDS as zeros (no clamped pointers, no select)
  const int sx = a.stride * a.stride;  // x pixels per dY pixel
  const i4v rsX = make_rsrc(a.x, (int64_t)a.N * H * W * C * 2 * sx);
  const i4v rsD = make_rsrc(a.dy, (int64_t)a.N * H * W * K * 2);
  constexpr int kOut = 0x7ff00000;  // any offset past both ranges
  // LDS-DMA is lane-linear: lane l of piece j fills bytes [1024 j + 16 l, +16) = one 16-byte chunk
  // of a pixel slot. The per-lane part of every piece's source offset is fixed for the kernel (the
  // window only moves the image row): rel = byte offset from the window origin, hrow = the pixel's
  // row in the window (kBad: pad chunk / past the slots / outside the image columns).
  constexpr int NPW = XPW + DPW;  // this wave's pieces: X pieces first, then dY pieces
  constexpr int kBad = -4096;
  int rel[NPW], hrow[NPW];
  int xch[XPW];  // PRO: the 8-channel chunk of each X piece this lane fills (-1: pad chunk / no piece)
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const bool isx = i < XPW;
    const int piece = wave + 8 * (isx ? i : i - XPW);
    const int byte = piece * 1024 + lane * 16, slot = byte / XSL, ch = (byte - slot * XSL) >> 4;
    if (isx) xch[i < XPW ? i : 0] = (piece < XP && ch < 8 * CT && slot < XS) ? ch : -1;
    if (isx) {
      const int hr = slot / HC, x = slot - hr * HC - P;
      const bool ok = piece < XP && ch < 8 * CT && slot < XS && x >= 0 && x < S * W;
      // 1x1 / stride 2 (flat windows of whole output rows): dY pixel x of the window reads x pixel
      // 2 x + 2 wout (x / wout) from the window's x origin (input rows are twice as long, and every
      // other one is skipped)
      const int xin = (R == 1 && a.stride == 2) ? 2 * x + 2 * a.wout * (x / a.wout) : x;
      rel[i] = (((hr - P) * S * W + xin) * C + c0 + ch * 8) * 2;
      hrow[i] = ok ? hr - P : kBad;
    } else {
      const int dbyte = byte, dsl = dbyte / DSL, dch = (dbyte - dsl * DSL) >> 4;
      const int grp = dsl >> 2, row = grp / G4, x = 4 * (grp - row * G4) + (dsl & 3);
      const bool ok = piece < DP && dch < TK / 8 && dsl < DS && row < TH && x < W;
      rel[i] = ((row * W + x) * K + k0 + dch * 8) * 2;
      hrow[i] = ok ? row : kBad;
    }
  }
  // piece i of window (n, y0) into buffer buf (wave-uniform guard: waves own different piece counts)
  auto issue_piece = [&](int i, int n, int y0, char* buf) {
    const bool isx = i < XPW;
    const int piece = wave + 8 * (isx ? i : i - XPW);
    if (piece >= (isx ? XP : DP)) return;
    const int sy = isx ? S : 1;  // X rows of a strided 3x3 window start at input row S y0
    const int y = sy * y0 + hrow[i];
    const bool ok = hrow[i] != kBad && y >= 0 && y < sy * H;
    const int off = ok ? (n * H + y0) * W * (isx ? C * sx : K) * 2 + rel[i] : kOut;
    if (isx) dma16(rsX, off, __builtin_amdgcn_readfirstlane(lds_addr(buf + piece * 1024)));
    else dma16(rsD, off, __builtin_amdgcn_readfirstlane(lds_addr(buf + BUFX + piece * 1024)));
  };
  auto win_origin = [&](int win, int& n, int& y0) {
    n = win / g.wpi;
    y0 = (win - n * g.wpi) * TH;
  };
  float* pss = reinterpret_cast<float*>(smem + 2 * BUF);  // PRO: scale[TC], shift[TC] of channels c0..
  if constexpr (PRO) {
    for (int i = tid; i < TC; i += kThreads) {
      pss[i] = a.pro_scale[c0 + i];
      pss[TC + i] = a.pro_shift[c0 + i];
    }
  }
  // PRO: this lane's landed X chunks of window (n, y0) in buffer buf -> relu(x * scale + shift)
  auto prologue = [&](int n, int y0, char* buf) {
    (void)n;
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
      const int piece = wave + 8 * i;
      const int y = S * y0 + hrow[i];
      if (xch[i] < 0 || hrow[i] == kBad || y < 0 || y >= S * H) continue;
      char* p = buf + piece * 1024 + lane * 16;
      typedef T t8 __attribute__((ext_vector_type(8)));
      t8 v = *reinterpret_cast<const t8*>(p);
      const float* sc = pss + xch[i] * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = from_f<T>(fmaxf(fmaf(to_f<T>(v[e]), sc[e], sc[TC + e]), 0.f));
      *reinterpret_cast<t8*>(p) = v;
    }
  };

  // per-lane fragment addresses, fixed for the whole kernel. Transposed read: lane 4q + p of each
  // 16-lane group names pixel q, columns 4p .. 4p+3 of its group's 16-column band; half h takes the
  // k-step's pixel groups 2h, 2h + 1 (the MFMA's k = 8h .. 8h + 7).
  const int g16 = lane >> 4, q = (lane & 15) >> 2, pc = lane & 3, h = lane >> 5;
  const int colb = 2 * (16 * (g16 & 1) + 4 * pc);
  const int a_off = (8 * h + q) * DSL + 2 * 32 * KT * kw + colb;  // dY: slot 16 ks + 8h + q (+4 for hi)
  constexpr int ng = TH * G4;  // real groups; padded groups read zero dY (and clamped X)
  int x_off[KSTEPS][2];        // X: slot of pixel q of groups 4 ks + 2h + j at shift (0, 0)
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int grp = min(4 * ks + 2 * h + j, ng - 1), row = grp / G4;
      x_off[ks][j] = S * (row * HC + 4 * (grp - row * G4) + q) * XSL + 2 * 32 * CT * cw + colb;
    }

  f16v acc[NOFF][KT];
#pragma unroll
  for (int j = 0; j < NOFF; ++j)
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][t][i] = 0.f;

  if (w_begin < w_end) {
    int n, y0;
    win_origin(w_begin, n, y0);
#pragma unroll
    for (int i = 0; i < NPW; ++i) issue_piece(i, n, y0, smem);
  }
  // fragments of k-step ks + 1 are read while the MFMAs of ks run (two register sets, one read pair
  // behind each MFMA, order pinned by sched_barrier)
  i4v fa[2][KT], fb[2][NOFF];
  if constexpr (PRO) __syncthreads();  // scale / shift visible
  for (int win = w_begin; win < w_end; ++win) {
    const char* xs = smem + ((win - w_begin) & 1) * BUF;
    const char* ds = xs + BUFX;
    wait_vmcnt<0>();  // this wave's pieces of window `win` have landed ...
    if constexpr (PRO) {
      // the first window's tiles here; every later window's were transformed at the end of the
      // window before it, where the VALU work overlaps that window's last MFMAs in the pipe
      if (win == w_begin) {
        int n0, y00;
        win_origin(win, n0, y00);
        asm volatile("" ::: "memory");
        prologue(n0, y00, const_cast<char*>(xs));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    raw_barrier();    // ... and everyone's; everyone is also done reading the other buffer
    // the next window's pieces are issued one behind each of the first MFMAs (their address math
    // co-issues with the matrix cores instead of stalling in front of them)
    const bool pre = win + 1 < w_end;
    int nn = 0, ny0 = 0;
    if (pre) win_origin(win + 1, nn, ny0);
    char* nbuf = smem + ((win + 1 - w_begin) & 1) * BUF;
    // PRO: the next window's tiles, once this wave's DMA for them has landed (nobody reads that buffer
    // during this window; the barrier at the next window's top publishes the result)
    auto prologue_next = [&]() __attribute__((always_inline)) {
      if constexpr (PRO) {
        if (pre) {
          wait_vmcnt<0>();
          asm volatile("" ::: "memory");
          prologue(nn, ny0, nbuf);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
    };
    auto read_a = [&](int ks, int buf) {
#pragma unroll
      for (int t = 0; t < KT; ++t) fa[buf][t] = frag2(ds + 16 * ks * DSL + 64 * t, a_off, a_off + 4 * DSL);
    };
    // offset j of this wave: rs = rs0 + j = r * R + s, LDS shift (r * HC + s) slots (wave-uniform
    // branch: the half-1 waves of an odd R*R own one offset fewer)
    auto read_b = [&](int ks, int buf, int j) {
      const int rs = rs0 + j, r = rs / R, s = rs - r * R;
      const char* base = xs + (r * HC + s) * XSL;
      fb[buf][j] = frag2(base, x_off[ks][0], x_off[ks][1]);
    };
    if constexpr (R == 1) {
      // k-step ks = 2u + half (WIDE: ks = u); the X slots of a flat 1x1 window are linear in ks
      constexpr int KL = WIDE ? KSTEPS : (KSTEPS + 1) / 2;
      auto kstep = [&](int u) { return WIDE ? u : 2 * u + half; };
      auto rd = [&](int u, int buf) {
        const int ks = kstep(u);
#pragma unroll
        for (int t = 0; t < KT; ++t) fa[buf][t] = frag2(ds + 16 * ks * DSL + 64 * t, a_off, a_off + 4 * DSL);
#pragma unroll
        for (int j = 0; j < NOFF; ++j) fb[buf][j] = frag2(xs + 16 * ks * XSL + 64 * j, x_off[0][0], x_off[0][1]);
      };
#pragma unroll
      for (int t = 0; t < NPW; ++t)  // the next window's pieces first: they have the whole window to land
        if (pre) issue_piece(t, nn, ny0, nbuf);
      rd(0, 0);
#pragma unroll
      for (int u = 0; u < KL; ++u) {
        const int cur = u & 1;
        if (kstep(u) < KSTEPS) {
#pragma unroll
          for (int j = 0; j < NOFF; ++j)
#pragma unroll
            for (int t = 0; t < KT; ++t) acc[j][t] = MfmaW<T>::run(fa[cur][t], fb[cur][j], acc[j][t]);
        }
        if (u + 1 < KL && kstep(u + 1) < KSTEPS) rd(u + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      prologue_next();
      continue;
    }
    read_a(0, 0);
#pragma unroll
    for (int j = 0; j < NOFF; ++j)
      if (j < noff) read_b(0, 0, j);
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int cur = ks & 1, nxt = cur ^ 1;
#pragma unroll
      for (int j = 0; j < NOFF; ++j) {
        if (j < noff)
#pragma unroll
          for (int t = 0; t < KT; ++t) acc[j][t] = MfmaW<T>::run(fa[cur][t], fb[cur][j], acc[j][t]);
        if (const int t = ks * NOFF + j; t < NPW && pre) issue_piece(t, nn, ny0, nbuf);
        if (ks + 1 < KSTEPS) {
          if (j == 0) read_a(ks + 1, nxt);
          if (j < noff) read_b(ks + 1, nxt, j);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int t = KSTEPS * NOFF; t < NPW; ++t)  // pieces left over when a window has few MFMAs (R = 1)
      if (pre) issue_piece(t, nn, ny0, nbuf);
    prologue_next();
  }

  if constexpr (R == 1 && !WIDE) {
    // the two waves of a SIMD hold partial sums of the same tile (even / odd k-steps): the odd
    // half hands its accumulators to the even half through LDS, so one partial slab per split
    float* red = reinterpret_cast<float*>(smem);  // NOFF * KT * 16 floats per lane, 4 waves
    constexpr int NA = NOFF * KT * 16;
    raw_barrier();  // every wave is done with the window buffers
    if (half == 1) {
#pragma unroll
      for (int jo = 0; jo < NOFF; ++jo)
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) red[((jo * KT + t) * 16 + i) * 256 + (wave & 3) * 64 + lane] = acc[jo][t][i];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int jo = 0; jo < NOFF; ++jo)
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[jo][t][i] += red[((jo * KT + t) * 16 + i) * 256 + (wave & 3) * 64 + lane];
    static_assert(NA * 256 * 4 <= 2 * BUF, "reduction staging fits in the window buffers");
  }
  // lane holds column c = c0 + 32 CT cw (+ 32 jo at R = 1) + (lane & 31) and rows
  // k = k0 + 32 KT kw + 32 t + 8 j + 4 h + i (acc[4 j + i])
#pragma unroll
  for (int jo = 0; jo < NOFF; ++jo) {
    if (jo >= noff) break;
    const int rs = R == 1 ? 0 : rs0 + jo;
    const int c = c0 + 32 * CT * cw + (R == 1 ? 32 * jo : 0) + (lane & 31);
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = k0 + 32 * KT * kw + 32 * t + 8 * j + 4 * h + i;
          const int64_t o = ((int64_t)k * RR + rs) * C + c;
          if (g.parts == 1 && !g.f32) out[o] = from_f<T>(acc[jo][t][4 * j + i]);
          else ws[(int64_t)split * K * RR * C + o] = acc[jo][t][4 * j + i];
        }
  }
}

// out[i] = sum over splits of ws[s][i] in a fixed order: a block owns 64 elements (16 float4 quads)
// x 16 split groups; group g sums splits g, g + 16, ... and the groups are added in order through
// LDS (deterministic, and 16x the workgroups of a one-thread-per-quad loop over 256 splits)
template <typename T>
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ ws, T* __restrict__ out, int64_t n,
                                                      int splits) {
  __shared__ float4 part[16][16];
  const int tq = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t i = ((int64_t)blockIdx.x * 16 + tq) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n)
    for (int j = sg; j < splits; j += 16) {
      const float4 v = *reinterpret_cast<const float4*>(ws + (int64_t)j * n + i);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  part[sg][tq] = acc;
  __syncthreads();
  if (sg == 0 && i < n) {
    float4 t = part[0][tq];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      t.x += part[k][tq].x;
      t.y += part[k][tq].y;
      t.z += part[k][tq].z;
      t.w += part[k][tq].w;
    }
    T o[4] = {from_f<T>(t.x), from_f<T>(t.y), from_f<T>(t.z), from_f<T>(t.w)};
    *reinterpret_cast<uint2*>(out + i) = *reinterpret_cast<const uint2*>(o);
  }
}

}  // namespace

bool conv_wgrad_plan(const ConvWgradArgs& a, ConvWgradGeo* geo) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!(a.R == 1 || a.R == 3) || a.N <= 0 || a.H <= 0 || a.W <= 0 || a.C % kTile || a.K % kTile || !al(a.x) ||
      !al(a.dy) || !al(a.out))
    return false;
  // stride 2: 1x1 (windows of whole output rows, W divides 112) or 3x3 (strided halo, the three
  // ResNet-50 output widths 28 / 14 / 7)
  const bool s2r3 = a.stride == 2 && a.R == 3;
  if (!(a.stride == 1 || (a.stride == 2 && a.R == 1 && 112 % a.W == 0) || (s2r3 && (a.W == 28 || a.W == 14 || a.W == 7))))
    return false;
  if (a.pro_scale && ((a.stride != 1 && !s2r3) || !a.pro_shift)) return false;
  // 32-bit buffer offsets (the out-of-image offset sits past both tensors)
  if (2 * (int64_t)a.N * a.H * a.W * std::max(a.C * a.stride * a.stride, a.K) >= 0x7ff00000ll) return false;
  ConvWgradGeo g;
  if (a.R == 1) {
    // no halo: the N*H*W pixels are one flat list, 112-pixel windows (one row of 28 groups)
    // wide tiles (K % 256, C % 128): 64-pixel windows (two window buffers of 56 KiB)
    const int64_t npix = (int64_t)a.N * a.H * a.W;
    // (and at least 4 such tiles: with fewer, the extra split partials cost more than the staging saves,
    // measured on the 128 -> 512 layer-2 shape)
    g.wide = a.stride == 1 && a.K % 256 == 0 && a.C % 128 == 0 && npix % 64 == 0 &&
             (a.K / 256) * (a.C / 128) >= 4;
    const int win = g.wide ? 64 : 112;
    if (npix % win) return false;
    g.G4 = win / 4;
    g.TH = 1;
    g.wpi = 1;
    g.nwin = (int)((int64_t)a.N * a.H * a.W / win);
  } else if (s2r3) {
    // stride 2: the X halo of a window is ~4x its dY pixels, so the windows are shorter (2 rows at
    // W = 28, 3 at 14, 7 at 7: <= 285 X slots, two buffers <= 139 KiB)
    g.G4 = (a.W + 3) / 4;
    g.TH = a.W == 28 ? 2 : (a.W == 14 ? 3 : 7);
    g.wpi = (a.H + g.TH - 1) / g.TH;
    g.nwin = a.N * g.wpi;
  } else {
    // ~112 pixels per window: 2 rows at W = 56, 4 at 28, 7 at 14 / 7 (the instantiated geometries)
    g.G4 = (a.W + 3) / 4;
    if (g.G4 == 14) g.TH = 2;
    else if (g.G4 == 7) g.TH = 4;
    else if (g.G4 == 4 || g.G4 == 2) g.TH = 7;
    else return false;
    g.wpi = (a.H + g.TH - 1) / g.TH;
    g.nwin = a.N * g.wpi;
  }
  g.ksteps = (g.TH * g.G4 + 3) / 4;
  // 128 output channels per workgroup (each wave two k sub-tiles sharing its X fragments) for the
  // 14- / 7-wide windows (measured 1.1x there; the 28-wide instantiation spills and is slower)
  g.kt = (a.K % 128 == 0 && (a.R == 1 || g.G4 == 4 || g.G4 == 2)) ? 2 : 1;
  g.ct = (a.R == 1 && a.C % 128 == 0) ? 2 : 1;  // 1x1: 128 input channels per workgroup where C allows
  // 256 x 256 wide tiles (each wave 64 x 128: eight MFMA tiles per k-step on six fragments instead of
  // four on four -- a quarter fewer LDS bytes per MFMA, and twice the MFMA work per window against its
  // fixed staging cost) where K, C % 256 and at least 32 such tiles remain (the large transformer
  // weight gradients)
  if (g.wide && a.C % 256 == 0 && (a.K / 256) * (a.C / 256) >= 32) g.ct = 4;
  g.ctiles = a.C / (kTile * g.ct);
  g.tiles = (a.K / (kTile * g.kt * (g.wide ? 2 : 1))) * g.ctiles;
  // one round of workgroups (one per CU), split over the windows
  int splits = std::max(1, 256 / g.tiles);
  splits = std::min(splits, g.nwin);
  g.wpw = (g.nwin + splits - 1) / splits;
  g.splits = (g.nwin + g.wpw - 1) / g.wpw;
  g.parts = g.splits;
  g.grid = (g.tiles * g.splits + 7) / 8 * 8;
  *geo = g;
  return true;
}

int64_t conv_wgrad_workspace(const ConvWgradGeo& g, const ConvWgradArgs& a) {
  return (g.parts > 1 || g.f32) ? (int64_t)g.parts * a.K * a.C * a.R * a.R : 0;
}

void conv_wgrad(int dt, const ConvWgradArgs& a, const ConvWgradGeo& g, float* ws, hipStream_t st, bool reduce) {
  const int64_t n = (int64_t)a.K * a.C * a.R * a.R;
  ConvWgradArgs b = a;
  if (a.R == 1) {  // flat pixel list: windows are the rows of an [nwin, 1, 112] image
    b.wout = a.W;
    b.N = g.nwin;
    b.H = 1;
    b.W = 4 * g.G4;
  }
  auto run = [&](auto tt) {
    using T = typename decltype(tt)::type;
    T* out = reinterpret_cast<T*>(a.out);
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(g.grid), dim3(kThreads), 0, st, b, g, ws, out); };
    auto pick = [&](auto proc) {
      constexpr bool P = decltype(proc)::value;
      if (a.R == 1 && g.wide && g.ct == 4) go(k_conv_wgrad<T, 1, 16, 1, 2, 4, P, true>);
      else if (a.R == 1 && g.wide) go(k_conv_wgrad<T, 1, 16, 1, 2, 2, P, true>);
      else if (a.R == 1) {
        if (g.ct == 2) g.kt == 2 ? go(k_conv_wgrad<T, 1, 28, 1, 2, 2, P>) : go(k_conv_wgrad<T, 1, 28, 1, 1, 2, P>);
        else g.kt == 2 ? go(k_conv_wgrad<T, 1, 28, 1, 2, 1, P>) : go(k_conv_wgrad<T, 1, 28, 1, 1, 1, P>);
      }
      else if (a.stride == 2) {
        if (g.G4 == 7) go(k_conv_wgrad<T, 3, 7, 2, 1, 1, P, false, 2>);
        else if (g.G4 == 4) g.kt == 2 ? go(k_conv_wgrad<T, 3, 4, 3, 2, 1, P, false, 2>) : go(k_conv_wgrad<T, 3, 4, 3, 1, 1, P, false, 2>);
        else g.kt == 2 ? go(k_conv_wgrad<T, 3, 2, 7, 2, 1, P, false, 2>) : go(k_conv_wgrad<T, 3, 2, 7, 1, 1, P, false, 2>);
      }
      else if (g.G4 == 14) go(k_conv_wgrad<T, 3, 14, 2, 1, 1, P>);
      else if (g.G4 == 7) go(k_conv_wgrad<T, 3, 7, 4, 1, 1, P>);
      else if (g.G4 == 4) g.kt == 2 ? go(k_conv_wgrad<T, 3, 4, 7, 2, 1, P>) : go(k_conv_wgrad<T, 3, 4, 7, 1, 1, P>);
      else g.kt == 2 ? go(k_conv_wgrad<T, 3, 2, 7, 2, 1, P>) : go(k_conv_wgrad<T, 3, 2, 7, 1, 1, P>);
    };
    if (a.pro_scale) pick(std::true_type{});
    else pick(std::false_type{});
    if (g.parts > 1 && reduce)
      hipLaunchKernelGGL(k_wgrad_reduce<T>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, ws, out, n, g.parts);
  };
  switch (dt) {
    case kF16: run(std::common_type<f16>{}); break;
    case kBF16: run(std::common_type<bf16>{}); break;
    default: throw std::runtime_error("conv_wgrad: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv_wgrad: ") + hipGetErrorString(e));
}

void conv_wgrad_reduce(int dt, const float* ws, void* out, int64_t n, int parts, hipStream_t st) {
  if (parts <= 1) return;
  const dim3 grid((unsigned)((n + 63) / 64));
  switch (dt) {
    case kF16: hipLaunchKernelGGL(k_wgrad_reduce<f16>, grid, dim3(256), 0, st, ws, (f16*)out, n, parts); break;
    case kBF16: hipLaunchKernelGGL(k_wgrad_reduce<bf16>, grid, dim3(256), 0, st, ws, (bf16*)out, n, parts); break;
    default: throw std::runtime_error("conv_wgrad_reduce: fp16 / bf16 only");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("conv_wgrad_reduce: ") + hipGetErrorString(e));
}

}  // namespace bh
