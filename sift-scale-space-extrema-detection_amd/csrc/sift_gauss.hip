// Gaussian scale space + Difference-of-Gaussians for one octave (gfx950).
//
// Replaces background.js:71-237 (computeGaussianScaleSpace, whose hot loop is
// SIFT_blurMatrix2DChunk, sift.js:72-149) and background.js:258-354
// (computeDifferenceOfGaussians / SIFT_subtractMatrix2DChunk, sift.js:154-188).
//
// The reference convolves every scale of an octave with a full 2D kernel of
// the SAME octave base (the blur is not incremental, background.js:173-177).
// The 2D kernel is exactly separable (w(i) w(j), sift.js:22-67).  One block
// owns a 64x32 output tile; each of its 4 waves owns 8 rows of it and walks
// all scales of the octave on its own (no block barrier after the staging):
//
//   vertical pass   base -> fp64 LDS strip rows 8 wv .. 8 wv + 7, columns
//                   x0 - r .. x0 + 63 + r: lanes are columns with an 8-row
//                   register window (every base value loaded once per
//                   window); the 2r halo columns are packed into one pass of
//                   (column, row-slice) lanes;
//   horizontal pass strip -> 4 adjacent columns x 2 rows per lane, the row
//                   window read with 16-byte LDS loads;
//   epilogue        L_s and DoG L_{s-1} - L_s (formed in fp64, rounded once)
//                   as 16-byte buffer stores; for s == S the fp64 seed of the
//                   next octave (background.js:114-118).
//
// A wave touches only its own strip rows, so the only ordering it needs is
// its own (wave_lds_fence).  Radii 0..RMAX run fully unrolled code
// specialised on the radius (every tap an SGPR operand of v_fma_f64, every
// load an immediate-offset LDS read or a buffer load with the row in an
// SGPR); larger radii run 8-wide chunks over zero-padded taps (fma(0, v, acc)
// == acc, so the results are identical).
//
// Octave 0's base is the 2x nearest-neighbour upsample of the input
// (background.js:84): B[y][x] = I[clamp(y>>1)][clamp(x>>1)], never
// materialised.  The block stages its input region (fp64) in LDS; the
// vertical pass runs on input columns only (the vertical sums depend on x
// only through x>>1) and the horizontal pass reads the half-resolution strip
// through the same index map -- the same operations on the same values as a
// full-resolution pass, half the loads.
//
// Every output pixel runs the same fma chain (taps in increasing order,
// vertical then horizontal, starting from 0.0) on its clamped neighbourhood:
// the result is translation invariant like the reference's 2D sum, and
// sift_exact.h reproduces any single pixel bit for bit.
//
// Roofline: octave 0 is HBM-bound on the plane stores (per octave pixel
// 4(S+3) + 4(S+2) bytes written against 1 byte of input read); the small
// octaves, whose radii double per octave, are bound by fp64 FMA issue.
#include <cstdlib>
#include <utility>

#include "sift_common.h"
#include "sift_kernels.h"
#include "sift_xmask.h"

#include <vector>

namespace sift {

constexpr int kGX = 64;              // tile columns
constexpr int kGY = 32;              // tile rows: 4 waves x 8
constexpr int kUR = 16;              // radii with unrolled code (octave 0)
#ifndef SIFT_UR1
#define SIFT_UR1 12
#endif
#ifndef SIFT_STORE_AUX
#define SIFT_STORE_AUX 18 // cache-policy bits of the plane stores (gfx950: 1 sc0, 2 nt, 16 sc1)
#endif
#ifndef SIFT_MINW1
#define SIFT_MINW1 1
#endif
#ifndef SIFT_W96
#define SIFT_W96 1  // 96-column kernel: minimum waves per SIMD (register budget; experiments)
#endif
#ifndef SIFT_TW96_OPQ
#define SIFT_TW96_OPQ 0  // 96-column kernel: per-scale opaque copies of the item map (1 with SIFT_TW96_SEQ 0)
#endif
#ifndef SIFT_TW96_SEQ
#define SIFT_TW96_SEQ 2  // 96-column kernel: horizontal items 0-1 side by side then 2, each group with its epilogue
                         // (122 VGPRs, 4 waves/SIMD; 1 = one at a time, 0 = all three interleaved, 138 VGPRs)
#endif
#ifndef SIFT_B128MAP
#define SIFT_B128MAP 1  // 96-column kernel: conflict-free ds_read_b128 item map (b128_group)
#endif
#ifndef SIFT_PF96
#define SIFT_PF96 2
#endif
#ifndef SIFT_VERT2
#define SIFT_VERT2 1  // octaves >= 1: two columns per lane, 16-byte loads (vert_glob2)
#endif
#ifndef SIFT_V2PF
#define SIFT_V2PF 4  // 16-byte rows in flight in vert_glob2 (4 and 6 measured equal; 4: 108 VGPRs)
#endif
constexpr bool kVert2 = SIFT_VERT2 != 0;
#ifndef SIFT_VGEN2
#define SIFT_VGEN2 1  // ... and for the generic radii up to 32 (vert_glob_gen2)
#endif
constexpr bool kVertGen2 = SIFT_VGEN2 != 0;
constexpr int kUR1 = SIFT_UR1;       // ... octaves >= 1 (SGPR budget: taps are SGPR operands)
constexpr int kUR96 = kUR1 < 12 ? kUR1 : 12;  // ... 96-column tiles (96 + 2r columns in 64 lanes x 2)
constexpr int kCG = kGX / 4;         // column groups of 4 outputs (16)
constexpr int kRS = 64 / kCG;        // row sub-groups per wave (4)
constexpr int kNR = 8 / kRS;         // rows per lane in the horizontal pass (2)
constexpr int kBW0 = kGX / 2 + kUR + 4;  // staged octave-0 region width (input columns)
constexpr int kPFV = 12;             // rows in flight, vertical pass from global memory
constexpr int kPFL = 4;              // rows in flight, vertical pass from LDS
constexpr int kPFH = 3;              // 16-byte reads in flight, horizontal pass
constexpr int kVertNO = 16;          // k_gauss_vert: rows per wave
constexpr int kVertRows = 4 * kVertNO;  // ... per block

__host__ __device__ constexpr int fl2(int a) { return a >> 1; }   // floor(a / 2)
__host__ __device__ constexpr int cl2(int a) { return (a + 1) >> 1; }  // ceil(a / 2), a >= 0

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct GTile {
  int h, w, x0, y0;
  int bx;              // tile column
  int lane, wv;        // wv wave-uniform (SGPR)
  int cg, rs;          // horizontal mapping (64-column tiles)
  int icg[4], irow[4]; // 96- / 128-column tiles: item i of the lane = columns 4 icg .. +3 of wave row irow
  int sw;              // strip stride
  int hrm;             // octave 0: ceil(RM / 2) of the staged region
  const double* S0;    // octave 0: staged input region [..][kBW0]
  __amdgpu_buffer_rsrc_t rsrc;  // o >= 1 (or materialised octave 0): fp64 base plane h x w
};

// ds_read_b128 serves a wave in four 16-lane groups, {0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32; lane -> (group, position in group).
__device__ __forceinline__ void b128_group(int lane, int& g, int& j) {
  const int l = lane & 31;
  int ga, ja;
  if (l < 4) ga = 0, ja = l;
  else if (l < 12) ga = 1, ja = l - 4;
  else if (l < 16) ga = 0, ja = l - 8;
  else if (l < 20) ga = 1, ja = l - 8;
  else if (l < 28) ga = 0, ja = l - 12;
  else ga = 1, ja = l - 16;
  g = 2 * (lane >> 5) + ga;
  j = ja;
}

// Register pinning: an empty asm that reads and writes the accumulators and
// clobbers memory.  The compiler keeps the source order of the fma chains
// and cannot hoist later loads above it, so the register window stays the
// size written (the scheduling-barrier builtin does not stop the selection
// DAG from delaying whole fma chains and keeping every loaded value alive).
template <int N>
__device__ __forceinline__ void pin(double (&a)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i])::"memory");
}

// LDS hand-off between the lanes of ONE wave: the wave's LDS operations
// execute in order, so waiting for its own outstanding ones (and keeping the
// compiler from moving LDS accesses across) is all the ordering needed.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Block barrier that orders LDS only: __syncthreads() is a release/acquire
// fence at workgroup scope and would also wait for every outstanding plane
// store of the wave (they are fire-and-forget otherwise).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Buffer descriptor of a wave-uniform pointer, the pointer's halves taken
// through readfirstlane: a per-scale plane offset the compiler computed in
// VGPRs (s * plane as a 64-bit VALU product) otherwise makes the descriptor
// divergent and every store through it a waterfall loop (4 readfirstlanes,
// compares and an exec loop per store instruction; r6 ISA of k_gauss_rw).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t urs(const void* p, unsigned bytes) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* q = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ double load_f64(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}

// ---------------------------------------------------------------------------
// Vertical window: acc[t] = sum_k w_k row_{t+k} (t < NO, k <= 2R) over the
// rows ld() returns in order, kPFV loads in flight.
// ---------------------------------------------------------------------------
template <int R, int NO, class Ld>
__device__ __forceinline__ void vwin(const cdouble* wp, Ld&& ld, double (&acc)[NO]) {
  constexpr int NJ = 2 * R + NO;
  constexpr int PF = NJ < kPFV ? NJ : kPFV;
  double v[NJ];
#pragma unroll
  for (int t = 0; t < NO; ++t) acc[t] = 0.0;
#pragma unroll
  for (int j = 0; j < PF; ++j) v[j] = ld();
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (j + PF < NJ) v[j + PF] = ld();
#pragma unroll
    for (int t = 0; t < NO; ++t) {
      const int k = j - t;
      if (k >= 0 && k <= 2 * R) acc[t] = fma((double)wp[k], v[j], acc[t]);
    }
    pin(acc);  // program order: loads and fma chains stay in their iteration
  }
}

// ---------------------------------------------------------------------------
// Vertical pass, base plane in global memory (L1/L2), this wave's rows:
// V[8 wv + t][c] = sum_k w_k B[y0 + 8 wv + t - R + k][x0 - R + c],
// c in [0, 64 + 2R).  Pass A: columns 0..63, one lane each, 8 rows.  Pass B:
// the 2R halo columns, lane -> (column 64 + l % 2R, row slice l / 2R of RB
// rows), so few lanes idle.
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void vert_glob(const GTile& T, const cdouble* wp, double* V) {
  const int yb = __builtin_amdgcn_readfirstlane(T.y0 + 8 * T.wv - R);
  const int w8 = T.w * 8;
  double* Vw = V + 8 * T.wv * T.sw;
  {
    const int xoff = clampi(T.x0 - R + T.lane, 0, T.w - 1) * 8;
    // Row offsets from a loop-carried SGPR counter (opaque to the compiler,
    // so it cannot precompute one SGPR per row of the window).
    int yy = yb;
    auto ld = [&]() -> double {
      const double v = load_f64(T.rsrc, xoff, clampi(yy, 0, T.h - 1) * w8);
      asm volatile("" : "+s"(yy));
      yy += 1;
      return v;
    };
    double acc[8];
    vwin<R, 8>(wp, ld, acc);
#pragma unroll
    for (int t = 0; t < 8; ++t) Vw[t * T.sw + T.lane] = acc[t];
  }
  if constexpr (R > 0) {
    constexpr int NB = 2 * R;
    static_assert(NB <= 64, "halo columns fit one packed pass");
    constexpr int G = 64 / NB;              // row slices side by side
    constexpr int RB = (8 + G - 1) / G;     // rows per slice
    constexpr int NSL = (8 + RB - 1) / RB;  // slices in use
    const int col = T.lane % NB, sl = T.lane / NB;
    if (sl < NSL) {
      const int lr = sl * RB;
      const int xoff = clampi(T.x0 - R + kGX + col, 0, T.w - 1) * 8;
      double acc[RB];
      if (yb >= 0 && yb + NSL * RB - 1 + 2 * R <= T.h - 1) {  // interior: no row clamping
        const int vo = xoff + lr * w8;
        int yy = yb;
        auto ld = [&]() -> double {
          const double v = load_f64(T.rsrc, vo, yy * w8);
          asm volatile("" : "+s"(yy));
          yy += 1;
          return v;
        };
        vwin<R, RB>(wp, ld, acc);
      } else {
        int yy = yb + lr;
        auto ld = [&]() -> double {
          const double v = load_f64(T.rsrc, xoff + clampi(yy, 0, T.h - 1) * w8, 0);
          yy += 1;
          return v;
        };
        vwin<R, RB>(wp, ld, acc);
      }
#pragma unroll
      for (int t = 0; t < RB; ++t)
        if (lr + t < 8) Vw[(lr + t) * T.sw + kGX + col] = acc[t];
    }
  }
}

// The same vertical pass with two adjacent strip columns per lane and one
// 16-byte load per row: the (64 + 2R) columns in ONE packed pass (no separate
// halo pass) and half the load instructions of vert_glob -- the octave-1
// launch is bound by its vertical loads' address processing (TA busy 0.84).
// Column clamping: the pair (x, x+1) is read at xa = clamp(x, 0, w - 2); at
// the left edge both columns are B[0] (the pair's first), at the right edge
// both are B[w-1] (its second).  Same fma chain per column, bit-identical.
template <int R, int TW = kGX>
__device__ __forceinline__ void vert_glob2(const GTile& T, const cdouble* wp, double* V) {
  constexpr int NC = TW + 2 * R;  // even
  constexpr int NPAIR = NC / 2;
  static_assert(NPAIR <= 64, "one lane per column pair");
  constexpr int NJ = 2 * R + 8;
  constexpr int PF = NJ < SIFT_V2PF ? NJ : SIFT_V2PF;  // 16-byte rows in flight
  const int p = T.lane;
  if (p >= NPAIR) return;
  const int yb = __builtin_amdgcn_readfirstlane(T.y0 + 8 * T.wv - R);
  const int w8 = T.w * 8;
  const int x = T.x0 - R + 2 * p;
  const int xoff = clampi(x, 0, T.w - 2) * 8;
  double a0[8], a1[8];
  double2 v[NJ];
  auto run = [&](auto ld) {
#pragma unroll
    for (int t = 0; t < 8; ++t) a0[t] = a1[t] = 0.0;
#pragma unroll
    for (int j = 0; j < PF; ++j) v[j] = ld();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j + PF < NJ) v[j + PF] = ld();
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int k = j - t;
        if (k >= 0 && k <= 2 * R) {
          a0[t] = fma((double)wp[k], v[j].x, a0[t]);
          a1[t] = fma((double)wp[k], v[j].y, a1[t]);
        }
      }
      pin(a0);
      pin(a1);
    }
  };
  int yy = yb;
  auto raw = [&]() -> double2 {
    const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(T.rsrc, xoff, clampi(yy, 0, T.h - 1) * w8, 0);
    asm volatile("" : "+s"(yy));
    yy += 1;
    return __builtin_bit_cast(double2, q);
  };
  // Tiles whose strip columns x0 - R .. x0 + TW + R - 1 all lie inside the
  // plane (wave-uniform) need no edge selects (4 VALU per 16-byte row).
  if (T.x0 - R >= 0 && T.x0 + TW + R <= T.w) {
    run(raw);
  } else {
    const bool lo_edge = x < 0, hi_edge = x >= T.w - 1;
    run([&]() -> double2 {
      const double2 d = raw();
      return make_double2(hi_edge ? d.y : d.x, lo_edge ? d.x : d.y);
    });
  }
  double* Vw = V + 8 * T.wv * T.sw + 2 * p;
#pragma unroll
  for (int t = 0; t < 8; ++t) *reinterpret_cast<double2*>(Vw + t * T.sw) = make_double2(a0[t], a1[t]);
}

// Generic radii: rows in chunks of 8 (chunk base jb), output t of the
// wave's 8 rows takes tap jb + k - t of chunk row k.  Taps outside [0, 2r]
// are zero and fma(0, v, acc) == acc, so the chunks skip them: the first
// chunk (jb = 0) has no taps for k < t, a tail chunk none for k - t > M =
// 2r - jb (and loads no row k > M + 7, past the window).  The same fma
// chains as the zero-padded form, term for term.
template <int M>
struct VChunk {
  static constexpr int kRows = M + 8 < 8 ? M + 8 : 8;  // rows k <= M + 7
  template <bool FIRST, class Fma>
  __device__ __forceinline__ static void run(Fma&& f) {
#pragma unroll
    for (int k = 0; k < kRows; ++k)
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (!(FIRST && k < t) && k - t <= M) f(k, t);
  }
};
// NO outputs per lane (k_gauss_vert: 16 rows per wave, half the window
// rows loaded per output): rows k <= M + NO - 1, the same skips.
template <int M, int NO>
struct VChunkN {
  static constexpr int kRows = M + NO < 8 ? M + NO : 8;
  template <bool FIRST, class Fma>
  __device__ __forceinline__ static void run(Fma&& f) {
#pragma unroll
    for (int k = 0; k < kRows; ++k)
#pragma unroll
      for (int t = 0; t < NO; ++t)
        if (!(FIRST && k < t) && k - t <= M) f(k, t);
  }
};
// m = 2r - jb (even): one body per tail (no zero taps at all: a chunk of 16
// outputs would spend most of a tail's 128 pairs on them).
template <bool FIRST, class Body>
__device__ __forceinline__ void vchunk16_dispatch(int m, Body&& body) {
  using F = std::integral_constant<bool, FIRST>;
  using N = std::integral_constant<bool, false>;
  if (FIRST) {
    if (m >= 7) body(VChunkN<7, 16>{}, F{});
    else body(VChunkN<7, 16>{}, N{});  // 2r < 7: zero-padded taps on both sides
    return;
  }
  switch (m >= 7 ? 7 : m) {
    case 7: body(VChunkN<7, 16>{}, N{}); break;
    case 6: body(VChunkN<6, 16>{}, N{}); break;
    case 4: body(VChunkN<4, 16>{}, N{}); break;
    case 2: body(VChunkN<2, 16>{}, N{}); break;
    case 0: body(VChunkN<0, 16>{}, N{}); break;
    case -2: body(VChunkN<-2, 16>{}, N{}); break;
    case -4: body(VChunkN<-4, 16>{}, N{}); break;
    case -6: body(VChunkN<-6, 16>{}, N{}); break;
    case -8: body(VChunkN<-8, 16>{}, N{}); break;
    case -10: body(VChunkN<-10, 16>{}, N{}); break;
    case -12: body(VChunkN<-12, 16>{}, N{}); break;
    default: body(VChunkN<-14, 16>{}, N{}); break;
  }
}

// m = 2r - jb (even).  Full chunks, and tail chunks with m >= 0, run all 64
// (k, t) pairs (a tail's few taps past 2r are zero padding); the first chunk
// skips its k < t triangle, the last chunks with m < 0 their rows past the
// window -- five bodies, so the register allocation of the kernel is not
// driven by a variant per radius.
template <bool FIRST, class Body>
__device__ __forceinline__ void vchunk_dispatch(int m, Body&& body) {
  using F = std::integral_constant<bool, FIRST>;
  using N = std::integral_constant<bool, false>;
  if (FIRST) {
    if (m >= 7) body(VChunk<7>{}, F{});
    else body(VChunk<7>{}, N{});  // 2r < 7: zero-padded taps on both sides
  } else if (m >= 0) {
    body(VChunk<7>{}, N{});
  } else if (m == -2) {
    body(VChunk<-2>{}, N{});
  } else if (m == -4) {
    body(VChunk<-4>{}, N{});
  } else {
    body(VChunk<-6>{}, N{});
  }
}

// vert_glob_gen with two columns per lane and 16-byte loads (radii up to 32:
// the 64 + 2r columns in one packed pass); the same 8-row chunks over
// zero-padded taps, so the same fma chains as vert_glob_gen.
__device__ __forceinline__ void vert_glob_gen2(const GTile& T, int r, const cdouble* wp, double* V) {
  const int NC = kGX + 2 * r, NJ = 2 * r + 8;
  const int p = T.lane;
  if (p >= NC / 2) return;
  const int yb = T.y0 + 8 * T.wv - r;
  const int x = T.x0 - r + 2 * p;
  const int xoff = clampi(x, 0, T.w - 2) * 8;
  const bool lo_edge = x < 0, hi_edge = x >= T.w - 1;
  // Tiles whose strip columns all lie inside the plane (wave-uniform) skip
  // the edge selects (4 VALU per 16-byte row), as in vert_glob2.
  const bool interior = T.x0 - r >= 0 && T.x0 + kGX + r <= T.w;
  double a0[8], a1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) a0[t] = a1[t] = 0.0;
  auto sweep = [&](auto edge) {
    auto chunk = [&](int jb, auto C, auto first) {
      using CC = decltype(C);
      double2 v[8];
#pragma unroll
      for (int k = 0; k < CC::kRows; ++k) {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(
            T.rsrc, xoff, __builtin_amdgcn_readfirstlane(clampi(yb + jb + k, 0, T.h - 1) * T.w * 8), 0);
        const double2 d = __builtin_bit_cast(double2, q);
        if constexpr (decltype(edge)::value) v[k] = make_double2(hi_edge ? d.y : d.x, lo_edge ? d.x : d.y);
        else v[k] = d;
      }
      const cdouble* w = wp + jb;
      CC::template run<decltype(first)::value>([&](int k, int t) {
        a0[t] = fma((double)w[k - t], v[k].x, a0[t]);
        a1[t] = fma((double)w[k - t], v[k].y, a1[t]);
      });
      pin(a0);
      pin(a1);
    };
    vchunk_dispatch<true>(2 * r, [&](auto C, auto f) { chunk(0, C, f); });
    for (int jb = 8; jb < NJ; jb += 8)
      vchunk_dispatch<false>(2 * r - jb, [&](auto C, auto f) { chunk(jb, C, f); });
  };
  if (interior) sweep(std::false_type{});
  else sweep(std::true_type{});
  double* Vw = V + 8 * T.wv * T.sw + 2 * p;
#pragma unroll
  for (int t = 0; t < 8; ++t) *reinterpret_cast<double2*>(Vw + t * T.sw) = make_double2(a0[t], a1[t]);
}

__device__ __forceinline__ void vert_glob_gen(const GTile& T, int r, const cdouble* wp, double* V) {
  const int NC = kGX + 2 * r, NJ = 2 * r + 8;
  const int yb = T.y0 + 8 * T.wv - r;
  for (int cb = 0; cb < NC; cb += 64) {
    const int c = cb + T.lane;
    const int xoff = clampi(T.x0 - r + min(c, NC - 1), 0, T.w - 1) * 8;
    double acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = 0.0;
    for (int jb = 0; jb < NJ; jb += 8) {
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[k] = load_f64(T.rsrc, xoff, __builtin_amdgcn_readfirstlane(clampi(yb + jb + k, 0, T.h - 1) * T.w * 8));
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = fma((double)wp[jb + k - t], v[k], acc[t]);  // zero-padded taps
      pin(acc);
    }
    if (c < NC) {
      double* dst = V + 8 * T.wv * T.sw + c;
#pragma unroll
      for (int t = 0; t < 8; ++t) dst[t * T.sw] = acc[t];
    }
  }
}

// ---------------------------------------------------------------------------
// Split vertical pass (large radii, gauss_vsplit).  A 64-column tile
// recomputes the vertical sums of its 2r halo columns: (64 + 2r) / 64 of the
// vertical work (2.5x at r = 47, 6.9x at r = 188), serialised in the tile's
// waves.  k_gauss_vert computes every (scale, row, column) sum once, one lane
// per column and eight rows per wave, into fp64 scratch planes, with
// vert_glob_gen's exact chunking (rows yb + jb + k, zero-padded taps in
// increasing order from 0.0): every value is bit-identical to the tile
// kernel's own.  The tile kernel then copies its strip (vert_copy).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gauss_vert(const Pyramid P, int o, const double* __restrict__ base,
                                                    double* __restrict__ vout, long long bstride,
                                                    long long vstride) {
  const Octave& oc = P.oct[o];
  // z = image * NS + (NS - 1 - scale): largest radius (longest chains) first,
  // blocks are dispatched in z order
  const int im = (int)blockIdx.z / P.NS;
  const int s = P.NS - 1 - ((int)blockIdx.z - im * P.NS);
  base += im * bstride;
  vout += im * vstride;
  const int r = oc.rad[s], h = oc.h, w = oc.w;
  const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int x = blockIdx.x * kGX + lane;
  const int y0 = blockIdx.y * kVertRows + kVertNO * wv;
  if (y0 >= h) return;  // wave-uniform
  const __amdgpu_buffer_rsrc_t rs = urs(const_cast<double*>(base), h * w * 8);
  const int xoff = min(x, w - 1) * 8;
  const int NJ = 2 * r + kVertNO, yb = y0 - r;
  double acc[kVertNO];
#pragma unroll
  for (int t = 0; t < kVertNO; ++t) acc[t] = 0.0;
  auto chunk = [&](int jb, auto C, auto first) {
    using CC = decltype(C);
    double v[8];
#pragma unroll
    for (int k = 0; k < CC::kRows; ++k)
      v[k] = load_f64(rs, xoff, __builtin_amdgcn_readfirstlane(clampi(yb + jb + k, 0, h - 1) * w * 8));
    const cdouble* wq = wp + jb;
    CC::template run<decltype(first)::value>([&](int k, int t) { acc[t] = fma((double)wq[k - t], v[k], acc[t]); });
    pin(acc);
  };
  // 16 rows per wave: the window's 2r + 16 rows serve 16 outputs (2r + 8
  // for 8 before: 12.75 -> 6.9 loads per output at r = 47), the same fma
  // chain per output (taps in increasing order from 0.0).
  vchunk16_dispatch<true>(2 * r, [&](auto C, auto f) { chunk(0, C, f); });
  for (int jb = 8; jb < NJ; jb += 8)
    vchunk16_dispatch<false>(2 * r - jb, [&](auto C, auto f) { chunk(jb, C, f); });
  if (x < w) {
    double* dst = vout + (long long)s * h * w + (long long)y0 * w + x;
#pragma unroll
    for (int t = 0; t < kVertNO; ++t)
      if (y0 + t < h) dst[(long long)t * w] = acc[t];
  }
}

// The wave's 8 strip rows, columns x0 - r .. x0 + 63 + r (clamped), from the
// split pass's plane of this scale; rows past the plane (outputs dropped)
// read its last row.
__device__ __forceinline__ void vert_copy(const GTile& T, int r, const double* __restrict__ src, double* V) {
  const int NC = kGX + 2 * r;
  double* Vw = V + 8 * T.wv * T.sw;
  const int yr = T.y0 + 8 * T.wv;
  for (int cb = 0; cb < NC; cb += 64) {
    const int c = cb + T.lane;
    const int xo = clampi(T.x0 - r + min(c, NC - 1), 0, T.w - 1);
    double v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = src[(long long)min(yr + t, T.h - 1) * T.w + xo];
    if (c < NC)
#pragma unroll
      for (int t = 0; t < 8; ++t) Vw[t * T.sw + c] = v[t];
  }
}

// ---------------------------------------------------------------------------
// Vertical pass, octave 0, staged input region: input column kb + c (kb =
// x0/2 - ceil(r/2)), output rows e + t (e = y0 + 8 wv, even).  Tap k of
// output row e + t reads input row e/2 + floor((t + k - r)/2), i.e. window
// row m = floor((t + k - r)/2) + ceil(r/2).
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void vert_o0(const GTile& T, const cdouble* wp, double* V) {
  constexpr int HR = cl2(R);
  constexpr int NC = fl2(kGX - 1 + R) + HR + 1;
  constexpr int M = fl2(7 + R) + HR + 1;
  static_assert(NC <= 64, "one lane per input column");
  const int c = T.lane;
  if (c < NC) {
    const double* sp = T.S0 + (4 * T.wv + T.hrm - HR) * kBW0 + (c + T.hrm - HR);
    double acc[8], v[M];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = 0.0;
#pragma unroll
    for (int m = 0; m < kPFL && m < M; ++m) v[m] = sp[m * kBW0];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m + kPFL < M) v[m + kPFL] = sp[(m + kPFL) * kBW0];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const int k = 2 * (m - HR) + R - t + d;
          if (k >= 0 && k <= 2 * R) acc[t] = fma((double)wp[k], v[m], acc[t]);
        }
      }
      pin(acc);
    }
    double* dst = V + 8 * T.wv * T.sw + c;
#pragma unroll
    for (int t = 0; t < 8; ++t) dst[t * T.sw] = acc[t];
  }
}

// ---------------------------------------------------------------------------
// Horizontal pass: lane -> columns 4 cg .. 4 cg + 3, rows 8 wv + rs + 4 i.
// o >= 1: out[q] = sum_k w_k V[row][4 cg + q + k].
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void horz_full(const GTile& T, const cdouble* wp, const double* V,
                                          double (&out)[kNR][4]) {
  // Both rows of the lane in one loop: 8 independent fma chains per wave
  // (4 leave the fp64 pipeline latency exposed).
  constexpr int NP = R + 2;  // double2 pairs per row
  const double* rp[kNR];
  double2 u[kNR][NP];
#pragma unroll
  for (int i = 0; i < kNR; ++i) {
    rp[i] = V + (8 * T.wv + T.rs + kRS * i) * T.sw + 4 * T.cg;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[i][q] = 0.0;
  }
#pragma unroll
  for (int n2 = 0; n2 < kPFH && n2 < NP; ++n2)
#pragma unroll
    for (int i = 0; i < kNR; ++i) u[i][n2] = *reinterpret_cast<const double2*>(rp[i] + 2 * n2);
#pragma unroll
  for (int n2 = 0; n2 < NP; ++n2) {
    if (n2 + kPFH < NP)
#pragma unroll
      for (int i = 0; i < kNR; ++i) u[i][n2 + kPFH] = *reinterpret_cast<const double2*>(rp[i] + 2 * (n2 + kPFH));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * n2 + e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = n - q;
        if (k >= 0 && k <= 2 * R)
#pragma unroll
          for (int i = 0; i < kNR; ++i) out[i][q] = fma((double)wp[k], e ? u[i][n2].y : u[i][n2].x, out[i][q]);
      }
    }
#pragma unroll
    for (int i = 0; i < kNR; ++i) pin(out[i]);
  }
}

// 96-column tiles (octaves >= 1 whose radii are all unrolled): 24 column
// groups x 8 rows = 192 items of 4 columns x 1 row, three per lane (item i =
// lane + 64 i), so the 64 + 2r-column vertical pass of a 64-wide tile becomes
// a 96 + 2r one with (96 + 2r) / 128 instead of (64 + 2r) / 128 of its lanes
// busy and a third fewer loads per output.  Same fma chain per output.
template <int R>
__device__ __forceinline__ void horz_full96(const GTile& T, const cdouble* wp, const double* V, double (&out)[3][4]) {
  constexpr int NP = R + 2;  // double2 pairs per row
  constexpr int PF96 = SIFT_PF96;  // 16-byte reads in flight per item
  const double* rp[3];
  double2 u[3][NP];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    rp[i] = V + (8 * T.wv + T.irow[i]) * T.sw + 4 * T.icg[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) out[i][q] = 0.0;
  }
#pragma unroll
  for (int n2 = 0; n2 < PF96 && n2 < NP; ++n2)
#pragma unroll
    for (int i = 0; i < 3; ++i) u[i][n2] = *reinterpret_cast<const double2*>(rp[i] + 2 * n2);
#pragma unroll
  for (int n2 = 0; n2 < NP; ++n2) {
    if (n2 + PF96 < NP)
#pragma unroll
      for (int i = 0; i < 3; ++i) u[i][n2 + PF96] = *reinterpret_cast<const double2*>(rp[i] + 2 * (n2 + PF96));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * n2 + e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = n - q;
        if (k >= 0 && k <= 2 * R)
#pragma unroll
          for (int i = 0; i < 3; ++i) out[i][q] = fma((double)wp[k], e ? u[i][n2].y : u[i][n2].x, out[i][q]);
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) pin(out[i]);
  }
}

// The same, one item at a time, each handed to epi(i, out) as soon as its
// 4 chains are done: only one item's accumulators and reads are live
// (SIFT_TW96_SEQ; the interleaved form keeps all three).
// Items [I0, I0 + NI) of the lane side by side (4 NI fma chains).
template <int R, int I0, int NI, class Epi>
__device__ __forceinline__ void horz96_group(const GTile& T, const cdouble* wp, const double* V, Epi&& epi) {
  constexpr int NP = R + 2;  // double2 pairs per row
  constexpr int PF = kPFH;
  const double* rp[NI];
  double out[NI][4];
  double2 u[NI][NP];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    rp[j] = V + (8 * T.wv + T.irow[I0 + j]) * T.sw + 4 * T.icg[I0 + j];
#pragma unroll
    for (int q = 0; q < 4; ++q) out[j][q] = 0.0;
  }
#pragma unroll
  for (int n2 = 0; n2 < PF && n2 < NP; ++n2)
#pragma unroll
    for (int j = 0; j < NI; ++j) u[j][n2] = *reinterpret_cast<const double2*>(rp[j] + 2 * n2);
#pragma unroll
  for (int n2 = 0; n2 < NP; ++n2) {
    if (n2 + PF < NP)
#pragma unroll
      for (int j = 0; j < NI; ++j) u[j][n2 + PF] = *reinterpret_cast<const double2*>(rp[j] + 2 * (n2 + PF));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * n2 + e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = n - q;
        if (k >= 0 && k <= 2 * R)
#pragma unroll
          for (int j = 0; j < NI; ++j) out[j][q] = fma((double)wp[k], e ? u[j][n2].y : u[j][n2].x, out[j][q]);
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) pin(out[j]);
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) epi(I0 + j, out[j]);
}

// SIFT_TW96_SEQ 1: items one at a time; 2: items 0-1 side by side, then 2.
template <int R, class Epi>
__device__ __forceinline__ void horz_full96_seq(const GTile& T, const cdouble* wp, const double* V, Epi&& epi) {
  if constexpr (SIFT_TW96_SEQ == 2) {
    horz96_group<R, 0, 2>(T, wp, V, epi);
    horz96_group<R, 2, 1>(T, wp, V, epi);
  } else {
    horz96_group<R, 0, 1>(T, wp, V, epi);
    horz96_group<R, 1, 1>(T, wp, V, epi);
    horz96_group<R, 2, 1>(T, wp, V, epi);
  }
}

__device__ __forceinline__ void horz_full_gen(const GTile& T, int r, const cdouble* wp, const double* V,
                                              double (&out)[kNR][4]) {
  const int NV = 2 * r + 4;
  const double* rp[kNR];
#pragma unroll
  for (int i = 0; i < kNR; ++i) {
    rp[i] = V + (8 * T.wv + T.rs + kRS * i) * T.sw + 4 * T.cg;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[i][q] = 0.0;
  }
  for (int nb = 0; nb < NV; nb += 8) {
    double u[kNR][8];
#pragma unroll
    for (int i = 0; i < kNR; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double2 p = *reinterpret_cast<const double2*>(rp[i] + nb + 2 * e);
        u[i][2 * e] = p.x;
        u[i][2 * e + 1] = p.y;
      }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < kNR; ++i) out[i][q] = fma((double)wp[nb + e - q], u[i][e], out[i][q]);  // zero-padded taps
#pragma unroll
    for (int i = 0; i < kNR; ++i) pin(out[i]);
  }
}

// Octave 0: strip column n <-> input column x0/2 - ceil(r/2) + n; tap k of
// output column x0 + 4 cg + q reads strip column 2 cg + floor((q + k - r)/2) + ceil(r/2).
template <int R>
__device__ __forceinline__ void horz_o0(const GTile& T, const cdouble* wp, const double* V,
                                        double (&out)[kNR][4]) {
  constexpr int HR = cl2(R);
  constexpr int NP = (fl2(R + 3) + HR + 2) / 2;  // double2 pairs per row
  const double* rp[kNR];
  double2 u[kNR][NP];
#pragma unroll
  for (int i = 0; i < kNR; ++i) {
    rp[i] = V + (8 * T.wv + T.rs + kRS * i) * T.sw + 2 * T.cg;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[i][q] = 0.0;
  }
#pragma unroll
  for (int n2 = 0; n2 < kPFH && n2 < NP; ++n2)
#pragma unroll
    for (int i = 0; i < kNR; ++i) u[i][n2] = *reinterpret_cast<const double2*>(rp[i] + 2 * n2);
#pragma unroll
  for (int n2 = 0; n2 < NP; ++n2) {
    if (n2 + kPFH < NP)
#pragma unroll
      for (int i = 0; i < kNR; ++i) u[i][n2 + kPFH] = *reinterpret_cast<const double2*>(rp[i] + 2 * (n2 + kPFH));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * n2 + e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const int k = 2 * (n - HR) + R - q + d;
          if (k >= 0 && k <= 2 * R)
#pragma unroll
            for (int i = 0; i < kNR; ++i) out[i][q] = fma((double)wp[k], e ? u[i][n2].y : u[i][n2].x, out[i][q]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kNR; ++i) pin(out[i]);
  }
}

// ---------------------------------------------------------------------------
// Radius dispatch (uniform branch): a binary search over the unrolled radii
// LO..HI (log2 compares and branches per dispatch instead of a compare chain
// of up to HI; every scale of every block dispatches twice).
// ---------------------------------------------------------------------------
template <int LO, int HI, class F>
__device__ __forceinline__ void rdispatch(int r, F&& f) {
  if constexpr (LO == HI) {
    f(std::integral_constant<int, LO>{});
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (r <= MID) rdispatch<LO, MID>(r, f);
    else rdispatch<MID + 1, HI>(r, f);
  }
}

#ifndef SIFT_BIN_STREAM
#define SIFT_BIN_STREAM 1  // binary radius dispatch in the streamed k_gauss_rw<RW, true> too
#endif
#ifndef SIFT_BIN_TILE
#define SIFT_BIN_TILE 1  // binary radius dispatch in the k_gauss_dog tile kernels of octaves >= 1
#endif
#ifndef SIFT_BIN_OCT0
#define SIFT_BIN_OCT0 1  // ... and in octave 0's (bit 0: vertical pass, bit 1: horizontal: +13 VGPRs)
#endif
// Measured (r6f / r6g, profiles/r6g_radius_dispatch_ab.txt): 4K octave 1
// (register window) 0.162 -> 0.149 ms, octave 2 (streamed) 0.095 -> 0.089 ms,
// octave 3's tiles -2 us; octave 0 keeps the compare chain (the binary form
// takes it from 92 to 105 VGPRs, 5 -> 4 waves per SIMD: 0.364 -> 0.383 ms;
// bounded to 96 it spills: 0.370 ms).
template <bool OCT0, int... Rs>
__device__ __forceinline__ void vert_any_(std::integer_sequence<int, Rs...>, const GTile& T, int r,
                                         const cdouble* wp, double* V) {
  constexpr int N = sizeof...(Rs) - 1;
  if constexpr (OCT0 ? (SIFT_BIN_OCT0 & 1) : SIFT_BIN_TILE) {
    if constexpr (OCT0) {
      rdispatch<0, N>(r, [&](auto R) { vert_o0<decltype(R)::value>(T, wp, V); });
    } else if (r <= N) {
      if (kVert2 && T.w >= 2) rdispatch<0, N>(r, [&](auto R) { vert_glob2<decltype(R)::value>(T, wp, V); });
      else rdispatch<0, N>(r, [&](auto R) { vert_glob<decltype(R)::value>(T, wp, V); });
    } else if (kVert2 && kVertGen2 && T.w >= 2 && r <= 32) {
      vert_glob_gen2(T, r, wp, V);
    } else {
      vert_glob_gen(T, r, wp, V);
    }
    return;
  }
  bool done = false;
  if constexpr (OCT0) {
    ((!done && r == Rs ? (vert_o0<Rs>(T, wp, V), done = true) : false), ...);
  } else {
    if (kVert2 && T.w >= 2) {
      ((!done && r == Rs ? (vert_glob2<Rs>(T, wp, V), done = true) : false), ...);
      if (kVertGen2 && !done && r <= 32) vert_glob_gen2(T, r, wp, V), done = true;
    } else {
      ((!done && r == Rs ? (vert_glob<Rs>(T, wp, V), done = true) : false), ...);
    }
    if (!done) vert_glob_gen(T, r, wp, V);
  }
}

template <bool OCT0, int... Rs>
__device__ __forceinline__ void horz_any_(std::integer_sequence<int, Rs...>, const GTile& T, int r,
                                         const cdouble* wp, const double* V, double (&out)[kNR][4]) {
  constexpr int N = sizeof...(Rs) - 1;
  if constexpr (OCT0 ? (SIFT_BIN_OCT0 & 2) : SIFT_BIN_TILE) {
    if constexpr (OCT0) {
      rdispatch<0, N>(r, [&](auto R) { horz_o0<decltype(R)::value>(T, wp, V, out); });
    } else if (r <= N) {
      rdispatch<0, N>(r, [&](auto R) { horz_full<decltype(R)::value>(T, wp, V, out); });
    } else {
      horz_full_gen(T, r, wp, V, out);
    }
    return;
  }
  bool done = false;
  if constexpr (OCT0) {
    ((!done && r == Rs ? (horz_o0<Rs>(T, wp, V, out), done = true) : false), ...);
  } else {
    ((!done && r == Rs ? (horz_full<Rs>(T, wp, V, out), done = true) : false), ...);
    if (!done) horz_full_gen(T, r, wp, V, out);
  }
}

template <int... Rs>
__device__ __forceinline__ void vert96_any_(std::integer_sequence<int, Rs...>, const GTile& T, int r,
                                           const cdouble* wp, double* V) {
  if constexpr (SIFT_BIN_TILE) {
    rdispatch<0, sizeof...(Rs) - 1>(r, [&](auto R) { vert_glob2<decltype(R)::value, 96>(T, wp, V); });
    return;
  }
  bool done = false;
  ((!done && r == Rs ? (vert_glob2<Rs, 96>(T, wp, V), done = true) : false), ...);
}
template <int... Rs>
__device__ __forceinline__ void horz96_any_(std::integer_sequence<int, Rs...>, const GTile& T, int r,
                                           const cdouble* wp, const double* V, double (&out)[3][4]) {
  if constexpr (SIFT_BIN_TILE) {
    rdispatch<0, sizeof...(Rs) - 1>(r, [&](auto R) { horz_full96<decltype(R)::value>(T, wp, V, out); });
    return;
  }
  bool done = false;
  ((!done && r == Rs ? (horz_full96<Rs>(T, wp, V, out), done = true) : false), ...);
}

template <class Epi, int... Rs>
__device__ __forceinline__ void horz96s_any_(std::integer_sequence<int, Rs...>, const GTile& T, int r,
                                            const cdouble* wp, const double* V, Epi&& epi) {
  if constexpr (SIFT_BIN_TILE) {
    rdispatch<0, sizeof...(Rs) - 1>(r, [&](auto R) { horz_full96_seq<decltype(R)::value>(T, wp, V, epi); });
    return;
  }
  bool done = false;
  ((!done && r == Rs ? (horz_full96_seq<Rs>(T, wp, V, epi), done = true) : false), ...);
}

// Unrolled radii 0..RMAX.
template <bool OCT0, int RMAX>
__device__ __forceinline__ void vert_any(const GTile& T, int r, const cdouble* wp, double* V) {
  vert_any_<OCT0>(std::make_integer_sequence<int, RMAX + 1>{}, T, r, wp, V);
}
template <bool OCT0, int RMAX>
__device__ __forceinline__ void horz_any(const GTile& T, int r, const cdouble* wp, const double* V,
                                         double (&out)[kNR][4]) {
  horz_any_<OCT0>(std::make_integer_sequence<int, RMAX + 1>{}, T, r, wp, V, out);
}

__device__ __forceinline__ void store4(float* p, const double (&v)[4], int nvalid) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nvalid) p[q] = (float)v[q];
}

// 16-byte buffer store; lanes whose offset is past the plane are dropped by
// the descriptor's range check.
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t rs, int voff, const double (&v)[4]) {
  const float4 f = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), rs, voff, 0, SIFT_STORE_AUX);
}

// ---------------------------------------------------------------------------
// Extrema decisions fused into the pass (XF).  Tiles overlap: a block
// computes 64 x 32 pixels at a stride of kFX x kFY, stores the kFX x kFY it
// owns (the last tile of a row / column all of its in-plane pixels) and
// decides the kFX x kFY pixels one column and one row in from its origin,
// whose 26 neighbours all lie in its tile (translation invariance makes the
// overlapping pixels bit-identical to their owners').  Each scale's DoG tile
// goes to an LDS ring of 3 fp32 planes; once DoG t+1 is there, every wave
// decides scale t for its own rows with the scan's logic (x_row_decide:
// fp32 comparisons, ties and threshold-adjacent values to the exact pass).
// Replaces the scan of this octave: its DoG planes are not read back.
// ---------------------------------------------------------------------------
constexpr int kRingPlane = kGY * kGX;  // floats per ring plane

// Scale t (DoG t-1, t, t+1 in ring slots (t-1)%3, t%3, (t+1)%3) for the
// wave's rows 8 wv .. 8 wv + 7; one lane per tile column.
__device__ __forceinline__ void fused_decide(const Pyramid& P, const GaussLaunch& L, const GTile& T,
                                             const float* ring, int t, unsigned& low) {
  const Octave& oc = P.oct[L.o];
  const int l = T.lane;
  const float* q0 = ring + ((t - 1) % 3) * kRingPlane + l;
  const float* q1 = ring + (t % 3) * kRingPlane + l;
  const float* q2 = ring + ((t + 1) % 3) * kRingPlane + l;
  const int x = T.x0 + l;
  const unsigned long long colmask = __ballot(l >= 1 && l <= kFX && x >= 1 && x <= T.w - 2);
  const unsigned key0 = oc.key_off + (unsigned)(t - 1) * (unsigned)T.h * (unsigned)T.w + (unsigned)x;
  const int r0 = 8 * T.wv;
  XWin<3> Wn;
  auto load = [&](float (&dst)[3], int j) {  // tile row r0 - 1 + j (clamped: only undecided rows read past)
    const int r = clampi(r0 - 1 + j, 0, kGY - 1) * kGX;
    dst[0] = q0[r];
    dst[1] = q1[r];
    dst[2] = q2[r];
  };
  {
    float a[3], b[3];
    load(a, 0);
    load(b, 1);
    x_derive<3, 0>(Wn, a);
    x_derive<3, 1>(Wn, b);
  }
  auto centre = [&](auto A_, auto B_, auto C_, int j) {
    constexpr int A = decltype(A_)::value, B = decltype(B_)::value, C = decltype(C_)::value;
    const int c = r0 + j - 1;  // tile row of the centre
    const int y = T.y0 + c;
    if (c < 1 || c > kFY || y < 1 || y > T.h - 2) return;  // wave-uniform
    const float vx0 = max3f(Wn.hx[A][0], Wn.hx[B][0], Wn.hx[C][0]), vn0 = min3f(Wn.hn[A][0], Wn.hn[B][0], Wn.hn[C][0]);
    const float vx2 = max3f(Wn.hx[A][2], Wn.hx[B][2], Wn.hx[C][2]), vn2 = min3f(Wn.hn[A][2], Wn.hn[B][2], Wn.hn[C][2]);
    const float v = Wn.cv[B][1];
    const float nmax = max3f(vx0, vx2, max3f(Wn.hx[A][1], Wn.hx[C][1], Wn.ex[B][1]));
    const float nmin = min3f(vn0, vn2, min3f(Wn.hn[A][1], Wn.hn[C][1], Wn.en[B][1]));
    unsigned long long ambmask;  // (the fused path lists ambiguous keys itself)
    unsigned long long lowmask;  // the low-contrast list is not fused (build_common)
    const unsigned long long bit =
        x_row_decide(v, nmax, nmin, colmask, L.X.c_lo, L.X.c_hi, false, key0 + (unsigned)y * (unsigned)T.w,
                     &L.X.counters[0], L.X.amb_keys, L.X.amb_cap, low, lowmask, ambmask);
    const unsigned long long word = bit >> 1;  // lanes 1..kFX -> bits 0..kFX-1
    if (l == 0) {
      const long long row = (long long)(t - 1) * T.h + y;
      L.X.bitmap[row * L.X.nw + T.bx] = word;
      if (word) atomicAdd(&L.X.rowcount[row], (unsigned)__popcll(word));
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  // rows j = 2..9 are derived into slot j % 3, centre row j - 1 uses slots (j-2, j-1, j) % 3
  {
    float a[3];
    load(a, 2); x_derive<3, 2>(Wn, a); centre(I0{}, I1{}, I2{}, 1);
    load(a, 3); x_derive<3, 0>(Wn, a); centre(I1{}, I2{}, I0{}, 2);
    load(a, 4); x_derive<3, 1>(Wn, a); centre(I2{}, I0{}, I1{}, 3);
    load(a, 5); x_derive<3, 2>(Wn, a); centre(I0{}, I1{}, I2{}, 4);
    load(a, 6); x_derive<3, 0>(Wn, a); centre(I1{}, I2{}, I0{}, 5);
    load(a, 7); x_derive<3, 1>(Wn, a); centre(I2{}, I0{}, I1{}, 6);
    load(a, 8); x_derive<3, 2>(Wn, a); centre(I0{}, I1{}, I2{}, 7);
    load(a, 9); x_derive<3, 0>(Wn, a); centre(I1{}, I2{}, I0{}, 8);
  }
}

// SWC > 0: compile-time strip stride (immediate LDS offsets); 0: L.sw.
// RMAX: radii with unrolled code.  XF: extrema decisions fused (above).
// TW: tile width (64; 96 for octaves >= 1 whose radii are all unrolled,
// horz_full96); NI items of 4 columns x 1 row per lane in the horizontal pass
// and the epilogue.
#ifndef SIFT_VS_KERNEL
#define SIFT_VS_KERNEL 1  // split-pass octaves run the VS instance of the tile kernel
#endif
#ifndef SIFT_VS_RMAX
#define SIFT_VS_RMAX 12  // ... with unrolled horizontal radii up to this
#endif
#ifndef SIFT_W0
#define SIFT_W0 1  // octave-0 tile kernel: minimum blocks (= waves) per SIMD the register allocation must allow
#endif
// VS: the split-pass instance (octaves with a k_gauss_vert launch): its strips
// come from the split pass's vertical sums only, so the vertical radius
// variants are not compiled into it (round 6: the shared instance spilled
// 126 SGPRs into VGPR lanes, readlane / writelane in every scale).
template <bool OCT0, int SWC, int RMAX, bool XF, int TW = kGX, bool VS = false>
__global__ __launch_bounds__(256, OCT0 ? SIFT_W0 : (TW == 96 ? SIFT_W96 : SIFT_MINW1)) void k_gauss_dog(const Pyramid P, const GaussLaunch L) {
  static_assert(TW == kGX || (TW == 96 && !OCT0 && !XF && RMAX <= 16), "96-column tiles: octaves >= 1, unrolled radii");
  constexpr int NI = TW == kGX ? kNR : 3;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[L.o];
  // 1D grid: block -> (scale group, tile).  Blocks are dispatched round-robin
  // over the 8 XCDs; with xcd_band, XCD k runs the k-th contiguous range of
  // tiles (a band of tile rows), so the base rows its vertical passes re-read
  // stay in its own L2.  Groups of one tile are adjacent (same base region).
  // Batch (L.nimg images of one geometry): blocks of image im follow those
  // of image im - 1; its planes, base and seeds are im * (stride) further.
  int lb = blockIdx.x;
  const int bpi = L.gx * L.gy * L.G;  // blocks per image
  if (L.xcd_band) {
    const int nb = bpi * L.nimg, q = nb >> 3, rm = nb & 7, xc = lb & 7;
    lb = xc * q + min(xc, rm) + (lb >> 3);
  }
  const int im = lb / bpi;
  lb -= im * bpi;
  float* const L_gauss = L.gauss ? L.gauss + im * L.gauss_bs : nullptr;
  float* const L_dog = L.dog + im * L.dog_bs;
  double* const L_next_seed = L.next_seed ? L.next_seed + im * L.seed_bs : nullptr;
  const double* const L_base = L.base ? L.base + im * L.base_bs : nullptr;
  double* const L_l64 = L.l64 ? L.l64 + im * L.l64_bs : nullptr;
  const double* const L_vsplit = L.vsplit ? L.vsplit + im * L.vsplit_bs : nullptr;
  const float* const img_b = OCT0 ? P.img + im * P.img_bstride : nullptr;
  const int bz = lb % L.G, bt = lb / L.G;
  const int bx = bt % L.gx, by = bt / L.gx + L.by0;
  GTile T;
  T.bx = bx;
  T.h = oc.h;
  T.w = oc.w;
  T.x0 = bx * (XF ? kFX : TW);
  T.y0 = by * (XF ? kFY : kGY);
  T.lane = threadIdx.x & 63;
  T.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T.cg = T.lane & (kCG - 1);
  T.rs = T.lane / kCG;
  if constexpr (TW == 96) {
#if SIFT_B128MAP
    int g, j;  // conflict-free ds_read_b128 item map
    b128_group(T.lane, g, j);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      T.icg[i] = 8 * i + (j & 7);
      T.irow[i] = 2 * g + (j >> 3);
    }
#else
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = T.lane + 64 * i;
      T.icg[i] = idx % 24;
      T.irow[i] = idx / 24;
    }
#endif
  }
  // item i of the lane: wave row irw(i), first column x0 + 4 icg(i)
  auto irw = [&](int i) { return TW == kGX ? T.rs + kRS * i : T.irow[i]; };
  auto icg = [&](int i) { return TW == kGX ? T.cg : T.icg[i]; };
  T.sw = SWC > 0 ? SWC : L.sw;
  T.hrm = cl2(oc.rmax);
  if (!OCT0)
    T.rsrc = urs(const_cast<double*>(L_base), T.h * T.w * 8);
  // One strip: every wave writes (vertical pass) and reads (horizontal pass)
  // only its own 8 strip rows.
  const int nstrip = kGY * T.sw;
  T.S0 = smem + nstrip;
  double* V = smem;
  // fused extrema: fp32 DoG ring after the strip and the staged region
  float* ring = nullptr;
  if constexpr (XF)
    ring = reinterpret_cast<float*>(smem + nstrip + (OCT0 ? (fl2(kGY - 1 + oc.rmax) + T.hrm + 1) * kBW0 : 0));
  unsigned xlow = 0;

  // The generic horizontal path reads (with zero taps) past the columns a
  // scale writes: those must be finite.
  if (L.zero)
    for (int i = threadIdx.x; i < nstrip; i += 256) smem[i] = 0.0;
  if (OCT0) {
    // Stage input rows y0/2 - hrm .. and columns x0/2 - hrm .. as fp64,
    // clamped (replicate edges): the region every scale's windows read.
    const int q0 = T.y0 / 2 - T.hrm, k0 = T.x0 / 2 - T.hrm;
    const int nr = fl2(kGY - 1 + oc.rmax) + T.hrm + 1;
    const int nc = fl2(kGX - 1 + oc.rmax) + T.hrm + 1;
    double* S0 = smem + nstrip;
    const int kk = clampi(k0 + T.lane, 0, P.W - 1);
    for (int rr = T.wv; rr < nr; rr += 4) {
      const float* src = img_b + (long long)clampi(q0 + rr, 0, P.H - 1) * P.img_stride;
      if (T.lane < nc) S0[rr * kBW0 + T.lane] = (double)src[kk];
    }
  }
  const long long plane = (long long)T.h * T.w;
  // Pixels this block stores: all of its tile, or with fused extrema the
  // kFX x kFY it owns (the last tile of a row / column: all it computes).
  bool own[NI];
  // Per-lane byte offsets of its output items in a plane (past the plane or
  // not owned: the store is dropped).
  int voff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = 8 * T.wv + irw(i);
    const int y = T.y0 + r;
    const int x = T.x0 + 4 * icg(i);
    const bool own_c = !XF || 4 * icg(i) < kFX || bx == L.gx - 1;
    own[i] = y < T.h && T.w - x > 0 && own_c && (!XF || r < kFY || by == L.gy - 1);
    voff[i] = own[i] ? (y * T.w + x) * 4 : 0x7ffffff0;
  }

  // Scale group of this block (small octaves split their scales over
  // blockIdx.z for parallelism; a group recomputes the scale before it as
  // the DoG's L_{s-1}, without storing it).
  const int s_begin = L.gb[bz], s_end = L.gb[bz + 1];
  const int s_first = max(0, s_begin - 1);
  __syncthreads();  // staged region / zeroed strip visible to every wave

  const bool st = !(L.dbg & 1);  // dbg 1: timing without plane stores
  double lprev[NI][4];
  for (int s = s_first; s < s_end; ++s) {
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);
    // Per-lane indices made opaque each scale: otherwise the compiler hoists
    // every radius variant's address arithmetic out of the scale loop and
    // keeps it all live (dozens of VGPRs, half the occupancy).
    GTile Ts = T;
    asm volatile("" : "+v"(Ts.lane), "+v"(Ts.cg), "+v"(Ts.rs));
#if SIFT_TW96_OPQ
    if constexpr (TW == 96) {
#pragma unroll
      for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Ts.icg[i]), "+v"(Ts.irow[i]));
    }
#endif
    if constexpr (TW == 96 && SIFT_TW96_SEQ) {
      // one item at a time: horizontal chains, then its stores, DoG and seed
      vert96_any_(std::make_integer_sequence<int, RMAX + 1>{}, Ts, oc.rad[s], wp, V);
      wave_lds_fence();  // this wave's strip rows written -> read by its other lanes
      const unsigned pb = (unsigned)plane * 4u;
      const bool stor = s >= s_begin && st;
      const __amdgpu_buffer_rsrc_t rg =
          urs(L_gauss ? L_gauss + s * plane : L_dog, pb);
      const __amdgpu_buffer_rsrc_t rd =
          urs(L_dog + (s > 0 ? s - 1 : 0) * plane, pb);
      horz96s_any_(std::make_integer_sequence<int, RMAX + 1>{}, Ts, oc.rad[s], wp, V,
                   [&](int i, const double (&o)[4]) {
                     double d[4];
#pragma unroll
                     for (int q = 0; q < 4; ++q) d[q] = lprev[i][q] - o[q];
                     const int y = T.y0 + 8 * T.wv + irw(i);
                     const int x = T.x0 + 4 * icg(i), nvalid = T.w - x;
                     if (stor) {
                       if (L.vec) {
                         if (L_gauss) bstore4(rg, voff[i], o);
                         if (s > 0) bstore4(rd, voff[i], d);
                       } else if (own[i]) {
                         const long long pp = (long long)y * T.w + x;
                         if (L_gauss) store4(L_gauss + s * plane + pp, o, nvalid);
                         if (s > 0) store4(L_dog + (s - 1) * plane + pp, d, nvalid);
                       }
                     }
                     if (s == P.S && L_next_seed && s >= s_begin && own[i] && !(y & 1)) {
                       double* sd = L_next_seed + (long long)(y >> 1) * L.next_w + (x >> 1);
                       sd[0] = o[0];
                       if (nvalid > 2) sd[1] = o[2];
                     }
#pragma unroll
                     for (int q = 0; q < 4; ++q) lprev[i][q] = o[q];
                   });
      wave_lds_fence();  // strip rows read before the next scale overwrites them
      continue;
    }
    double out[NI][4];
    if constexpr (TW == 96) {
      vert96_any_(std::make_integer_sequence<int, RMAX + 1>{}, Ts, oc.rad[s], wp, V);
      wave_lds_fence();  // this wave's strip rows written -> read by its other lanes
      horz96_any_(std::make_integer_sequence<int, RMAX + 1>{}, Ts, oc.rad[s], wp, V, out);
    } else {
      if constexpr (VS) {
        vert_copy(Ts, oc.rad[s], L_vsplit + (long long)s * plane, V);
      } else if constexpr (!OCT0) {
        if (L_vsplit) vert_copy(Ts, oc.rad[s], L_vsplit + (long long)s * plane, V);
        else vert_any<OCT0, RMAX>(Ts, oc.rad[s], wp, V);
      } else {
        vert_any<OCT0, RMAX>(Ts, oc.rad[s], wp, V);
      }
      wave_lds_fence();  // this wave's strip rows written -> read by its other lanes
      horz_any<OCT0, RMAX>(Ts, oc.rad[s], wp, V, out);
    }
    wave_lds_fence();  // strip rows read before the next scale overwrites them

    double d[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) d[i][q] = lprev[i][q] - out[i][q];
    if (s >= s_begin && (st || out[0][0] == 12345.0)) {
      if (L.vec) {
        const unsigned pb = (unsigned)plane * 4u;
        if (L_gauss) {
          const __amdgpu_buffer_rsrc_t rg = urs(L_gauss + s * plane, pb);
#pragma unroll
          for (int i = 0; i < NI; ++i) bstore4(rg, voff[i], out[i]);
        }
        if (s > 0) {
          const __amdgpu_buffer_rsrc_t rd = urs(L_dog + (s - 1) * plane, pb);
#pragma unroll
          for (int i = 0; i < NI; ++i) bstore4(rd, voff[i], d[i]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int y = T.y0 + 8 * T.wv + irw(i);
          const int x = T.x0 + 4 * icg(i), nvalid = T.w - x;
          if (own[i]) {
            const long long pp = (long long)y * T.w + x;
            if (L_gauss) store4(L_gauss + s * plane + pp, out[i], nvalid);
            if (s > 0) store4(L_dog + (s - 1) * plane + pp, d[i], nvalid);
          }
        }
      }
    }
    if constexpr (XF) {
      // DoG s-1 into ring slot (s-1) % 3, then decide scale s-2 once DoG
      // s-3, s-2, s-1 are all there (scales 1..S; s runs to S+2).
      if (s >= 1) {
        if (s >= 4) lds_barrier();  // the decision of scale s-3 has read slot (s-1) % 3
#pragma unroll
        for (int i = 0; i < kNR; ++i) {
          const float4 f = make_float4((float)d[i][0], (float)d[i][1], (float)d[i][2], (float)d[i][3]);
          *reinterpret_cast<float4*>(ring + ((s - 1) % 3) * kRingPlane + (8 * T.wv + T.rs + kRS * i) * kGX +
                                     4 * T.cg) = f;
        }
        if (s >= 3) {
          lds_barrier();  // every wave's rows of DoG s-1 are in the ring
          if (!(L.dbg & 2)) fused_decide(P, L, Ts, ring, s - 2, xlow);  // dbg 2: timing without the decisions
        }
      }
    }
    if (L_l64 && s >= s_begin) {  // fp64 plane for the exact passes
      double* lp = L_l64 + s * plane;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int y = T.y0 + 8 * T.wv + irw(i);
        const int x = T.x0 + 4 * icg(i), nvalid = T.w - x;
        if (own[i]) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (q < nvalid) lp[(long long)y * T.w + x + q] = out[i][q];
        }
      }
    }
    if (s == P.S && L_next_seed && s >= s_begin) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int y = T.y0 + 8 * T.wv + irw(i);
        const int x = T.x0 + 4 * icg(i), nvalid = T.w - x;
        if (own[i] && !(y & 1)) {
          double* sd = L_next_seed + (long long)(y >> 1) * L.next_w + (x >> 1);
          sd[0] = out[i][0];
          if (nvalid > 2) sd[1] = out[i][2];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) lprev[i][q] = out[i][q];
  }
  if constexpr (XF) {
    if (T.lane == 0 && xlow) atomicAdd(&L.X.counters[1], xlow);
  }
}

// ---------------------------------------------------------------------------
// Register-window tiles for octaves >= 1 (k_gauss_rw).  k_gauss_dog re-reads
// its fp64 base window from L1/L2 once per SCALE (S+3 times) and every wave
// re-reads the 2r rows it shares with the waves above and below: at 4K the
// active blocks of an XCD need ~4 MiB of base lines, its L2 holds 40-60 % of
// those re-reads and the rest stream from the Infinity Cache at ~7 TB/s,
// which bounds the vertical pass (the same loop from an L2-resident plane or
// from LDS issues fp64 fmas 3-4x faster: profiles/r4_fma_probe.txt).  Here
// every lane of a 256-lane block owns ONE strip column and keeps that
// column's window of 8 + 2 RW base rows in registers for ALL scales of the
// octave (RW >= the octave's largest radius): each base value is loaded once
// per block, and the vertical pass of every scale is register fmas only,
//   V[t][c] = sum_k w_k win_c[t + k + RW - r],  t < 8,
// taps in increasing order from 0.0 (k_gauss_dog's chain).  Strip column c
// <-> image column x0 - RW + c, so the 256 columns hold the vertical sums of
// an output tile of TW = 224 (RW <= 16) or 192 (RW <= 32) columns and its
// halo for every radius <= RW: no separate halo pass.  The strip (8 rows,
// double-buffered in LDS) is shared by the block's 4 waves: one barrier per
// scale.  Horizontal pass: items of 8 columns x 1 row (8 fma chains per
// lane); the items of a ds_read_b128 lane group are 4 column groups x 4 rows
// (strip stride 2 mod 4 doubles: conflict-free).  Same fma chain per output
// as k_gauss_dog: bit-identical planes.
// ---------------------------------------------------------------------------
template <int RW>
struct RwGeom {
  static constexpr int NW = 8 + 2 * RW;              // window rows per lane
  static constexpr int TW = RW <= 16 ? 224 : RW <= 24 ? 192 : 160;  // output columns per tile
  static constexpr int NCG = TW / 4;                  // column groups of 4
  static_assert(2 * RW <= 256 - TW, "halo fits the strip");
};
constexpr int kRwRows = 8;    // output rows per tile
constexpr int kRwSW = 264;    // strip row stride (doubles), 0 mod 8
constexpr int kRwStrip = kRwRows * kRwSW + 8;  // doubles per strip buffer
// Strip row t starts at rw_row(t): rows 4..7 one 16-byte quad further, so a
// ds_read_b128 lane group reading 8 column groups of rows t and t + 4 hits
// 16 distinct bank quads.
__host__ __device__ constexpr int rw_row(int t) { return t * kRwSW + 2 * (t >> 2); }
#ifndef SIFT_RWPF
#define SIFT_RWPF 3  // 16-byte strip reads in flight per row, horizontal pass
#endif
#ifndef SIFT_RWTAPS
#define SIFT_RWTAPS 8  // taps per reload of the tap pointer (0: never: the compiler keeps them in SGPRs)
#endif
#ifndef SIFT_RWS_DEFAULT
#define SIFT_RWS_DEFAULT 1  // streamed k_gauss_rw for radii 13..24 (gauss_rws; profiles/r5k_streamed_rw_ab.txt)
#endif
#ifndef SIFT_RW_WPE
#define SIFT_RW_WPE 1  // minimum waves per SIMD the register allocation must allow
#endif

// Vertical pass of one strip column: acc[t] = sum_k w_k win[t + k + RW - R].
// Tap loads: the tap pointer is made opaque every 8 taps, so the compiler
// loads each group of taps where it is used instead of keeping 2r + 1 taps
// in SGPRs.
template <int R, int RW>
__device__ __forceinline__ void rw_vert(const double (&win)[RwGeom<RW>::NW], const cdouble* wp, double (&acc)[8]) {
  constexpr int D = RW - R;
  const cdouble* wq = wp;
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = 0.0;
#pragma unroll
  for (int k = 0; k <= 2 * R; ++k) {
    if (SIFT_RWTAPS > 0 && k % (SIFT_RWTAPS > 0 ? SIFT_RWTAPS : 1) == 0) asm volatile("" : "+s"(wq));
    const double wk = wq[k];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = fma(wk, win[t + k + D], acc[t]);
  }
}

// Horizontal pass of one item (4 columns x rows A, B): out[i][q] = sum_k w_k
// V[row_i][b + q + k], b = 4 cg + RW - R (strip column of the first tap of
// output column x0 + 4 cg); 16-byte reads from the even column at or before b.
template <int R, int RW>
__device__ __forceinline__ void rw_horz(const double* ra, const double* rb, const cdouble* wp, double (&out)[2][4]) {
  constexpr int D = (RW - R) & 1;           // b odd: element n is pair (n + 1) / 2, half (n + 1) & 1
  constexpr int NE = 4 + 2 * R;             // elements n = 0 .. 3 + 2R
  constexpr int NP = (NE - 1 + D) / 2 + 1;  // pairs per row
  constexpr int PF = NP < SIFT_RWPF ? NP : SIFT_RWPF;
  const double* pa = ra + ((RW - R) - D);   // even column
  const double* pb = rb + ((RW - R) - D);
  double2 u[2][NP];
  const cdouble* wq = wp;
#pragma unroll
  for (int q = 0; q < 4; ++q) out[0][q] = out[1][q] = 0.0;
  // An odd-D item does not use its first pair's .x: that value is marked used
  // (empty asm), so every read stays one aligned ds_read_b128 (the compiler
  // would otherwise drop it and re-pair the reads as 8-byte-aligned
  // ds_read2_b64s, which conflict).
  auto rd = [](const double* q) { return *reinterpret_cast<const double2*>(q); };
#pragma unroll
  for (int n2 = 0; n2 < PF; ++n2) {
    u[0][n2] = rd(pa + 2 * n2);
    u[1][n2] = rd(pb + 2 * n2);
  }
  if constexpr (D) asm volatile("" ::"v"(u[0][0].x), "v"(u[1][0].x));
#pragma unroll
  for (int n2 = 0; n2 < NP; ++n2) {
    if (n2 + PF < NP) {
      u[0][n2 + PF] = rd(pa + 2 * (n2 + PF));
      u[1][n2 + PF] = rd(pb + 2 * (n2 + PF));
    }
    if (SIFT_RWTAPS > 0 && n2 % (SIFT_RWTAPS > 0 ? SIFT_RWTAPS / 2 : 1) == 0) asm volatile("" : "+s"(wq));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * n2 + e - D;  // element index
      if (n < 0 || n >= NE) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = n - q;
        if (k >= 0 && k <= 2 * R) {
          const double wk = wq[k];
          out[0][q] = fma(wk, e ? u[0][n2].y : u[0][n2].x, out[0][q]);
          out[1][q] = fma(wk, e ? u[1][n2].y : u[1][n2].x, out[1][q]);
        }
      }
    }
    pin(out[0]);
    pin(out[1]);
  }
}

template <int RW, int... Rs>
__device__ __forceinline__ void rw_vert_any_(std::integer_sequence<int, Rs...>, int r,
                                            const double (&win)[RwGeom<RW>::NW], const cdouble* wp,
                                            double (&acc)[8]) {
  rdispatch<0, sizeof...(Rs) - 1>(r, [&](auto R) { rw_vert<decltype(R)::value, RW>(win, wp, acc); });
}
// BIN: binary dispatch (the register-window kernel); the streamed kernels keep
// the compare chain (the binary form cost k_gauss_rw<24, true> 82 -> 100 VGPRs).
template <int RW, bool BIN = true, int... Rs>
__device__ __forceinline__ void rw_horz_any_(std::integer_sequence<int, Rs...>, int r, const double* ra,
                                            const double* rb, const cdouble* wp, double (&out)[2][4]) {
  if constexpr (BIN) {
    rdispatch<0, sizeof...(Rs) - 1>(r, [&](auto R) { rw_horz<decltype(R)::value, RW>(ra, rb, wp, out); });
  } else {
    bool done = false;
    ((!done && r == Rs ? (rw_horz<Rs, RW>(ra, rb, wp, out), done = true) : false), ...);
  }
}
// Streamed vertical pass of one strip column (k_gauss_rw<RW, true>): the
// scale's own window rows y0 - r .. y0 + 7 + r loaded per scale from the base
// plane (L2-resident for the mid-radius octaves: XCD-banded tiles), in
// vert_glob_gen's 8-row chunks over zero-padded taps -- the same fma chain per
// output as the register window, bit for bit.
__device__ __forceinline__ void rw_vert_stream(__amdgpu_buffer_rsrc_t rs, int xoff, int y0, int h, int w, int r,
                                               const cdouble* wp, double (&acc)[8]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = 0.0;
  const int yb = y0 - r, NJ = 2 * r + 8;
  auto chunk = [&](int jb, auto C, auto first) {
    using CC = decltype(C);
    double v[8];
#pragma unroll
    for (int k = 0; k < CC::kRows; ++k)
      v[k] = load_f64(rs, xoff, __builtin_amdgcn_readfirstlane(clampi(yb + jb + k, 0, h - 1) * w * 8));
    const cdouble* wq = wp + jb;
    CC::template run<decltype(first)::value>([&](int k, int t) { acc[t] = fma((double)wq[k - t], v[k], acc[t]); });
    pin(acc);
  };
  vchunk_dispatch<true>(2 * r, [&](auto C, auto f) { chunk(0, C, f); });
  for (int jb = 8; jb < NJ; jb += 8) vchunk_dispatch<false>(2 * r - jb, [&](auto C, auto f) { chunk(jb, C, f); });
}

template <int RW, bool STREAM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_RW_WPE))) void k_gauss_rw(const Pyramid P, const GaussLaunch L) {
  using G = RwGeom<RW>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[L.o];
  // 1D grid: block -> (scale group, tile) as in k_gauss_dog (XCD bands, batches image-major).
  int lb = blockIdx.x;
  const int bpi = L.gx * L.gy * L.G;
  if (L.xcd_band) {
    const int nb = bpi * L.nimg, q = nb >> 3, rm = nb & 7, xc = lb & 7;
    lb = xc * q + min(xc, rm) + (lb >> 3);
  }
  const int im = lb / bpi;
  lb -= im * bpi;
  float* const L_gauss = L.gauss ? L.gauss + im * L.gauss_bs : nullptr;
  float* const L_dog = L.dog + im * L.dog_bs;
  double* const L_next_seed = L.next_seed ? L.next_seed + im * L.seed_bs : nullptr;
  const double* const L_base = L.base + im * L.base_bs;
  const int bz = lb % L.G, bt = lb / L.G;
  const int bx = bt % L.gx, by = bt / L.gx + L.by0;
  const int h = oc.h, w = oc.w;
  const int x0 = bx * G::TW, y0 = by * kRwRows;
  const int c = threadIdx.x;  // strip column
  // The lane's base window: rows y0 - RW .. y0 + 7 + RW of image column x0 - RW + c (clamped).
  const __amdgpu_buffer_rsrc_t brs =
      urs(const_cast<double*>(L_base), h * w * 8);
  const int bxoff = clampi(x0 - RW + c, 0, w - 1) * 8;
  double win[STREAM ? 1 : G::NW];
  if constexpr (!STREAM) {
#pragma unroll
    for (int j = 0; j < G::NW; ++j)
      win[j] = load_f64(brs, bxoff, __builtin_amdgcn_readfirstlane(clampi(y0 - RW + j, 0, h - 1) * w * 8));
  }
  // Horizontal items of 4 columns x 2 rows: ds_read_b128 lane group gid =
  // 4 wv + g (b128_group) at position j: column group cg = 8 (gid >> 1) +
  // (j & 7), rows a = gid & 1 or 2 + (gid & 1) and a + 4, the half-groups in
  // opposite order (j < 8: a = gid & 1 first; j >= 8: a + 4 first), so every
  // read instruction covers two rows 6 or 2 apart (odd quad offsets through
  // rw_row: conflict-free) and every store instruction 128 contiguous bytes
  // of a row per half-group.
  int hcg, hr0, hr1;
  {
    int g, j;
    b128_group(c & 63, g, j);
    const int gid = 4 * (c >> 6) + g;
    hcg = 8 * (gid >> 1) + (j & 7);
    hr0 = j < 8 ? (gid & 1) : 6 + (gid & 1);
    hr1 = j < 8 ? 4 + (gid & 1) : 2 + (gid & 1);
  }
  const bool hact = hcg < G::NCG;  // lanes with an item
  const long long plane = (long long)h * w;
  const int s_begin = L.gb[bz], s_end = L.gb[bz + 1];
  const int s_first = max(0, s_begin - 1);
  const bool st = !(L.dbg & 1);  // dbg 1: timing without plane stores
  double lprev[2][4];
  for (int s = s_first; s < s_end; ++s) {
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);
    const int r = oc.rad[s];
    double* Vs = smem + (s & 1) * kRwStrip;
    {
      double acc[8];
      if constexpr (STREAM) {
        int xo = bxoff;
        asm volatile("" : "+v"(xo));  // per-scale opaque: no hoisted per-radius addresses
        rw_vert_stream(brs, xo, y0, h, w, r, wp, acc);
      } else {
        rw_vert_any_<RW>(std::make_integer_sequence<int, RW + 1>{}, r, win, wp, acc);
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) Vs[rw_row(t) + c] = acc[t];
    }
    // Strip s complete; every wave is past its horizontal pass of scale s - 1
    // (the other buffer), so the next scale may overwrite that one.
    lds_barrier();
    if (hact) {
      int hc = hcg, h0 = hr0, h1 = hr1;
      asm volatile("" : "+v"(hc), "+v"(h0), "+v"(h1));  // per-scale opaque: no hoisted per-radius addresses
      double o[2][4];
      rw_horz_any_<RW, !STREAM || SIFT_BIN_STREAM>(std::make_integer_sequence<int, RW + 1>{}, r, Vs + rw_row(h0) + 4 * hc,
                                Vs + rw_row(h1) + 4 * hc, wp, o);
      const int x = x0 + 4 * hc, nvalid = w - x;
      const unsigned pb = (unsigned)plane * 4u;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int y = y0 + (i ? h1 : h0);
        const bool own = y < h && nvalid > 0;
        double d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = lprev[i][q] - o[i][q];
        if (s >= s_begin && st) {
          if (L.vec) {
            const int voff = own ? (y * w + x) * 4 : 0x7ffffff0;  // dropped past the plane
            if (L_gauss)
              bstore4(urs(L_gauss + s * plane, pb), voff, o[i]);
            if (s > 0)
              bstore4(urs(L_dog + (s - 1) * plane, pb), voff, d);
          } else if (own) {
            const long long pp = (long long)y * w + x;
            if (L_gauss) store4(L_gauss + s * plane + pp, o[i], nvalid);
            if (s > 0) store4(L_dog + (s - 1) * plane + pp, d, nvalid);
          }
        }
        if (s == P.S && L_next_seed && s >= s_begin && own && !(y & 1)) {
          double* sd = L_next_seed + (long long)(y >> 1) * L.next_w + (x >> 1);
          sd[0] = o[i][0];
          if (nvalid > 2) sd[1] = o[i][2];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) lprev[i][q] = o[i][q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pipelined streamed tiles (k_gauss_rwp, round 6).  The streamed
// k_gauss_rw<RW, true> waits for every 8-row chunk of a scale's vertical
// window before its fmas: at 4K octave 2 a wave spends half its life in
// s_waitcnt (r6a stall counters: wait 13.4 K of 26.4 K quad-cycles, 260
// buffer loads in ~35 dependent rounds, 3.1 K SALU).  Here the chunks are
// double-buffered in registers: chunk j + 1's 8 loads are issued before chunk
// j's 64 fmas, and the last chunk of a scale issues the NEXT scale's first
// chunk, which lands during the barrier, the horizontal pass and the stores.
// For the compiler's waitcnt pass to count the loads exactly, every scale
// issues the same buffer stores (a lane with nothing to store -- no item,
// past the plane, a recomputed scale -- has its store dropped by the
// descriptor's range check) and every chunk loads 8 rows (clamped; taps past
// 2r are zero padding, fma(0, v, acc) == acc).  The fma chain of every output
// is k_gauss_rw's (taps in increasing order from 0.0): bit-identical planes.
// Interior chunks (no row clamping) take one SALU add per row.
// Measured (r6b / r6c, experiments build, SIFT_RWP / SIFT_RWP_BIG): GPU suite
// green with both on, but not faster -- 4K octave 2 0.091 -> 0.093-0.094 ms,
// octave 3 (split pass + tile kernel 0.057 ms) -> 0.069-0.072 ms as one
// k_gauss_rwp<48> launch.  The wave's s_waitcnt time fell (13.4 K -> 8.4 K
// quad-cycles) and its issue stalls rose by as much (4.4 K -> 9.6 K): the
// loads were not what bounded it (profiles/r6b_pipelined_streamed_ab.txt).
// Off by default.
// ---------------------------------------------------------------------------
// (Row offsets on two paths, the loads after the join: the waitcnt pass
// merges paths pessimistically, so loads issued on different paths would
// make it wait for them one by one.)
__device__ __forceinline__ void rwp_load(__amdgpu_buffer_rsrc_t rs, int xoff, int rb, int h, int w8, double (&v)[8]) {
  int so[8];
  if (rb >= 0 && rb + 7 <= h - 1) {
    so[0] = rb * w8;
#pragma unroll
    for (int k = 1; k < 8; ++k) so[k] = so[k - 1] + w8;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) so[k] = clampi(rb + k, 0, h - 1) * w8;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) asm volatile("" : "+s"(so[k]));
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = load_f64(rs, xoff, so[k]);
}

// acc[t] += w[8j + k - t] v[k] over the chunk's rows k (wq = taps + 8j, zero padded).
template <bool FIRST>
__device__ __forceinline__ void rwp_fma(const cdouble* wq, const double (&v)[8], double (&acc)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (!(FIRST && k < t)) acc[t] = fma((double)wq[k - t], v[k], acc[t]);
  pin(acc);
}

__device__ __forceinline__ void bstore_f64x2(__amdgpu_buffer_rsrc_t rs, int voff, double a, double b) {
  const double2 d = make_double2(a, b);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d), rs, voff, 0, 0);
}

// Horizontal pass of one item for radii beyond the unrolled ones (r > 24):
// element m of the row is strip column b - D + m (b = RW - r + 4 cg, D = b & 1,
// so the 16-byte reads are aligned), tap of output q = m - D - q; 8 elements
// per step over zero-padded taps -- the same chain per output as rw_horz.
// The strip columns past 255 that the last items' steps read are zero
// (k_gauss_rwp clears them).
template <int RW>
__device__ __forceinline__ void rwp_horz_gen(const double* ra, const double* rb, int r, const cdouble* wp,
                                             double (&out)[2][4]) {
  const int D = (RW - r) & 1;
  const double* pa = ra + (RW - r) - D;
  const double* pb = rb + (RW - r) - D;
  const cdouble* wq = wp - D;
  const int nstep = (2 * r + 4 + D + 7) >> 3;
#pragma unroll
  for (int q = 0; q < 4; ++q) out[0][q] = out[1][q] = 0.0;
  for (int st = 0; st < nstep; ++st) {
    double2 u[2][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      u[0][e] = *reinterpret_cast<const double2*>(pa + 8 * st + 2 * e);
      u[1][e] = *reinterpret_cast<const double2*>(pb + 8 * st + 2 * e);
    }
    const cdouble* w8 = wq + 8 * st;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double wk = w8[m - q];
        out[0][q] = fma(wk, (m & 1) ? u[0][m >> 1].y : u[0][m >> 1].x, out[0][q]);
        out[1][q] = fma(wk, (m & 1) ? u[1][m >> 1].y : u[1][m >> 1].x, out[1][q]);
      }
    pin(out[0]);
    pin(out[1]);
  }
}

// L64: also store the fp64 Gaussian planes (the exact passes' patches of
// octaves whose radii exceed the unrolled ones read them: sift_exact.h).
template <int RW, bool L64>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_RW_WPE))) void k_gauss_rwp(const Pyramid P, const GaussLaunch L) {
  using G = RwGeom<RW>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[L.o];
  int lb = blockIdx.x;
  const int bpi = L.gx * L.gy * L.G;
  if (L.xcd_band) {
    const int nb = bpi * L.nimg, q = nb >> 3, rm = nb & 7, xc = lb & 7;
    lb = xc * q + min(xc, rm) + (lb >> 3);
  }
  const int im = lb / bpi;
  lb -= im * bpi;
  float* const L_gauss = L.gauss ? L.gauss + im * L.gauss_bs : nullptr;
  float* const L_dog = L.dog + im * L.dog_bs;
  double* const L_next_seed = L.next_seed ? L.next_seed + im * L.seed_bs : nullptr;
  double* const L_l64 = L64 ? L.l64 + im * L.l64_bs : nullptr;
  const double* const L_base = L.base + im * L.base_bs;
  const int bz = lb % L.G, bt = lb / L.G;
  const int bx = bt % L.gx, by = bt / L.gx + L.by0;
  const int h = oc.h, w = oc.w, w8 = w * 8;
  const int x0 = bx * G::TW, y0 = by * kRwRows;
  const int c = threadIdx.x;  // strip column
  const __amdgpu_buffer_rsrc_t brs =
      urs(const_cast<double*>(L_base), h * w * 8);
  const int bxoff = clampi(x0 - RW + c, 0, w - 1) * 8;
  if constexpr (RW > 24) {  // zero the strip columns past 255 (read by rwp_horz_gen's last steps)
    constexpr int GAP = 14;  // doubles from a row's column 256 to the next row (<= 14)
    const int b = c / (8 * GAP), t = (c / GAP) & 7, j = c % GAP;
    const int a = rw_row(t) + 256 + j, end = t < 7 ? rw_row(t + 1) : kRwStrip;
    if (b < 2 && a < end) smem[b * kRwStrip + a] = 0.0;
  }
  // Horizontal items as in k_gauss_rw; lanes without an item read item NCG - 1 and store nothing.
  int hcg, hr0, hr1;
  {
    int g, j;
    b128_group(c & 63, g, j);
    const int gid = 4 * (c >> 6) + g;
    hcg = 8 * (gid >> 1) + (j & 7);
    hr0 = j < 8 ? (gid & 1) : 6 + (gid & 1);
    hr1 = j < 8 ? 4 + (gid & 1) : 2 + (gid & 1);
  }
  const bool hact = hcg < G::NCG;
  if (!hact) hcg = G::NCG - 1;
  const long long plane = (long long)h * w;
  const unsigned pb = (unsigned)plane * 4u;
  const unsigned sbytes = L_next_seed ? (unsigned)((h + 1) / 2) * (unsigned)L.next_w * 8u : 0u;
  int voff[2], soff[2], loff[2];
  {
    const int x = x0 + 4 * hcg;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int y = y0 + (i ? hr1 : hr0);
      const bool own = hact && y < h && x < w;
      voff[i] = own ? (y * w + x) * 4 : 0x7ffffff0;
      loff[i] = own ? (y * w + x) * 8 : 0x7fffffe0;
      soff[i] = own && !(y & 1) ? ((y >> 1) * L.next_w + (x >> 1)) * 8 : 0x7ffffff0;
    }
  }
  const int s_begin = L.gb[bz], s_end = L.gb[bz + 1];
  const int s_first = max(0, s_begin - 1);
  const bool st = !(L.dbg & 1);  // dbg 1: timing without plane stores
  double lprev[2][4];
  double va[8], vb[8];
  constexpr int NCH = (2 * RW + 15) >> 3;  // chunks of the widest window
  rwp_load(brs, bxoff, y0 - oc.rad[s_first], h, w8, va);
  {
    // Six empty stores (a zero-size descriptor the compiler cannot see is
    // empty) after the first chunk's loads: the loop is entered with the
    // same vector-memory queue as every scale leaves it (next chunk, then
    // the scale's six stores), so the waitcnt pass's merge at the loop head
    // waits only for the loads (vmcnt(6)), not for everything.
    const __amdgpu_buffer_rsrc_t rz =
        urs(L_dog, (unsigned)L.dbg & 0x40000000u);
    const double zz[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 4; ++i) bstore4(rz, 16 * i, zz);
#pragma unroll
    for (int i = 0; i < (L64 ? 6 : 2); ++i) bstore_f64x2(rz, 64 + 16 * i, 0.0, 0.0);
  }
  bool nb = false;  // this scale's first chunk is in vb
  for (int s = s_first; s < s_end; ++s) {
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);
    const int r = oc.rad[s];
    const int nch = (2 * r + 15) >> 3;  // ceil((2r + 8) / 8)
    const int rnext = y0 - oc.rad[min(s + 1, s_end - 1)];  // (the last scale's is never used)
    const int rb = y0 - r;
#pragma unroll
    for (int k = 0; k < 8; ++k) va[k] = nb ? vb[k] : va[k];
    double acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = 0.0;
    // Chunk positions unrolled (uniform guards): chunk j is in va for even j,
    // vb for odd j; position j issues chunk j + 1 (or the next scale's first
    // chunk) into the other buffer before its fmas.
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      if (j < nch) {
        const int rl = j + 1 < nch ? rb + 8 * (j + 1) : rnext;
        if (j & 1) {
          rwp_load(brs, bxoff, rl, h, w8, va);
          rwp_fma<false>(wp + 8 * j, vb, acc);
        } else {
          rwp_load(brs, bxoff, rl, h, w8, vb);
          if (j == 0) rwp_fma<true>(wp, va, acc);
          else rwp_fma<false>(wp + 8 * j, va, acc);
        }
      }
    }
    nb = nch & 1;
    double* Vs = smem + (s & 1) * kRwStrip;
#pragma unroll
    for (int t = 0; t < 8; ++t) Vs[rw_row(t) + c] = acc[t];
    lds_barrier();
    int hc = hcg, h0 = hr0, h1 = hr1;
    asm volatile("" : "+v"(hc), "+v"(h0), "+v"(h1));  // per-scale opaque: no hoisted per-radius addresses
    double o[2][4];
    constexpr int RU = RW < 24 ? RW : 24;  // unrolled radii
    if (RW <= 24 || r <= RU)
      rw_horz_any_<RW, false>(std::make_integer_sequence<int, RU + 1>{}, r, Vs + rw_row(h0) + 4 * hc,
                              Vs + rw_row(h1) + 4 * hc, wp, o);
    else
      rwp_horz_gen<RW>(Vs + rw_row(h0) + 4 * hc, Vs + rw_row(h1) + 4 * hc, r, wp, o);
    const bool sto = s >= s_begin && st;
    const __amdgpu_buffer_rsrc_t rg = urs(L_gauss ? L_gauss + s * plane : L_dog, sto && L_gauss ? pb : 0u);
    const __amdgpu_buffer_rsrc_t rd = urs(L_dog + (s > 0 ? s - 1 : 0) * plane, sto && s > 0 ? pb : 0u);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      double d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = lprev[i][q] - o[i][q];
      bstore4(rg, voff[i], o[i]);
      bstore4(rd, voff[i], d);
    }
    {  // the next octave's base: L_S at even rows and columns (dropped at every other scale)
      const __amdgpu_buffer_rsrc_t rsd =
          urs(L_next_seed ? (void*)L_next_seed : (void*)L_dog, s == P.S && s >= s_begin ? sbytes : 0u);
#pragma unroll
      for (int i = 0; i < 2; ++i) bstore_f64x2(rsd, soff[i], o[i][0], o[i][2]);
    }
    if constexpr (L64) {  // fp64 plane s for the exact passes
      const __amdgpu_buffer_rsrc_t rl =
          urs(L_l64 + s * plane, sto ? (unsigned)plane * 8u : 0u);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        bstore_f64x2(rl, loff[i], o[i][0], o[i][1]);
        bstore_f64x2(rl, loff[i] + 16, o[i][2], o[i][3]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) lprev[i][q] = o[i][q];
  }
}

// Octaves >= 1 through k_gauss_rw: radii up to SIFT_RW_R (the register
// window of 8 + 2 RW rows per lane; default 12: octave 1 at 4K and 1080p,
// 0.172 -> 0.158 ms at 4K; RW 24 for octave 2 measured slower, 0.097 ->
// 0.100 ms: profiles/r4r_register_window_ab.txt), planes of at least 2
// columns (SIFT_RW=0: k_gauss_dog, A/B builds).
static int rw_width(const Pyramid& P, int o) {
  const int R = P.oct[o].rmax;
  return R <= 12 ? 12 : R <= 16 ? 16 : R <= 24 ? 24 : R <= 48 ? 48 : 0;
}

// The pipelined streamed kernel (k_gauss_rwp) issues the same 16-byte buffer
// stores at every scale, so it needs every plane it writes 16-byte aligned:
// octave width a multiple of 4, plane offsets (and a batch's per-image
// strides) multiples of 16 bytes, the next octave's base likewise.
static bool rwp_ok(const Pyramid& P, int o) {
  static const int on = exp_knob("SIFT_RWP", 0);
  const Octave& oc = P.oct[o];
  if (!on || o < 1 || (oc.w & 3) || 8.0 * oc.h * oc.w >= 2147483648.0) return false;
  if ((oc.dog_off & 3) || (oc.gauss_off & 3)) return false;
  if (o + 1 < P.O && (P.oct[o + 1].seed_off & 1)) return false;
  if (P.nimg > 1) {
    const long long tot = P.ND > 0 ? P.dog_bstride / P.ND : 0;
    if ((P.dog_bstride & 3) || ((tot * P.NS) & 3) || (P.seed_bstride & 1)) return false;
  }
  return true;
}

// Octaves whose radii exceed the unrolled ones (25..48: 4K / 1080p octave 3,
// 8K octave 3) run k_gauss_rwp<48> -- one launch, 160-column tiles, the
// split pass's scratch round trip gone -- and keep their fp64 planes for the
// exact passes (the split pass's vertical sums served them before).
static bool rwp_big(const Pyramid& P, int o) {
  static const int on = exp_knob("SIFT_RWP_BIG", 0);
  const int r = P.oct[o].rmax;
  return on && r > 24 && r <= 48 && P.oct[o].w >= 2 && rwp_ok(P, o);
}

// Octaves >= 1 whose radii exceed the register window (SIFT_RW_R) up to 24
// run k_gauss_rw with the streamed vertical pass (rw_vert_stream): 208-column
// tiles in a 256-column strip instead of k_gauss_dog's 64-column tiles with
// (64 + 2r) / 64 of the vertical work (SIFT_RWS=0: k_gauss_dog, A/B builds).
// SIFT_RWS bit 0: radii 13..24; bit 1: also the register-window octaves
// (radii <= 12) streamed.  Radii 25..48: rwp_big.
static bool gauss_rws(const Pyramid& P, int o) {
  static const int on = exp_knob("SIFT_RWS", SIFT_RWS_DEFAULT);
  static const int rlim = exp_knob("SIFT_RW_R", 12);
  const int r = P.oct[o].rmax;
  if (o >= 1 && r > 24) return rwp_big(P, o);
  if (!on || o < 1 || P.oct[o].w < 2 || gauss_keep_l64(P, o)) return false;
  return r > std::min(rlim, 24) ? (on & 1) != 0 : (on & 2) != 0;
}

bool gauss_wide(const Pyramid& P, int o) {
  static const int on = exp_knob("SIFT_RW", 1);
  static const int rlim = exp_knob("SIFT_RW_R", 12);
  return (on && o >= 1 && P.oct[o].w >= 2 && P.oct[o].rmax <= std::min(rlim, 24) && rw_width(P, o) > 0 &&
          !gauss_keep_l64(P, o)) ||
         gauss_rws(P, o);
}

// k_gauss_rwp for a streamed octave (its launch: the pointers as well).
static bool gauss_rwp(const Pyramid& P, const GaussLaunch& L) {
  const bool seed_ok = !L.next_seed || ((L.next_w & 1) == 0 && !(reinterpret_cast<uintptr_t>(L.next_seed) & 15));
  const bool l64_ok = !L.l64 || !(reinterpret_cast<uintptr_t>(L.l64) & 15);
  return rwp_ok(P, L.o) && L.vec && seed_ok && l64_ok;
}

static int rw_tile_w(const Pyramid& P, int o) {
  const int RW = rw_width(P, o);
  return RW <= 16 ? 224 : RW <= 24 ? 192 : 160;
}
static size_t rw_lds(const Pyramid& P, int o) { (void)P; (void)o; return sizeof(double) * 2 * kRwStrip; }

// Materialised octave-0 base (fp64), for octave-0 radii beyond kUR.
__global__ __launch_bounds__(256) void k_upsample_base(const Pyramid P, double* __restrict__ b) {
  const int h = P.oct[0].h, w = P.oct[0].w;
  const long long n = (long long)h * w;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    b[i] = (double)P.img[(long long)min(y >> 1, P.H - 1) * P.img_stride + min(x >> 1, P.W - 1)];
  }
}

// DoG from a caller-supplied fp32 Gaussian pyramid (foreign scale space):
// D[t] = L[t] - L[t+1] in fp64 (exact for fp32 operands), rounded once.
__global__ __launch_bounds__(256) void k_dog_from_gauss(const float* __restrict__ g,
                                                        float* __restrict__ d, long long plane,
                                                        int nd) {
  const long long n = plane * nd;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    d[i] = (float)((double)g[i] - (double)g[i + plane]);
  }
}

bool gauss_needs_base0(const Pyramid& P) { return P.oct[0].rmax > kUR; }

// Octaves o >= 1 whose largest radius reaches SIFT_L64_R (default 90; 0 =
// never) also store their fp64 Gaussian planes: the exact passes read them
// instead of recomputing 3x3x3 patches with 189- and 377-tap chains (8K O=6
// S=5: octaves 4 and 5; at 4K octave 3, radius 47, it measured slower: 0.71 -> 0.74 ms pass).
bool gauss_keep_l64(const Pyramid& P, int o) {
  static const int rmin = exp_knob("SIFT_L64_R", 90);
  return o >= 1 && ((rmin > 0 && P.oct[o].rmax >= rmin) || rwp_big(P, o));
}

// Octaves o >= 1 whose largest radius reaches SIFT_VSPLIT_R (default 40; 0 =
// never) run the split vertical pass (k_gauss_vert) before the tile kernel.
bool gauss_vsplit(const Pyramid& P, int o) {
  static const int rmin = exp_knob("SIFT_VSPLIT_R", 40);
  return o >= 1 && rmin > 0 && P.oct[o].rmax >= rmin && !gauss_wide(P, o);
}

static bool staged0(const Pyramid& P, int o) { return o == 0 && !gauss_needs_base0(P); }

// 96-column tiles (horz_full96) for octaves >= 1 whose radii all have
// unrolled code and no split pass (SIFT_TW96=0: always 64, experiments).
static int tile_w(const Pyramid& P, int o) {
  static const int tw96 = exp_knob("SIFT_TW96", 1);
  const Octave& oc = P.oct[o];
  return (tw96 && o >= 1 && kVert2 && oc.rmax <= kUR96 && oc.w >= 2 && !gauss_vsplit(P, o)) ? 96 : kGX;
}

constexpr int kSW0 = 2 * (kCG - 1) + 8 + 6;   // octave-0 strip stride for rmax <= 8
constexpr int kSW1 = 2 * (kCG - 1) + kUR + 6;  // ... rmax <= kUR

// Strip row stride (doubles).  Octaves >= 1: covers the widest read of the
// horizontal pass (generic path: 4 (kCG - 1) + round_up(2r + 4, 8)), and is
// 2 mod 4 so that the two rows a ds_read_b128 phase reads fall in disjoint
// bank halves.
static int strip_stride(const Pyramid& P, int o) {
  const int R = P.oct[o].rmax;
  if (staged0(P, o)) return R <= 8 ? kSW0 : kSW1;
  const int tw = tile_w(P, o);
  int sw = R <= kUR1 ? tw + 2 * R + 4 : tw + 2 * R + 12;
  if (sw % 4 == 0) sw += 2;
  return sw;
}

static size_t staged_bytes(const Pyramid& P, int o) {
  if (!staged0(P, o)) return 0;
  const int R = P.oct[0].rmax;
  return sizeof(double) * (size_t)(fl2(kGY - 1 + R) + cl2(R) + 1) * kBW0;
}

size_t gauss_lds_bytes(const Pyramid& P, int o, bool fused) {
  if (!fused && gauss_wide(P, o)) return rw_lds(P, o);
  return sizeof(double) * kGY * strip_stride(P, o) + staged_bytes(P, o) +
         (fused ? sizeof(float) * 3 * kRingPlane : 0);
}

bool gauss_can_fuse(const Pyramid& P, int o) {
  const Octave& oc = P.oct[o];
  // staged0 implies octave 0, which never splits its scales (scale_groups)
  return staged0(P, o) && oc.h >= 3 && oc.w >= 3 && P.S >= 1 &&
         gauss_lds_bytes(P, o, true) <= 160 * 1024;
}

// Cost of one scale of a tile, in units of one fp64 tap per output of both
// passes; the constant covers the strip round trip and the plane stores.
static int scale_cost(const Octave& oc, int s) { return 2 * oc.rad[s] + 1 + 8; }

// Split the NS scales of octave o into G contiguous groups (blockIdx.z) so
// that the most expensive group -- which also recomputes the scale before it
// as the DoG's L[s-1] -- is as cheap as possible (radii grow with s, so equal
// scale counts would leave the last group with most of the work).  Returns
// the max group cost; gb[0..G] are the group boundaries.
static int split_scales(const Pyramid& P, int o, int G, int* gb) {
  const Octave& oc = P.oct[o];
  const int NS = P.NS;
  // best[g][e]: min over splits of scales [0, e) into g groups of the max group cost
  int best[kMaxScales + 1][kMaxScales + 1], cut[kMaxScales + 1][kMaxScales + 1];
  auto cost = [&](int b, int e) {
    int c = 0;
    for (int s = std::max(0, b - 1); s < e; ++s) c += scale_cost(oc, s);
    return c;
  };
  for (int e = 0; e <= NS; ++e) best[1][e] = cost(0, e), cut[1][e] = 0;
  for (int g = 2; g <= G; ++g)
    for (int e = g; e <= NS; ++e) {
      best[g][e] = 1 << 30;
      for (int b = g - 1; b < e; ++b) {
        const int c = std::max(best[g - 1][b], cost(b, e));
        if (c < best[g][e]) best[g][e] = c, cut[g][e] = b;
      }
    }
  gb[G] = NS;
  for (int g = G, e = NS; g >= 1; --g) {
    gb[g - 1] = g > 1 ? cut[g][e] : 0;
    e = gb[g - 1];
  }
  return best[G][NS];
}

// Scale groups per octave: small octaves split their scales so that enough
// blocks fill the 256 CUs (octave 0 never splits: it is HBM-write bound and
// every split recomputes a scale).  SIFT_GAUSS_GROUPS="g1,g2,..."
// overrides the group count of octaves 1, 2, ... (experiments).
static int scale_groups(const Pyramid& P, int o) {
  static const std::vector<int> env = [] {
    std::vector<int> v;
#ifdef SIFT_EXPERIMENTS
    if (const char* e = std::getenv("SIFT_GAUSS_GROUPS"))
      for (const char* p = e; *p;) {
        v.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p) ++p;
      }
#endif
    return v;
  }();
  if (o == 0) return 1;
  if (o - 1 < (int)env.size() && env[o - 1] > 0) return std::min(env[o - 1], P.NS);
  // Measured (4K, O=4, S=5; tools/experiments/gpu_groups.sh): every split adds the
  // recomputed scale to the total work, so an octave splits only until it
  // has ~1.5 blocks per CU -- 60x68 tiles: 1 group; 30x34: 1 (G=2: 116 us,
  // G=4: 126-140 us, G=1: 103 us); 15x17: 2 (70.8 us; G=1 94 us, G=4 85 us).
  const Octave& oc = P.oct[o];
  const int tw = tile_w(P, o);
  const long long tiles = (long long)((oc.w + tw - 1) / tw) * ((oc.h + kGY - 1) / kGY);
  // (Split-pass octaves measured the same: 2048 instead of 400 blocks made
  // 4K octave 3 0.054 -> 0.073 ms.)
  int g = 1;
  while (g < P.NS && tiles * g < 400) ++g;
  return g;
}

template <bool O0, int SWC, int RMAX, bool XF>
static void set_attr() {
  (void)hipFuncSetAttribute((const void*)k_gauss_dog<O0, SWC, RMAX, XF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
}

// The base of octave o+1 alone (sift_detect_from_seed_range_device: an
// octave below the scanned one only feeds its successor).  background.js:
// 114-118 samples L_o[S] at even rows and columns, so only those values are
// evaluated, with the tile kernels' fma chains (vertical then horizontal,
// taps in increasing order, from 0.0; the oracle's CONV_SEPARABLE_FMA_VH):
// k_seed_vert forms the vertical sums of the even rows (every column),
// k_seed_horz the horizontal sums at the even columns.  3/8 of one scale's
// work instead of all S+3 scales with their planes.
#ifndef SIFT_SEED_BATCH
#define SIFT_SEED_BATCH 8  // 16 measured the same (r5aq: 34.7 vs 35.2 us at 8K octave 3)
#endif
constexpr int kSeedBatch = SIFT_SEED_BATCH;

__global__ __launch_bounds__(256) void k_seed_vert(const Pyramid P, int o, const double* __restrict__ base,
                                                   double* __restrict__ vrow) {
  const Octave& oc = P.oct[o];
  const int x = blockIdx.x * 256 + threadIdx.x, yp = blockIdx.y;
  if (x >= oc.w) return;
  const int r = oc.rad[P.S], h = oc.h;
  const double* __restrict__ wt = P.wts + oc.wofs[P.S];
  const double* __restrict__ col = base + x;
  const long long w = oc.w;
  // kSeedBatch loads in flight ahead of their fma steps (the chain's order is
  // kept): 95 taps at r = 47 are 6 dependent load rounds instead of 95
  double acc = 0.0;
  int j = 0;
  for (; j + kSeedBatch <= 2 * r + 1; j += kSeedBatch) {
    double v[kSeedBatch];
#pragma unroll
    for (int k = 0; k < kSeedBatch; ++k) v[k] = col[clampi(2 * yp + j + k - r, 0, h - 1) * w];
#pragma unroll
    for (int k = 0; k < kSeedBatch; ++k) acc = __builtin_fma(wt[j + k], v[k], acc);
  }
  for (; j <= 2 * r; ++j) acc = __builtin_fma(wt[j], col[clampi(2 * yp + j - r, 0, h - 1) * w], acc);
  vrow[(long long)yp * w + x] = acc;
}

__global__ __launch_bounds__(256) void k_seed_horz(const Pyramid P, int o, const double* __restrict__ vrow,
                                                   double* __restrict__ next) {
  const Octave& oc = P.oct[o];
  const int nw = P.oct[o + 1].w;
  const int xp = blockIdx.x * 256 + threadIdx.x, yp = blockIdx.y;
  if (xp >= nw) return;
  const int r = oc.rad[P.S], w = oc.w;
  const double* __restrict__ wt = P.wts + oc.wofs[P.S];
  const double* __restrict__ row = vrow + (long long)yp * w;
  double acc = 0.0;
  int i = 0;
  for (; i + kSeedBatch <= 2 * r + 1; i += kSeedBatch) {
    double v[kSeedBatch];
#pragma unroll
    for (int k = 0; k < kSeedBatch; ++k) v[k] = row[clampi(2 * xp + i + k - r, 0, w - 1)];
#pragma unroll
    for (int k = 0; k < kSeedBatch; ++k) acc = __builtin_fma(wt[i + k], v[k], acc);
  }
  for (; i <= 2 * r; ++i) acc = __builtin_fma(wt[i], row[clampi(2 * xp + i - r, 0, w - 1)], acc);
  next[(long long)yp * nw + xp] = acc;
}

size_t seed_only_scratch(const Pyramid& P, int o) {
  return (size_t)P.oct[o + 1].h * P.oct[o].w;
}

hipError_t launch_seed_only(const Pyramid& P, int o, const double* base, double* vrow, double* next,
                            hipStream_t st) {
  if (o < 0 || o + 1 >= P.O || !base || !vrow || !next) return hipErrorInvalidValue;
  const Octave& oc = P.oct[o];
  const Octave& on = P.oct[o + 1];
  if (2 * (on.h - 1) > oc.h - 1 || 2 * (on.w - 1) > oc.w - 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_seed_vert, dim3((oc.w + 255) / 256, on.h), dim3(256), 0, st, P, o, base, vrow);
  hipLaunchKernelGGL(k_seed_horz, dim3((on.w + 255) / 256, on.h), dim3(256), 0, st, P, o, vrow, next);
  return hipGetLastError();
}

hipError_t launch_upsample_base(const Pyramid& P, double* base0, hipStream_t st) {
  const long long n = (long long)P.oct[0].h * P.oct[0].w;
  const int blocks = (int)std::min<long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_upsample_base, dim3(blocks), dim3(256), 0, st, P, base0);
  return hipGetLastError();
}

int gauss_tile_rows(const Pyramid& P, int o) { return (P.oct[o].h + kGY - 1) / kGY; }

// Blocks per CU of the octave-o >= 1 launches: the vertical passes re-read
// the base window of every active block once per scale, and the active
// blocks of an XCD share its 4 MiB L2.  SIFT_GAUSS_BPC="b1,b2,..." caps the
// blocks per CU of octaves 1, 2, ... by padding the dynamic LDS
// (experiments; 0 = no cap).
static size_t occupancy_lds(int o, size_t lds) {
  static const std::vector<int> bpc = [] {
    std::vector<int> v;
#ifdef SIFT_EXPERIMENTS
    if (const char* e = std::getenv("SIFT_GAUSS_BPC"))
      for (const char* p = e; *p;) {
        v.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p) ++p;
      }
#endif
    return v;
  }();
  if (o < 1 || o - 1 >= (int)bpc.size() || bpc[o - 1] <= 0) return lds;
  const size_t cap = (size_t)160 * 1024 / bpc[o - 1] - 1024;
  return std::max(lds, cap);
}

hipError_t launch_gauss_dog(const Pyramid& P, GaussLaunch L, hipStream_t st, int ty_begin, int ty_end,
                            const char** kname) {
  const char* kn_dummy = nullptr;
  const char*& kn = kname ? *kname : kn_dummy;
  static_assert(kGY == kGaussTileRows, "tile rows");
  const Octave& oc = P.oct[L.o];
  if (L.nimg < 1) L.nimg = 1;
  if (L.fuse && !gauss_can_fuse(P, L.o)) return hipErrorInvalidValue;
  if (L.nimg > 1 && (L.fuse || ty_end >= 0)) return hipErrorInvalidValue;  // batches: whole octaves, no fused decisions
  if (!L.fuse && !L.vsplit && gauss_wide(P, L.o)) {
    if (!L.base) return hipErrorInvalidValue;
    const int RW = rw_width(P, L.o), tw = rw_tile_w(P, L.o);
    L.gx = (oc.w + tw - 1) / tw;
    L.gy = (oc.h + kRwRows - 1) / kRwRows;
    // Scale groups while the octave has fewer than SIFT_RW_MINB tiles x
    // groups (each group recomputes the scale before it).
    static const int minb = exp_knob("SIFT_RW_MINB", 600);
    int G = 1;
    while (G < P.NS && (long long)L.gx * L.gy * G < minb) ++G;
    split_scales(P, L.o, G, L.gb);
    L.G = G;
    L.by0 = 0;
    if (ty_end >= 0) {  // a band of kGY-row tile rows: the same rows in 8-row tiles
      if (ty_begin < 0 || ty_begin >= ty_end) return hipErrorInvalidValue;
      const int rb = ty_begin * (kGY / kRwRows), re = std::min(L.gy, ty_end * (kGY / kRwRows));
      if (rb >= re) return hipErrorInvalidValue;
      L.by0 = rb;
      L.gy = re - rb;
    }
    static const int xband = exp_knob("SIFT_XCD_BAND", -1);
    L.xcd_band = (xband >> (L.o - 1)) & 1;
    L.sw = kRwSW;
    static const int dbg = exp_knob("SIFT_GAUSS_DBG", 0);
    L.dbg = dbg;
    const bool a16 = !((reinterpret_cast<uintptr_t>(L.dog)) & 15) &&
                     (!L.gauss || !((reinterpret_cast<uintptr_t>(L.gauss)) & 15)) &&
                     (L.nimg <= 1 || ((L.dog_bs & 3) == 0 && (!L.gauss || (L.gauss_bs & 3) == 0)));  // every image's planes
    L.vec = (a16 && (oc.w & 3) == 0 && 4.0 * oc.h * oc.w < 2147483648.0) ? 1 : 0;
    L.zero = 0;
    const dim3 grid(L.gx * L.gy * L.G * L.nimg);
    const size_t lds = occupancy_lds(L.o, rw_lds(P, L.o));
    // (the streamed kernels use the tile geometry of their RW, as the window ones)
    if (RW == 48) {  // rwp_big: no other kernel for these radii in this geometry
      if (!gauss_rwp(P, L) || !L.l64) return hipErrorInvalidValue;
      hipLaunchKernelGGL((k_gauss_rwp<48, true>), grid, dim3(256), lds, st, P, L);
      kn = "k_gauss_rwp<48,l64>";
    } else if (gauss_rws(P, L.o) && gauss_rwp(P, L)) {
      if (RW == 12) hipLaunchKernelGGL((k_gauss_rwp<12, false>), grid, dim3(256), lds, st, P, L);
      else if (RW == 16) hipLaunchKernelGGL((k_gauss_rwp<16, false>), grid, dim3(256), lds, st, P, L);
      else hipLaunchKernelGGL((k_gauss_rwp<24, false>), grid, dim3(256), lds, st, P, L);
      kn = RW == 12 ? "k_gauss_rwp<12>" : RW == 16 ? "k_gauss_rwp<16>" : "k_gauss_rwp<24>";
    } else if (gauss_rws(P, L.o)) {
      if (RW == 12) hipLaunchKernelGGL((k_gauss_rw<12, true>), grid, dim3(256), lds, st, P, L);
      else if (RW == 16) hipLaunchKernelGGL((k_gauss_rw<16, true>), grid, dim3(256), lds, st, P, L);
      else hipLaunchKernelGGL((k_gauss_rw<24, true>), grid, dim3(256), lds, st, P, L);
      kn = RW == 12 ? "k_gauss_rw<12,true>" : RW == 16 ? "k_gauss_rw<16,true>" : "k_gauss_rw<24,true>";
    } else {
      if (RW == 12) hipLaunchKernelGGL(k_gauss_rw<12>, grid, dim3(256), lds, st, P, L);
      else if (RW == 16) hipLaunchKernelGGL(k_gauss_rw<16>, grid, dim3(256), lds, st, P, L);
      else hipLaunchKernelGGL(k_gauss_rw<24>, grid, dim3(256), lds, st, P, L);
      kn = RW == 12 ? "k_gauss_rw<12>" : RW == 16 ? "k_gauss_rw<16>" : "k_gauss_rw<24>";
    }
    return hipGetLastError();
  }
  const int G = scale_groups(P, L.o);
  split_scales(P, L.o, G, L.gb);
  const int tw = tile_w(P, L.o);
  L.gx = L.fuse ? fused_words_per_row(oc.w) : (oc.w + tw - 1) / tw;
  L.gy = L.fuse ? (oc.h - 2 + kFY - 1) / kFY : (oc.h + kGY - 1) / kGY;
  L.by0 = 0;
  if (ty_end >= 0) {  // a band of tile rows
    if (L.fuse || L.vsplit || ty_begin < 0 || ty_end > L.gy || ty_begin >= ty_end) return hipErrorInvalidValue;
    L.by0 = ty_begin;
    L.gy = ty_end - ty_begin;
  }
  L.G = L.fuse ? 1 : G;
  if (L.fuse && L.gx != L.X.nw) return hipErrorInvalidValue;
  // XCD-banded tile order for octaves >= 1 (SIFT_XCD_BAND: bit o-1 of the
  // value; default all).  Measured (4K, O=4, S=5): isolated pass 0.748 ->
  // 0.730 ms, pipelined bench +0.5-1 % (tools/gpu_envab.sh).
  static const int xband = exp_knob("SIFT_XCD_BAND", -1);
  static const int xband0 = exp_knob("SIFT_XCD_BAND0", 0);
  L.xcd_band = L.o >= 1 ? ((xband >> (L.o - 1)) & 1) : xband0;
  const dim3 grid(L.gx * L.gy * L.G * L.nimg);
  const size_t lds = gauss_lds_bytes(P, L.o, L.fuse != 0);
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    set_attr<true, kSW0, 8, false>();
    set_attr<true, kSW1, kUR, false>();
    set_attr<false, 0, kUR1, false>();
    (void)hipFuncSetAttribute((const void*)k_gauss_dog<false, 0, SIFT_VS_RMAX, false, kGX, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_gauss_dog<false, 0, kUR96, false, 96>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    set_attr<true, kSW0, 8, true>();
    set_attr<true, kSW1, kUR, true>();
    attr_set = true;
  }
  L.sw = strip_stride(P, L.o);
  static const int dbg = exp_knob("SIFT_GAUSS_DBG", 0);
  L.dbg = dbg;
  const bool a16 = !((reinterpret_cast<uintptr_t>(L.dog)) & 15) &&
                   (!L.gauss || !((reinterpret_cast<uintptr_t>(L.gauss)) & 15)) &&
                   (L.nimg <= 1 || ((L.dog_bs & 3) == 0 && (!L.gauss || (L.gauss_bs & 3) == 0)));  // every image's planes
  L.vec = (a16 && (oc.w & 3) == 0 && 4.0 * oc.h * oc.w < 2147483648.0) ? 1 : 0;
  L.zero = oc.rmax > (staged0(P, L.o) ? kUR : kUR1) ? 1 : 0;
  if (L.vsplit) {
    if (L.o == 0 || !L.base) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gauss_vert, dim3((oc.w + kGX - 1) / kGX, (oc.h + kVertRows - 1) / kVertRows, P.NS * L.nimg),
                       dim3(256), 0, st, P, L.o, L.base, L.vsplit, L.base_bs, L.vsplit_bs);
  }
  if (L.fuse) {  // staged octave 0 (gauss_can_fuse)
    if (L.sw == kSW0) hipLaunchKernelGGL((k_gauss_dog<true, kSW0, 8, true>), grid, dim3(256), lds, st, P, L);
    else hipLaunchKernelGGL((k_gauss_dog<true, kSW1, kUR, true>), grid, dim3(256), lds, st, P, L);
    kn = "k_gauss_dog<octave0,fused extrema>";
  } else if (tw == 96) {
    hipLaunchKernelGGL((k_gauss_dog<false, 0, kUR96, false, 96>), grid, dim3(256), occupancy_lds(L.o, lds), st, P, L);
    kn = "k_gauss_dog<96>";
  } else if (staged0(P, L.o) && L.sw == kSW0) {
    hipLaunchKernelGGL((k_gauss_dog<true, kSW0, 8, false>), grid, dim3(256), lds, st, P, L);
    kn = "k_gauss_dog<octave0>";
  } else if (staged0(P, L.o)) {
    hipLaunchKernelGGL((k_gauss_dog<true, kSW1, kUR, false>), grid, dim3(256), lds, st, P, L);
    kn = "k_gauss_dog<octave0>";
  } else {
    if (L.vsplit && SIFT_VS_KERNEL) {
      hipLaunchKernelGGL((k_gauss_dog<false, 0, SIFT_VS_RMAX, false, kGX, true>), grid, dim3(256),
                         occupancy_lds(L.o, lds), st, P, L);
    } else {
      hipLaunchKernelGGL((k_gauss_dog<false, 0, kUR1, false>), grid, dim3(256), occupancy_lds(L.o, lds), st, P, L);
    }
    kn = L.vsplit ? "k_gauss_vert + k_gauss_dog<64>" : L.o == 0 ? "k_gauss_dog<octave0,fp64 base>" : "k_gauss_dog<64>";
  }
  return hipGetLastError();
}

hipError_t launch_dog_from_gauss(const float* g, float* d, long long plane, int nd,
                                 hipStream_t st) {
  long long n = plane * nd;
  int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_dog_from_gauss, dim3(blocks), dim3(256), 0, st, g, d, plane, nd);
  return hipGetLastError();
}

}  // namespace sift
