// Gaussian scale space + Difference-of-Gaussians for one octave (gfx950).
//
// Replaces background.js:71-237 (computeGaussianScaleSpace, whose hot loop is
// SIFT_blurMatrix2DChunk, sift.js:72-149) and background.js:258-354
// (computeDifferenceOfGaussians / SIFT_subtractMatrix2DChunk, sift.js:154-188).
//
// The reference convolves every scale of an octave with a full 2D kernel of
// the SAME octave base (the blur is not incremental, background.js:173-177).
// The 2D kernel is exactly separable (w(i) w(j), sift.js:22-67).  Each 64x32
// output tile stages its base region once in LDS (fp64, replicated edges) and
// then, per scale:
//   vertical pass   base region -> fp64 LDS strip V[32][64+2r]: an 8-row
//                   register sliding window per column;
//   horizontal pass strip -> 8 outputs per thread (4 rows x 2 adjacent
//                   columns from 16-byte reads of aligned column pairs);
//   epilogue        L_s (fp32), DoG L_{s-1} - L_s formed in fp64 and rounded
//                   once (fp32), and for s == S the fp64 seed of the next
//                   octave (background.js:114-118).
// Radii 0..kRT run fully unrolled code with exactly 2r+1 taps per output
// (taps in SGPRs); larger radii use a zero-padded runtime loop.  When the
// base region does not fit (large radii, small octaves) the vertical pass
// reads the base from global memory (L1/L2) instead.
//
// Octave 0's base is the 2x nearest-neighbour upsample of the input
// (background.js:84): B[y][x] = I[clamp(y)>>1][clamp(x)>>1], never
// materialised: the tile stages input pixels, and the vertical sums (which
// depend on x only through x>>1) are computed once per input column and
// written to both strip columns 2k, 2k+1 -- the same operations on the same
// data, i.e. a pure common subexpression.
//
// Every output pixel runs the same operation sequence on its clamped
// neighbourhood (translation invariant, like the reference's 2D sum), so
// pixels with identical neighbourhoods get bit-identical values and fp32 ties
// mean what fp64 ties mean in the reference.  sift_exact.h recomputes single
// pixels with the same sums in the same fma order.
//
// Roofline: HBM-bound on the plane stores: per octave pixel 4(S+3) + 4(S+2)
// bytes written (+2 for the fp64 seed) against 1 (octave 0) or 8 bytes of
// base read.  fp64 VALU: 2(2r+1) FMAs per pixel and scale (octave 0: the
// vertical half is shared by column pairs) plus the 2r-column halo.
#include <cstdlib>
#include <utility>

#include "sift_common.h"
#include "sift_kernels.h"

namespace sift {

constexpr int kRT = -1;  // radii with unrolled code paths (-1: none; the generic loops are near-exact)

struct TileCtx {
  const Pyramid* P;
  const Octave* oc;
  double* sV;    // strip [32][VW]
  double* sB;    // staged base region [BR][BW] (nullptr: read global)
  int h, w, R, VW, BW, rlo, x0, y0, lane, wv;
  int kb_all;    // octave 0: first staged input column
};

template <bool OCT0, bool STAGED, int RAD>
__device__ __forceinline__ void vert_pass(const TileCtx& T, const cdouble* wp, int r_rt) {
  const int r = RAD >= 0 ? RAD : r_rt;
  const int h = T.h, w = T.w;
  const int ty = T.wv * kVT;
  const int yb = T.y0 + ty - r;
  const Pyramid& P = *T.P;
  // columns: o>=1 -> strip columns c = 0 .. 63+2r (x = x0-r+c);
  //          o==0 -> input columns k = kb .. ke (strip columns 2k-(x0-r), +1)
  const int kb = (T.x0 - r) >> 1;
  const int ncols = OCT0 ? (((T.x0 + kTX - 1 + r) >> 1) - kb + 1) : (kTX + 2 * r);
  for (int cb = 0; cb < ncols; cb += 64) {
    const int col = cb + T.lane;
    // source column: staged index or global column
    int scol;
    if (STAGED) scol = OCT0 ? min(kb + col - T.kb_all, T.BW - 1) : min(col + T.R - r, T.BW - 1);
    else scol = OCT0 ? clampi(kb + col, 0, P.W - 1) : clampi(T.x0 - r + col, 0, w - 1);
    auto src = [&](int j) -> double {
      const int yy = clampi(yb + j, 0, h - 1);
      if (STAGED) return T.sB[((OCT0 ? (yy >> 1) : yy) - T.rlo) * T.BW + scol];
      if (OCT0) return (double)P.img[(long long)(yy >> 1) * P.img_stride + scol];
      return P.seeds[T.oc->seed_off + (long long)yy * w + scol];
    };
    double acc[kVT];
#pragma unroll
    for (int t = 0; t < kVT; ++t) acc[t] = 0.0;
    if constexpr (RAD >= 0) {
      double v = src(0);
#pragma unroll
      for (int j = 0; j < 2 * RAD + kVT; ++j) {
        const double vn = j + 1 < 2 * RAD + kVT ? src(j + 1) : 0.0;  // one row ahead
#pragma unroll
        for (int t = 0; t < kVT; ++t) {
          const int k = j - t;
          if (k >= 0 && k <= 2 * RAD) acc[t] = fma((double)wp[k], v, acc[t]);
        }
        __builtin_amdgcn_sched_barrier(0);
        v = vn;
      }
    } else {
#pragma unroll 8
      for (int j = 0; j < 2 * r + kVT; ++j) {
        const double v = src(j);
#pragma unroll
        for (int t = 0; t < kVT; ++t) acc[t] = fma(wp[j - t], v, acc[t]);  // zero-padded taps
      }
    }
    if (col < ncols) {
      double* dst = T.sV + ty * T.VW;
      if (OCT0) {
        const int u = 2 * (kb + col) - (T.x0 - r);  // strip column of x = 2k
#pragma unroll
        for (int t = 0; t < kVT; ++t) {
          if (u >= 0 && u < kTX + 2 * r) dst[t * T.VW + u] = acc[t];
          if (u + 1 >= 0 && u + 1 < kTX + 2 * r) dst[t * T.VW + u + 1] = acc[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < kVT; ++t) dst[t * T.VW + col] = acc[t];
      }
    }
  }
}

// Horizontal pass for one scale: lane -> column pair p = lane & 31 (output
// columns x0+2p, x0+2p+1), rows ty + 2m + (lane >> 5), m = 0..3.
// out[2m + c] = sum_i w_i V[row][2p + c + i], taps in increasing i.
template <int RAD>
__device__ __forceinline__ void horz_pass(const TileCtx& T, const cdouble* wp, int r_rt, double (&out)[kVT]) {
  const int r = RAD >= 0 ? RAD : r_rt;
  const int p = T.lane & 31, half = T.lane >> 5;
  const double* base = T.sV + (T.wv * kVT + half) * T.VW + 2 * p;
#pragma unroll
  for (int q = 0; q < kVT; ++q) out[q] = 0.0;
  if constexpr (RAD >= 0) {
    // Software-pipelined one column pair ahead; the scheduling barriers keep
    // the compiler from hoisting the whole unrolled window (register blow-up).
    double2 cur[kVT / 2], nxt[kVT / 2];
#pragma unroll
    for (int m = 0; m < kVT / 2; ++m) cur[m] = *reinterpret_cast<const double2*>(base + 2 * m * T.VW);
#pragma unroll
    for (int m2 = 0; m2 <= RAD; ++m2) {  // window column pairs 2m2, 2m2+1
      if (m2 < RAD) {
#pragma unroll
        for (int m = 0; m < kVT / 2; ++m)
          nxt[m] = *reinterpret_cast<const double2*>(base + 2 * m * T.VW + 2 * (m2 + 1));
      }
      const int i0 = 2 * m2, i1 = 2 * m2 + 1;
#pragma unroll
      for (int m = 0; m < kVT / 2; ++m) {
        const double2 v = cur[m];
        out[2 * m] = fma((double)wp[i0], v.x, out[2 * m]);
        if (i0 >= 1) out[2 * m + 1] = fma((double)wp[i0 - 1], v.x, out[2 * m + 1]);
        if (i1 <= 2 * RAD) out[2 * m] = fma((double)wp[i1], v.y, out[2 * m]);
        out[2 * m + 1] = fma((double)wp[i1 - 1], v.y, out[2 * m + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < kVT / 2; ++m) cur[m] = nxt[m];
    }
  } else {
#pragma unroll 1
    for (int m2 = 0; m2 <= r; ++m2) {
      const double w0 = wp[2 * m2], w1 = wp[2 * m2 + 1], wm = wp[2 * m2 - 1];  // zero-padded
#pragma unroll
      for (int m = 0; m < kVT / 2; ++m) {
        const double2 v = *reinterpret_cast<const double2*>(base + 2 * m * T.VW + 2 * m2);
        out[2 * m] = fma(w0, v.x, out[2 * m]);
        out[2 * m + 1] = fma(wm, v.x, out[2 * m + 1]);
        out[2 * m] = fma(w1, v.y, out[2 * m]);
        out[2 * m + 1] = fma(w0, v.y, out[2 * m + 1]);
      }
    }
  }
}

template <bool OCT0, bool STAGED, int RAD>
__device__ __forceinline__ void scale_step(const TileCtx& T, const cdouble* wp, int r, double (&out)[kVT]) {
  vert_pass<OCT0, STAGED, RAD>(T, wp, r);
  __syncthreads();
  horz_pass<RAD>(T, wp, r, out);
  __syncthreads();  // the strip is rewritten by the next scale
}

template <bool OCT0, bool STAGED, int... Rs>
__device__ __forceinline__ void dispatch_scale(std::integer_sequence<int, Rs...>, const TileCtx& T,
                                               const cdouble* wp, int r, double (&out)[kVT]) {
  bool done = false;
  ((!done && r == Rs ? (scale_step<OCT0, STAGED, Rs>(T, wp, r, out), done = true) : false), ...);
  if (!done) scale_step<OCT0, STAGED, -1>(T, wp, r, out);
}

// Staged base region of a tile (rows rlo..rhi, BW columns): octave 0 stages
// input pixels (rows q = y>>1, columns k = x>>1); octave o>=1 the fp64 seed.
struct Region {
  int rlo, rhi, BW, kb_all;
};

__host__ __device__ inline Region tile_region(const Pyramid& P, int o, int x0, int y0) {
  const Octave& oc = P.oct[o];
  const int R = oc.rmax;
  Region g;
  if (o == 0) {
    g.rlo = max(0, (y0 - R) >> 1);
    g.rhi = min(P.H - 1, (y0 + kTY - 1 + R) >> 1);
    g.kb_all = (x0 - R) >> 1;
    g.BW = ((x0 + kTX - 1 + R) >> 1) - g.kb_all + 1;
  } else {
    g.rlo = max(0, y0 - R);
    g.rhi = min(oc.h - 1, y0 + kTY - 1 + R);
    g.kb_all = 0;
    g.BW = kTX + 2 * R;
  }
  return g;
}

template <bool OCT0, bool STAGED>
__global__ __launch_bounds__(256) void k_gauss_dog(const Pyramid P, const GaussLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  TileCtx T;
  T.P = &P;
  T.oc = &P.oct[L.o];
  T.h = T.oc->h;
  T.w = T.oc->w;
  T.R = T.oc->rmax;
  T.VW = kTX + 2 * T.R + 2;  // even: 16-byte aligned column pairs
  T.x0 = blockIdx.x * kTX;
  T.y0 = blockIdx.y * kTY;
  T.lane = threadIdx.x & 63;
  T.wv = threadIdx.x >> 6;
  T.sV = smem;
  T.sB = nullptr;
  T.rlo = 0;
  T.BW = 0;
  T.kb_all = 0;
  const int h = T.h, w = T.w;
  if (STAGED) {
    const Region g = tile_region(P, L.o, T.x0, T.y0);
    T.rlo = g.rlo;
    T.BW = g.BW;
    T.kb_all = g.kb_all;
    T.sB = smem + kTY * T.VW;
    // Row segments per wave, 4 rows per batch: all loads of a batch are in
    // flight before the first LDS store (no per-element latency chain).
    const int nr = g.rhi - g.rlo + 1;
    for (int rb = T.wv * 4; rb < nr; rb += 16) {
      for (int cc = T.lane; cc < g.BW; cc += 64) {
        double v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int rr = min(rb + k, nr - 1);
          if (OCT0) v[k] = (double)P.img[(long long)(g.rlo + rr) * P.img_stride + clampi(g.kb_all + cc, 0, P.W - 1)];
          else v[k] = P.seeds[T.oc->seed_off + (long long)(g.rlo + rr) * w + clampi(T.x0 - T.R + cc, 0, w - 1)];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (rb + k < nr) T.sB[(rb + k) * g.BW + cc] = v[k];
      }
    }
    __syncthreads();
  }
  const long long plane = (long long)h * w;
  const int p = T.lane & 31, half = T.lane >> 5;
  const int x = T.x0 + 2 * p;
  double lprev[kVT];
#pragma unroll
  for (int q = 0; q < kVT; ++q) lprev[q] = 0.0;

  // Scale group of this block (small octaves split their scales over
  // blockIdx.z for parallelism; a group recomputes the scale before it as
  // the DoG's L_{s-1}, without storing it).
  const int G = gridDim.z, per = (P.NS + G - 1) / G;
  const int s_begin = blockIdx.z * per, s_end = min(P.NS, s_begin + per);
  for (int s = max(0, s_begin - 1); s < s_end; ++s) {
    const bool store = s >= s_begin;
    const int r = T.oc->rad[s];
    // Taps through the constant address space: wave-uniform scalar loads.
    const cdouble* wp = (const cdouble*)(P.wts + T.oc->wofs[s]);
    double out[kVT];
    dispatch_scale<OCT0, STAGED>(std::make_integer_sequence<int, kRT + 1>{}, T, wp, r, out);

#pragma unroll
    for (int m = 0; m < kVT / 2; ++m) {
      const int y = T.y0 + T.wv * kVT + 2 * m + half;
      if (store && y < h && x < w) {
        const long long pp = (long long)y * w + x;
        const double a = out[2 * m], b = out[2 * m + 1];
        const bool has_b = x + 1 < w;
        if (L.gauss) {
          float* g = L.gauss + s * plane + pp;
          if (has_b && !(((long long)s * plane + pp) & 1)) {  // float2 needs 8-byte alignment
            *reinterpret_cast<float2*>(g) = make_float2((float)a, (float)b);
          } else {
            g[0] = (float)a;
            if (has_b) g[1] = (float)b;
          }
        }
        if (s > 0) {  // lprev = L_{s-1}: computed here even when s-1 belongs to the previous group
          float* d = L.dog + (s - 1) * plane + pp;
          const float da = (float)(lprev[2 * m] - a), db = (float)(lprev[2 * m + 1] - b);
          if (has_b && !(((long long)(s - 1) * plane + pp) & 1)) {
            *reinterpret_cast<float2*>(d) = make_float2(da, db);
          } else {
            d[0] = da;
            if (has_b) d[1] = db;
          }
        }
        if (s == P.S && L.next_seed && !(y & 1))
          L.next_seed[(long long)(y >> 1) * L.next_w + (x >> 1)] = a;
      }
    }
#pragma unroll
    for (int q = 0; q < kVT; ++q) lprev[q] = out[q];
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

static size_t strip_bytes(const Octave& oc) { return sizeof(double) * (size_t)kTY * (kTX + 2 * oc.rmax + 2); }

static size_t region_bytes(const Pyramid& P, int o) {
  const Octave& oc = P.oct[o];
  const int R = oc.rmax;
  if (o == 0) return sizeof(double) * (size_t)std::min(P.H, (kTY + 2 * R) / 2 + 2) * ((kTX + 2 * R) / 2 + 2);
  return sizeof(double) * (size_t)std::min(oc.h, kTY + 2 * R) * (kTX + 2 * R);
}

// Octave 0 stages its (tiny) input region; octaves o >= 1 read the fp64 seed
// through L1/L2, which keeps the LDS per block small and occupancy high.
// SIFT_STAGE_OCTAVES (bit mask, default 1) overrides for A/B measurements.
static bool staged(const Pyramid& P, int o) {
  static const int mask = [] {
    const char* e = std::getenv("SIFT_STAGE_OCTAVES");
    return e ? std::atoi(e) : 1;
  }();
  return ((mask >> o) & 1) && strip_bytes(P.oct[o]) + region_bytes(P, o) <= 96 * 1024;
}

// Scale groups per octave: enough blocks to fill 256 CUs several times.
static int scale_groups(const Pyramid& P, int o) {
  const Octave& oc = P.oct[o];
  const long long tiles = (long long)((oc.w + kTX - 1) / kTX) * ((oc.h + kTY - 1) / kTY);
  int g = 1;
  while (g < P.NS / 2 && tiles * g < 2048) g *= 2;
  return g;
}

size_t gauss_lds_bytes(const Pyramid& P, int o) {
  return strip_bytes(P.oct[o]) + (staged(P, o) ? region_bytes(P, o) : 0);
}

template <bool O0, bool ST>
static void set_attr() {
  (void)hipFuncSetAttribute((const void*)k_gauss_dog<O0, ST>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_gauss_dog(const Pyramid& P, const GaussLaunch& L, hipStream_t st) {
  const Octave& oc = P.oct[L.o];
  dim3 grid((oc.w + kTX - 1) / kTX, (oc.h + kTY - 1) / kTY, scale_groups(P, L.o));
  const size_t lds = gauss_lds_bytes(P, L.o);
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    set_attr<true, true>();
    set_attr<true, false>();
    set_attr<false, true>();
    set_attr<false, false>();
    attr_set = true;
  }
  const bool o0 = L.o == 0, stg = staged(P, L.o);
  if (o0 && stg) hipLaunchKernelGGL((k_gauss_dog<true, true>), grid, dim3(256), lds, st, P, L);
  else if (o0) hipLaunchKernelGGL((k_gauss_dog<true, false>), grid, dim3(256), lds, st, P, L);
  else if (stg) hipLaunchKernelGGL((k_gauss_dog<false, true>), grid, dim3(256), lds, st, P, L);
  else hipLaunchKernelGGL((k_gauss_dog<false, false>), grid, dim3(256), lds, st, P, L);
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
