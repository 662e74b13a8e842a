// 26-neighbour extrema scan + ordering (gfx950).
//
// Replaces findCandidateKeypoints (background.js:359-450) and its kernel
// SIFT_findExtremas (sift.js:212-316): for DoG scales s = 1..S, a pixel
// strictly greater (or strictly smaller) than all 26 neighbours, border
// excluded, is an extremum; |v| >= 0.8*thr makes it a candidate, otherwise it
// is a low-contrast extremum.
//
// The planes are fp32 roundings of fp64 values.  Rounding is monotone, so an
// fp32 comparison decides the fp64 one unless the two fp32 values are equal:
// such ties (and |v| within rounding of 0.8*thr) are flagged and re-decided
// by k_exact_extrema from an fp64 pointwise recompute.  Records are appended
// with wave-aggregated atomics, then sorted by key = (octave, scale, y, x),
// which is exactly the reference's output order (raster order per trio).
#include "sift_exact.h"
#include "sift_kernels.h"

namespace sift {

constexpr int kXRows = 16;  // rows per wave in the extrema scan

__device__ __forceinline__ unsigned lane_prefix(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// Wave-aggregated append: returns this lane's slot (valid where pred).
__device__ __forceinline__ unsigned wave_append(bool pred, unsigned* counter) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0ull) return 0u;
  const int leader = __ffsll((long long)mask) - 1;
  unsigned base = 0u;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, (unsigned)__popcll(mask));
  base = __shfl(base, leader);
  return base + lane_prefix(mask);
}

__global__ __launch_bounds__(256) void k_extrema(const Pyramid P, const ExtremaLaunch L) {
  const Octave& oc = P.oct[L.o];
  const int h = oc.h, w = oc.w;
  const int s = blockIdx.z + 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int x = 1 + blockIdx.x * 64 + lane;
  const int ybeg = 1 + (blockIdx.y * 4 + wv) * kXRows;
  if (ybeg > h - 2) return;  // wave-uniform
  const int yend = min(h - 2, ybeg + kXRows - 1);
  const long long plane = (long long)h * w;
  const float* __restrict__ D = P.dog + oc.dog_off;
  const float* __restrict__ Dm = D + (s - 1) * plane;
  const float* __restrict__ Dc = D + s * plane;
  const float* __restrict__ Dp = D + (s + 1) * plane;
  const bool col_ok = x <= w - 2;
  const int xc = col_ok ? x : 1;  // keep loads in bounds for idle lanes

  // 3 planes x 3 rows x 3 cols sliding down the column.
  float m[3][3], c[3][3], p[3][3];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const long long row = (long long)(ybeg - 1 + a) * w + xc - 1;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      m[a][b] = Dm[row + b];
      c[a][b] = Dc[row + b];
      p[a][b] = Dp[row + b];
    }
  }
  const double T = P.pix_thr;
  for (int y = ybeg; y <= yend; ++y) {
    {
      const long long row = (long long)(y + 1) * w + xc - 1;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        m[2][b] = Dm[row + b];
        c[2][b] = Dc[row + b];
        p[2][b] = Dp[row + b];
      }
    }
    const float v = c[1][1];
    bool gt = false, lt = false, eq = false;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        gt |= (m[a][b] > v) | (p[a][b] > v);
        lt |= (m[a][b] < v) | (p[a][b] < v);
        eq |= (m[a][b] == v) | (p[a][b] == v);
        if (a != 1 || b != 1) {
          gt |= c[a][b] > v;
          lt |= c[a][b] < v;
          eq |= c[a][b] == v;
        }
      }
    const bool possible = !gt || !lt;         // every neighbour <= v, or every one >= v
    const bool certain = possible && !eq;     // strict in fp32 => strict in fp64
    bool ext, tie;
    if (L.exact_planes) { ext = certain; tie = false; }
    else { ext = possible; tie = !certain; }
    ext = ext && col_ok;
    const double av = fabs((double)v);
    unsigned flags = tie ? kFlagTie : 0u;
    bool low_certain;
    if (L.exact_planes) {
      low_certain = av < T;
    } else {
      const double e = av * 0x1p-24 + 1e-300;  // |v - v_fp64| <= ulp/2 <= |v| 2^-24
      low_certain = av + e < T;
      if (!low_certain && av - e < T) flags |= kFlagContrast;
    }
    const bool count_low = ext && low_certain && !tie;
    const bool emit = ext && !count_low;
    const unsigned long long lowmask = __ballot(count_low);
    if (lowmask && lane == __ffsll((long long)lowmask) - 1) atomicAdd(&L.counters[1], (unsigned)__popcll(lowmask));
    const unsigned slot = wave_append(emit, &L.counters[0]);
    if (emit && slot < L.cap) {
      L.keys[slot] = oc.key_off + (unsigned)(s - 1) * (unsigned)plane + (unsigned)y * (unsigned)w + (unsigned)x;
      L.payload[slot] = ((unsigned long long)__float_as_uint(v) << 32) | flags;
    }
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      m[0][b] = m[1][b]; m[1][b] = m[2][b];
      c[0][b] = c[1][b]; c[1][b] = c[2][b];
      p[0][b] = p[1][b]; p[1][b] = p[2][b];
    }
  }
}

__global__ __launch_bounds__(256) void k_cand_init(const CandInit C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool fl = false;
  if (i < C.n) {
    const unsigned long long pl = C.payload[i];
    const unsigned flags = (unsigned)(pl & 0xffffffffull);
    const float v = __uint_as_float((unsigned)(pl >> 32));
    C.keep[i] = flags ? 0u : 1u;
    C.value[i] = (double)v;
    fl = flags != 0u;
  }
  const unsigned slot = wave_append(fl, &C.counters[2]);
  if (fl) C.flagged[slot] = (unsigned)i;
}

// One 64-thread block (one wave) per flagged candidate.
__global__ __launch_bounds__(64) void k_exact_extrema(const Pyramid P, const CandInit C) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const unsigned idx = C.flagged[blockIdx.x];
  int o, s, y, x;
  decode_key(P, C.keys[idx], o, s, y, x);
  double* d27 = smem;
  double* Lbuf = smem + 32;
  double* sh = smem + 32 + 40;
  wave_dog_patch(P, o, s, y, x, sh, Lbuf, d27);
  if (threadIdx.x == 0) {
    const double v = d27[13];
    bool gt = false, lt = false;
    for (int q = 0; q < 27; ++q) {
      if (q == 13) continue;
      gt |= d27[q] >= v;  // a neighbour >= v rules out a strict maximum
      lt |= d27[q] <= v;
    }
    const bool ext = !gt || !lt;
    const bool cand = ext && fabs(v) >= P.pix_thr;
    C.keep[idx] = cand ? 1u : 0u;
    C.value[idx] = v;
    if (ext && !cand) atomicAdd(&C.counters[1], 1u);
  }
}

__global__ __launch_bounds__(256) void k_scatter_cand(const unsigned* __restrict__ keep,
                                                      const unsigned* __restrict__ pos,
                                                      const unsigned* __restrict__ keys,
                                                      const double* __restrict__ val, int n,
                                                      unsigned* __restrict__ out_key,
                                                      double* __restrict__ out_val) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && keep[i]) {
    out_key[pos[i]] = keys[i];
    out_val[pos[i]] = val[i];
  }
}

hipError_t launch_extrema(const Pyramid& P, const ExtremaLaunch& L, hipStream_t st) {
  const Octave& oc = P.oct[L.o];
  if (oc.h < 3 || oc.w < 3 || P.S < 1) return hipSuccess;  // no interior pixels
  const int inner_h = oc.h - 2, inner_w = oc.w - 2;
  dim3 grid((inner_w + 63) / 64, (inner_h + 4 * kXRows - 1) / (4 * kXRows), P.S);
  hipLaunchKernelGGL(k_extrema, grid, dim3(256), 0, st, P, L);
  return hipGetLastError();
}

hipError_t launch_cand_init(const CandInit& C, hipStream_t st) {
  if (C.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cand_init, dim3((C.n + 255) / 256), dim3(256), 0, st, C);
  return hipGetLastError();
}

size_t exact_lds_bytes(const Pyramid& P) {
  int rmax = 0;
  for (int o = 0; o < P.O; ++o) rmax = std::max(rmax, P.oct[o].rmax);
  return sizeof(double) * (size_t)(32 + 40 + exact_scratch_doubles(rmax));
}

hipError_t launch_exact_extrema(const Pyramid& P, const CandInit& C, unsigned n_flagged,
                                hipStream_t st) {
  if (n_flagged == 0) return hipSuccess;
  hipLaunchKernelGGL(k_exact_extrema, dim3(n_flagged), dim3(64), exact_lds_bytes(P), st, P, C);
  return hipGetLastError();
}

hipError_t launch_scatter_candidates(const unsigned* keep, const unsigned* pos, const unsigned* keys,
                                     const double* val, int n, unsigned* out_key, double* out_val,
                                     hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_cand, dim3((n + 255) / 256), dim3(256), 0, st, keep, pos, keys, val, n,
                     out_key, out_val);
  return hipGetLastError();
}

}  // namespace sift
