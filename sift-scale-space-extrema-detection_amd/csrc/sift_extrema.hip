// 26-neighbour extrema scan with ordered, sort-free emission (gfx950).
//
// Replaces findCandidateKeypoints (background.js:359-450) and its kernel
// SIFT_findExtremas (sift.js:212-316): for DoG scales s = 1..S a pixel
// strictly greater (or strictly smaller) than all 26 neighbours, border
// excluded, is an extremum; |v| >= 0.8*thr makes it a candidate, otherwise
// it is a low-contrast extremum.  Output order is the reference's: octave,
// scale, then raster (y, x).
//
// k_extrema: one block per (64-column word, strip of kXStrip rows), one wave
// per DoG scale, sliding a 3-row window down the strip.  Each lane loads its
// column of the three DoG planes, takes x-1 / x+1 from its neighbours with
// DPP wave shifts (word edges from one extra load), reduces the 26
// neighbours with max3/min3, and ballots the candidate mask of the 64 pixels
// straight into a bitmap word [s][y][x/64] plus a per-row popcount.  k_emit
// expands the bitmap in order after an exclusive scan of the row counts --
// the candidate list comes out sorted without a sort.
//
// The planes are fp32 roundings of fp64 values.  Rounding is monotone, so an
// fp32 comparison decides the fp64 one unless two fp32 values tie; ties and
// |v| within rounding of 0.8*thr go to a short list that k_exact_extrema
// re-decides from an fp64 pointwise recompute (sift_exact.h).
#include "sift_exact.h"
#include "sift_kernels.h"

namespace sift {

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

// Value of lane-1 (lane 0 takes `edge`) / lane+1 (lane 63 takes `edge`).
__device__ __forceinline__ float from_left(float v, float edge) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_right(float v, float edge) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x130, 0xF, 0xF, false));
}

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }
__device__ __forceinline__ float min3f(float a, float b, float c) { return fminf(a, fminf(b, c)); }

// One block per (64-column word, strip of kXStrip rows); wave s-1 of the
// block scans DoG scale s.  The S waves of a block read overlapping planes
// at the same rows, so each plane streams from HBM about once (L1/L2 reuse).
__global__ __launch_bounds__(576) void k_extrema(const Pyramid P, const ExtremaLaunch L) {
  const Octave& oc = P.oct[L.o];
  const int h = oc.h, w = oc.w;
  const int lane = threadIdx.x & 63;
  const int s = 1 + (threadIdx.x >> 6);
  const int xw = blockIdx.x;
  const int y0 = 1 + blockIdx.y * kXStrip;
  const int y1 = min(h - 2, y0 + kXStrip - 1);
  const long long plane = (long long)h * w;
  const float* __restrict__ D = P.dog + oc.dog_off;
  const float* __restrict__ Dm = D + (s - 1) * plane;
  const float* __restrict__ Dc = D + s * plane;
  const float* __restrict__ Dq = D + (s + 1) * plane;
  const double T = P.pix_thr;
  const int x = xw * 64 + lane;
  const int xc = min(x, w - 1);
  const bool is_edge = lane == 0 || lane == 63;
  const int xe = clampi(lane == 0 ? x - 1 : x + 1, 0, w - 1);
  const bool col_ok = x >= 1 && x <= w - 2;
  unsigned low = 0;

  // Sliding 3-row window: per plane the 3-wide max/min of rows y-1, y, y+1;
  // the centre plane also keeps the 2-wide (x-1, x+1) max/min and the value.
  float mx[3][3], mn[3][3], emx[3], emn[3], cv[3];
  const float* planes[3] = {Dm, Dc, Dq};
  auto derive = [&](const float (&v3)[3], const float (&e3)[3], int slot) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float v = v3[q];
      const float vl = from_left(v, e3[q]), vr = from_right(v, e3[q]);
      mx[q][slot] = max3f(vl, v, vr);
      mn[q][slot] = min3f(vl, v, vr);
      if (q == 1) {
        emx[slot] = fmaxf(vl, vr);
        emn[slot] = fminf(vl, vr);
        cv[slot] = v;
      }
    }
  };
  auto fetch = [&](int yy, float (&v3)[3], float (&e3)[3]) {
    const long long row = (long long)min(yy, h - 1) * w;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      v3[q] = planes[q][row + xc];
      e3[q] = is_edge ? planes[q][row + xe] : 0.0f;
    }
  };
  {
    float v3[3], e3[3];
    fetch(y0 - 1, v3, e3);
    derive(v3, e3, 0);
    fetch(y0, v3, e3);
    derive(v3, e3, 1);
  }
  // Rows are fetched kXG at a time so several loads per lane are in flight.
  float pv[kXG][3], pe[kXG][3];
  for (int y = y0; y <= y1; ++y) {
    const int g = (y - y0) % kXG;
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < kXG; ++k) fetch(y + 1 + k, pv[k], pe[k]);
    }
    // select group slot g (static indices keep the arrays in registers)
    float v3[3], e3[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) { v3[q] = pv[0][q]; e3[q] = pe[0][q]; }
#pragma unroll
    for (int k = 1; k < kXG; ++k)
      if (g == k) {
#pragma unroll
        for (int q = 0; q < 3; ++q) { v3[q] = pv[k][q]; e3[q] = pe[k][q]; }
      }
    derive(v3, e3, 2);
    const float v = cv[1];
    const float nmax = max3f(max3f(mx[0][0], mx[0][1], mx[0][2]), max3f(mx[2][0], mx[2][1], mx[2][2]),
                             max3f(mx[1][0], mx[1][2], emx[1]));
    const float nmin = min3f(min3f(mn[0][0], mn[0][1], mn[0][2]), min3f(mn[2][0], mn[2][1], mn[2][2]),
                             min3f(mn[1][0], mn[1][2], emn[1]));
    const bool possible = v >= nmax || v <= nmin;  // no neighbour strictly beyond v
    const bool certain = v > nmax || v < nmin;     // strict in fp32 => strict in fp64
    bool ext, tie;
    if (L.exact_planes) { ext = certain; tie = false; }
    else { ext = possible; tie = !certain; }
    ext = ext && col_ok;
    const double av = fabs((double)v);
    bool low_certain, contrast_amb = false;
    if (L.exact_planes) {
      low_certain = av < T;
    } else {
      const double e = av * 0x1p-24 + 1e-300;  // |v - v_fp64| <= ulp/2 <= |v| 2^-24
      low_certain = av + e < T;
      contrast_amb = !low_certain && av - e < T;
    }
    const bool count_low = ext && low_certain && !tie;
    const bool bit = ext && !count_low;
    low += count_low ? 1u : 0u;
    const unsigned long long word = __ballot(bit);
    if (lane == 0) {
      L.bitmap[((long long)(s - 1) * h + y) * L.nw + xw] = word;
      if (word) atomicAdd(&L.rowcount[(s - 1) * h + y], (unsigned)__popcll(word));
    }
    const bool amb = bit && (tie || contrast_amb);
    if (__ballot(amb)) {  // rare
      const unsigned slot = wave_append(amb, &L.counters[0]);
      if (amb && slot < L.amb_cap)
        L.amb_keys[slot] = oc.key_off + (unsigned)(s - 1) * (unsigned)plane + (unsigned)y * (unsigned)w + (unsigned)x;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      mx[q][0] = mx[q][1]; mx[q][1] = mx[q][2];
      mn[q][0] = mn[q][1]; mn[q][1] = mn[q][2];
    }
    emx[0] = emx[1]; emx[1] = emx[2];
    emn[0] = emn[1]; emn[1] = emn[2];
    cv[0] = cv[1]; cv[1] = cv[2];
  }
  // wave sum of the low-contrast count, one atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) low += __shfl_xor(low, off);
  if (lane == 0 && low) atomicAdd(&L.counters[1], low);
}

// One wave per (scale, row) of one octave: expand the row's bitmap words in
// order at the row's offset.  Candidate values are the fp32 plane values
// (ambiguous ones get their exact fp64 value from k_exact_extrema).
__global__ __launch_bounds__(256) void k_emit(const Pyramid P, const EmitLaunch E) {
  const Octave& oc = P.oct[E.o];
  const int h = oc.h, w = oc.w;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // (s-1)*h + y
  if (row >= P.S * h) return;
  const int s = row / h + 1, y = row - (s - 1) * h;
  if (y < 1 || y > h - 2) return;
  const unsigned cnt = E.rowcount[row];
  if (cnt == 0) return;
  unsigned base = E.rowoff[E.row_base + row];
  const long long plane = (long long)h * w;
  const float* __restrict__ Dc = P.dog + oc.dog_off + s * plane + (long long)y * w;
  const unsigned kbase = oc.key_off + (unsigned)(s - 1) * (unsigned)plane + (unsigned)y * (unsigned)w;
  for (int xw0 = 0; xw0 < E.nw; xw0 += 64) {
    const int xw = xw0 + lane;
    unsigned long long word = xw < E.nw ? E.bitmap[(long long)row * E.nw + xw] : 0ull;
    unsigned c = (unsigned)__popcll(word);
    // inclusive wave scan of c
    unsigned inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned t = __shfl_up(inc, off);
      if (lane >= off) inc += t;
    }
    unsigned pos = base + inc - c;
    while (word) {
      const int b = __ffsll((long long)word) - 1;
      word &= word - 1;
      const int x = xw * 64 + b;
      E.keys[pos] = kbase + (unsigned)x;
      E.value[pos] = (double)Dc[x];
      E.keep[pos] = 1u;
      ++pos;
    }
    base += __shfl(inc, 63);
  }
}

// One 64-thread block (one wave) per ambiguous candidate: fp64 recompute of
// the 3x3x3 patch decides extremum and contrast exactly.
__global__ __launch_bounds__(64) void k_exact_extrema(const Pyramid P, const ExactLaunch X) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const unsigned key = X.amb_keys[blockIdx.x];
  // position of key in the ordered candidate list (binary search)
  unsigned lo = 0, hi = X.n;
  while (lo < hi) {
    const unsigned mid = (lo + hi) >> 1;
    if (X.keys[mid] < key) lo = mid + 1; else hi = mid;
  }
  const unsigned idx = lo;
  int o, s, y, x;
  decode_key(P, key, o, s, y, x);
  double* d27 = smem;
  double* Lbuf = smem + 32;
  double* sh = smem + 32 + 40;
  wave_dog_patch(P, o, s, y, x, sh, Lbuf, d27);
  if (threadIdx.x == 0 && idx < X.n && X.keys[idx] == key) {
    const double v = d27[13];
    bool gt = false, lt = false;
    for (int q = 0; q < 27; ++q) {
      if (q == 13) continue;
      gt |= d27[q] >= v;  // a neighbour >= v rules out a strict maximum
      lt |= d27[q] <= v;
    }
    const bool ext = !gt || !lt;
    const bool cand = ext && fabs(v) >= P.pix_thr;
    X.keep[idx] = cand ? 1u : 0u;
    X.value[idx] = v;
    if (ext && !cand) atomicAdd(&X.counters[1], 1u);
    if (!cand) atomicAdd(&X.counters[2], 1u);  // dropped entries
  }
}

hipError_t launch_extrema(const Pyramid& P, const ExtremaLaunch& L, hipStream_t st) {
  const Octave& oc = P.oct[L.o];
  if (oc.h < 3 || oc.w < 3 || P.S < 1) return hipSuccess;  // no interior pixels
  const int strips = (oc.h - 2 + kXStrip - 1) / kXStrip;
  hipLaunchKernelGGL(k_extrema, dim3(L.nw, strips), dim3(64 * P.S), 0, st, P, L);
  return hipGetLastError();
}

hipError_t launch_emit(const Pyramid& P, const EmitLaunch& E, hipStream_t st) {
  const Octave& oc = P.oct[E.o];
  if (oc.h < 3 || oc.w < 3) return hipSuccess;
  const int rows = P.S * oc.h;
  hipLaunchKernelGGL(k_emit, dim3((rows + 3) / 4), dim3(256), 0, st, P, E);
  return hipGetLastError();
}

size_t exact_lds_bytes(const Pyramid& P) {
  int rmax = 0;
  for (int o = 0; o < P.O; ++o) rmax = std::max(rmax, P.oct[o].rmax);
  return sizeof(double) * (size_t)(32 + 40 + exact_scratch_doubles(rmax));
}

hipError_t launch_exact_extrema(const Pyramid& P, const ExactLaunch& X, unsigned n_amb, hipStream_t st) {
  if (n_amb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_exact_extrema, dim3(n_amb), dim3(64), exact_lds_bytes(P), st, P, X);
  return hipGetLastError();
}

}  // namespace sift
