// Wave-level pieces of the 26-neighbour extrema decision (gfx950), shared by
// the extrema scan (k_extrema, sift_extrema.hip) and the decisions fused into
// the Gaussian+DoG pass (k_gauss_dog, sift_gauss.hip).  One lane per column;
// x-1 / x+1 come from DPP wave shifts.  SIFT_findExtremas, sift.js:212-316:
// strict 26-neighbour min/max, |v| >= 0.8 thr -> candidate, else low contrast.
#pragma once
#include "sift_common.h"

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

// Lane l-1 / lane l+1 of a wave (DPP wave shifts; lanes 0 / 63 get 0, they
// are halo lanes whose results are never used).
__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

// IEEE 754-2019 maximum / minimum (v_maximum3_f32 / v_minimum3_f32 on
// gfx950): a NaN operand gives NaN, so a NaN neighbour makes every strict
// comparison of the centre false, as the reference's comparisons do
// (sift.js:227-256; caller-supplied planes may hold NaN / Inf).  fmaxf /
// fminf would lower to v_max_f32 behind a canonicalising v_max_f32 x, x, x of
// every loaded or DPP-moved operand (3 extra VALU per plane row), and
// -fno-honor-nans would let the compiler turn these into v_max_f32, which
// drops the NaN (tests/test_gpu_parity.py::test_foreign_dog_with_nonfinite_values).
__device__ __forceinline__ float fmax2(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float fmin2(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmax2(a, fmax2(b, c)); }
__device__ __forceinline__ float min3f(float a, float b, float c) { return fmin2(a, fmin2(b, c)); }

// Per-wave state of the 3-row window over NP consecutive DoG planes (the
// centre planes 1..NP-2 are scales, 0 and NP-1 their outer neighbours).
// Slot k holds the row whose offset from the group's first centre row is
// k mod 3; all indices are compile-time constants, so nothing rotates.
template <int NP>
struct XWin {
  float hx[3][NP], hn[3][NP];  // 3-wide max / min of a row
  float ex[3][NP], en[3][NP];  // 2-wide (x-1, x+1) max / min (centre planes)
  float cv[3][NP];             // the value (every plane: the outer ones feed the patch capture)
  float raw[3][NP];            // loaded, not yet derived rows
};

// Row reductions of one loaded row (all NP planes) into window slot K.
template <int NP, int K>
__device__ __forceinline__ void x_derive(XWin<NP>& Wn, const float (&src)[NP]) {
#if defined(SIFT_X_PROBE) && SIFT_X_PROBE > 1  // timing probe: loads only
#pragma unroll
  for (int q = 0; q < NP; ++q) { Wn.hx[K][q] = src[q]; Wn.hn[K][q] = src[q]; }
  return;
#endif
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const float v = src[q];
    const float l = from_left(v), r = from_right(v);
    const float m2 = fmax2(l, r), n2 = fmin2(l, r);
    Wn.hx[K][q] = fmax2(m2, v);
    Wn.hn[K][q] = fmin2(n2, v);
    Wn.cv[K][q] = v;
    if (q >= 1 && q <= NP - 2) {
      Wn.ex[K][q] = m2;
      Wn.en[K][q] = n2;
    }
  }
}

// The decision of one centre row (one lane per column) on fp32 DoG values: v
// the centre, nmax / nmin the max / min of its 26 neighbours.  fp32 rounding
// is monotone, so a comparison of fp32 values decides the fp64 one unless the
// values tie; ties and |v| within fp32 rounding of 0.8 thr (c_lo <= |v| <
// c_hi) are ambiguous: kept in the candidate bitmap and their keys (key of
// this lane) appended for the exact fp64 pass.  Certain low-contrast extrema
// are counted into `low` and returned in `lowmask` (the reference's
// lowContrastKeypoints, sift.js:293-306).  Returns the candidate lanes
// (ambiguous included).
// Most rows of a word hold no extremum at a given scale: one ballot decides,
// the rest is skipped (lane-mask logic in SALU).
__device__ __forceinline__ unsigned long long x_row_decide(float v, float nmax, float nmin,
                                                           unsigned long long colmask, float c_lo, float c_hi,
                                                           bool exact_planes, unsigned key, unsigned* amb_count,
                                                           unsigned* amb_keys, unsigned amb_cap, unsigned& low,
                                                           unsigned long long& lowmask, unsigned long long& ambmask) {
  lowmask = 0ull;
  ambmask = 0ull;
  // two compare masks OR-ed in SALU (a ballot of the || goes through a
  // v_cndmask + v_cmp of the combined lane bool: 2 VALU per scale and row)
  const unsigned long long ext_any =
      (__builtin_amdgcn_ballot_w64(v >= nmax) | __builtin_amdgcn_ballot_w64(v <= nmin)) & colmask;
  if (!ext_any) return 0ull;
  const float av = __builtin_fabsf(v);
  const unsigned long long gt = __ballot(v > nmax), lt = __ballot(v < nmin);
  const unsigned long long lo = __ballot(av < c_lo), hi = __ballot(av >= c_hi);
  const unsigned long long certain = (gt | lt) & colmask;
  unsigned long long ext, tie;
  if (exact_planes) { ext = certain; tie = 0ull; }
  else { ext = ext_any; tie = ext & ~certain; }
  const unsigned long long count_low = ext & lo & ~tie;
  const unsigned long long bit = ext & ~count_low;
  const unsigned long long amb = bit & (tie | ~hi);
  low += (unsigned)__popcll(count_low);
  lowmask = count_low;
  ambmask = amb;
  if (amb && amb_keys) {  // rare: ties / contrast within fp32 rounding of the threshold
    const bool mine = (amb >> (threadIdx.x & 63)) & 1ull;
    const unsigned slot = wave_append(mine, amb_count);
    if (mine && slot < amb_cap) amb_keys[slot] = key;
  }
  return bit;
}

}  // namespace sift
