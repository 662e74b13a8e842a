// Exact fp64 pointwise recompute of a 3x3x3 DoG patch, one wave per patch.
//
// Used only where an fp32 plane value cannot decide a comparison (extremum
// ties, contrast and refinement decisions within the fp32 error bound).  It
// evaluates the SAME separable sums as k_gauss_dog, term for term and in the
// same fma order, straight from the octave base (input image / fp64 seed), so
// its values equal the fp64 values k_gauss_dog formed before rounding.
#pragma once
#include "sift_common.h"

namespace sift {

// LDS hand-off between the lanes of one wave: its LDS operations complete in
// order, so waiting for its own (and a wave barrier) is all the ordering.
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

constexpr int kExactBatch = 16;  // <= kWPad: the zero taps after a weight vector cover a partial batch
static_assert(kExactBatch <= kWPad, "batched taps stay inside the zero padding");

// LDS doubles one wave needs: 4 L-scales x 3 rows x (2R+3) vertical sums.
__host__ __device__ inline int exact_scratch_doubles(int rmax) { return 12 * (2 * rmax + 3) + 36; }

// DoG patch d[k][a][c] of image im for DoG scales s-1+k (k = 0..2), rows
// y-1+a, cols x-1+c, from the L-scales s-1..s+2.  Result in lds d27[27] (visible to all
// lanes of the calling wave).  One wave per call: the LDS hand-offs are
// wave-local (wave_sync), so several waves of a block may each work on their
// own patch with their own sh / Lbuf / d27.  The four L-scales' vertical sums run side by side (one pass over
// 12 (2r+3) independent fma chains), then 36 lanes form the horizontal sums:
//   V_t[a][c] = sum_j w_j B(clamp(y-1+a-r+j), clamp(x-1-r+c))
//   L_t[a][b] = sum_i w_i V_t[a][b + i]            (output column x-1+b)
// NT = 64: one wave per patch (wave-local hand-offs).  NT > 64: the NT
// threads of a block share one patch (its vertical chains spread NT wide:
// at radius 47 a wave's lanes walk ~15 chains of 95 dependent loads each,
// the latency of the exact refinement; block barriers for the hand-offs).
template <int NT>
__device__ inline void dog_patch(const Pyramid& P, int im, int o, int s, int y, int x, double* sh,
                                 double* Lbuf /*36*/, double* d27) {
  const Octave& oc = P.oct[o];
  const int h = oc.h, w = oc.w;
  const int lane = NT == 64 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  auto wave_sync = [] {
    if (NT == 64) sift::wave_sync();
    else __syncthreads();
  };
  if (oc.l64_off >= 0) {  // the wide-radius path kept this octave's fp64 Gaussian planes: the values themselves
    if (lane < 27) {
      const int k = lane / 9, q = lane - 9 * k, a = q / 3, c = q - 3 * a;
      const long long plane = (long long)h * w;
      const double* L0 = P.l64 + im * P.l64_bstride + oc.l64_off + (long long)(s - 1 + k) * plane + (long long)(y - 1 + a) * w + (x - 1 + c);
      d27[lane] = L0[0] - L0[plane];
    }
    wave_sync();
    return;
  }
  const int nc0 = 2 * oc.rad[s - 1] + 3, nc1 = 2 * oc.rad[s] + 3, nc2 = 2 * oc.rad[s + 1] + 3,
            nc3 = 2 * oc.rad[s + 2] + 3;
  const int o1 = 3 * nc0, o2 = o1 + 3 * nc1, o3 = o2 + 3 * nc2, o4 = o3 + 3 * nc3;
  if (P.vsum && o == P.vsum_oct) {
    // The split pass already formed every vertical sum of this octave (the
    // same chain, bit for bit): 8 independent loads per lane in flight
    // instead of 12 (2r+3) chains of 2r+1 dependent steps (4K octave 3:
    // ~18 rounds of 95 per lane).
    const double* vb = P.vsum + im * P.vsum_bstride + (long long)(y - 1) * w;
    const long long plane = (long long)h * w;
    for (int i0 = lane; i0 < o4; i0 += 8 * NT) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = min(i0 + u * NT, o4 - 1);
        const int k = idx >= o3 ? 3 : idx >= o2 ? 2 : idx >= o1 ? 1 : 0;
        const int base = k == 3 ? o3 : k == 2 ? o2 : k == 1 ? o1 : 0;
        const int nc = k == 3 ? nc3 : k == 2 ? nc2 : k == 1 ? nc1 : nc0;
        const int t = s - 1 + k, r = oc.rad[t];
        const int li = idx - base;
        const int a = li / nc, c = li - nc * a;
        v[u] = vb[t * plane + (long long)a * w + clampi(x - 1 - r + c, 0, w - 1)];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + u * NT < o4) sh[i0 + u * NT] = v[u];
    }
  } else
  for (int idx = lane; idx < o4; idx += NT) {
    const int k = idx >= o3 ? 3 : idx >= o2 ? 2 : idx >= o1 ? 1 : 0;
    const int base = k == 3 ? o3 : k == 2 ? o2 : k == 1 ? o1 : 0;
    const int nc = k == 3 ? nc3 : k == 2 ? nc2 : k == 1 ? nc1 : nc0;
    const int t = s - 1 + k, r = oc.rad[t];
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
    const int li = idx - base;
    const int a = li / nc, c = li - nc * a;
    const int xx = clampi(x - 1 - r + c, 0, w - 1);
    const int yb = y - 1 + a - r;
    // 16 loads in flight ahead of their fmas (the chain is latency bound
    // otherwise); taps past 2r are the zero padding of wts: fma(0, v, acc) ==
    // acc, so the sum is the same chain, bit for bit.
    double acc = 0.0;
    for (int jb = 0; jb <= 2 * r; jb += kExactBatch) {
      double v[kExactBatch];
#pragma unroll
      for (int k = 0; k < kExactBatch; ++k) v[k] = base_at(P, im, o, clampi(yb + jb + k, 0, h - 1), xx);
#pragma unroll
      for (int k = 0; k < kExactBatch; ++k) acc = fma(wp[jb + k], v[k], acc);
    }
    sh[idx] = acc;
  }
  wave_sync();
  if (lane < 36) {
    const int k = lane / 9, q = lane - 9 * k;
    const int a = q / 3, b = q - 3 * a;
    const int base = k == 3 ? o3 : k == 2 ? o2 : k == 1 ? o1 : 0;
    const int nc = k == 3 ? nc3 : k == 2 ? nc2 : k == 1 ? nc1 : nc0;
    const int t = s - 1 + k, r = oc.rad[t];
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
    double acc = 0.0;
    for (int i = 0; i <= 2 * r; ++i) acc = fma(wp[i], sh[base + a * nc + b + i], acc);
    Lbuf[lane] = acc;
  }
  wave_sync();
  if (lane < 27) {
    const int k = lane / 9, q = lane - 9 * k;
    d27[lane] = Lbuf[9 * k + q] - Lbuf[9 * (k + 1) + q];
  }
  wave_sync();
}

__device__ inline void wave_dog_patch(const Pyramid& P, int im, int o, int s, int y, int x, double* sh,
                                      double* Lbuf /*36*/, double* d27) {
  dog_patch<64>(P, im, o, s, y, x, sh, Lbuf, d27);
}

}  // namespace sift
