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

// LDS doubles one wave needs: 3 rows x (2R+3) vertical sums + 4 scales x 9 outputs.
__host__ __device__ inline int exact_scratch_doubles(int rmax) { return 3 * (2 * rmax + 3) + 36; }

// L at rows y-1..y+1, cols x-1..x+1 of L-scale t -> out[9] (row-major).
// Requires blockDim.x == 64 (one wave): __syncthreads() is a wave barrier.
__device__ inline void wave_L_patch(const Pyramid& P, int o, int t, int y, int x, double* sh,
                                    double* out) {
  const Octave& oc = P.oct[o];
  const int h = oc.h, w = oc.w, r = oc.rad[t];
  const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
  const int lane = threadIdx.x & 63;
  const int nc = 2 * r + 3;  // columns x-1-r .. x+1+r
  // vertical: V[a][c] = sum_j w_j B(clamp(y-1+a-r+j), clamp(x-1-r+c))
  for (int idx = lane; idx < 3 * nc; idx += 64) {
    const int a = idx / nc, c = idx - nc * a;
    const int xx = clampi(x - 1 - r + c, 0, w - 1);
    const int yb = y - 1 + a - r;
    double acc = 0.0;
    for (int j = 0; j <= 2 * r; ++j) acc = fma(wp[j], base_at(P, o, clampi(yb + j, 0, h - 1), xx), acc);
    sh[idx] = acc;
  }
  __syncthreads();
  // horizontal: L[a][b] = sum_i w_i V[a][b + i]  (output column x-1+b)
  if (lane < 9) {
    const int a = lane / 3, b = lane - 3 * a;
    double acc = 0.0;
    for (int i = 0; i <= 2 * r; ++i) acc = fma(wp[i], sh[a * nc + b + i], acc);
    out[lane] = acc;
  }
  __syncthreads();
}

// DoG patch d[k][a][c] for DoG scales s-1+k (k = 0..2), rows y-1+a, cols
// x-1+c: L-scales s-1..s+2.  Result in lds d27[27] (visible to all lanes).
__device__ inline void wave_dog_patch(const Pyramid& P, int o, int s, int y, int x, double* sh,
                                      double* Lbuf /*36*/, double* d27) {
  for (int k = 0; k < 4; ++k) wave_L_patch(P, o, s - 1 + k, y, x, sh, Lbuf + 9 * k);
  const int lane = threadIdx.x & 63;
  if (lane < 27) {
    const int k = lane / 9, q = lane - 9 * k;
    d27[lane] = Lbuf[9 * k + q] - Lbuf[9 * (k + 1) + q];
  }
  __syncthreads();
}

}  // namespace sift
