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

// LDS doubles one wave needs: strip of 3 x (2R+3) + 4 scales x 9 outputs.
__host__ __device__ inline int exact_scratch_doubles(int rmax) { return 3 * (2 * rmax + 5) + 36; }

// Octave 0: the folded form k_gauss_o0 evaluates (input rows q, parity taps).
__device__ inline void wave_L_patch_o0(const Pyramid& P, int t, int y, int x, double* sh, double* out) {
  const Octave& oc = P.oct[0];
  const int H = P.H, W = P.W, r = oc.rad[t], c = fold_half(r);  // strip: nr <= 2c + 3 rows
  const int lane = threadIdx.x & 63;
  const int qbase = ((y - 1) >> 1) - c;
  const int nr = ((y + 1) >> 1) - ((y - 1) >> 1) + 2 * c + 1;
  for (int idx = lane; idx < 3 * nr; idx += 64) {
    const int rr = idx / 3, cc = idx - 3 * rr;
    const int q = clampi(qbase + rr, 0, H - 1);
    const int X = clampi(x - 1 + cc, 0, oc.w - 1);
    const int e = X & 1, p = X >> 1, kmin = fold_kmin(e, r);
    const cdouble* fw = (const cdouble*)(P.wts + P.f0ofs[e][t]);
    const float* row = P.img + (long long)q * P.img_stride;
    double acc = 0.0;
    for (int j = 0; j <= r; ++j) acc = fma(fw[j], (double)row[clampi(p + kmin + j, 0, W - 1)], acc);
    sh[idx] = acc;
  }
  __syncthreads();
  if (lane < 9) {
    const int a3 = lane / 3, cc = lane - 3 * a3;
    const int Y = clampi(y - 1 + a3, 0, oc.h - 1);
    const int e = Y & 1, a = Y >> 1, kmin = fold_kmin(e, r);
    const cdouble* fw = (const cdouble*)(P.wts + P.f0ofs[e][t]);
    double acc = 0.0;
    // strip row a+k-qbase holds input row clamp(a+k), as k_gauss_o0 reads it
    for (int j = 0; j <= r; ++j) acc = fma(fw[j], sh[(a + kmin + j - qbase) * 3 + cc], acc);
    out[lane] = acc;
  }
  __syncthreads();
}

// L at rows y-1..y+1, cols x-1..x+1 of L-scale t -> out[9] (row-major).
// Requires blockDim.x == 64 (one wave): __syncthreads() is a wave barrier.
__device__ inline void wave_L_patch(const Pyramid& P, int o, int t, int y, int x, double* sh,
                                    double* out) {
  if (o == 0) {
    wave_L_patch_o0(P, t, y, x, sh, out);
    return;
  }
  const Octave& oc = P.oct[o];
  const int h = oc.h, w = oc.w, r = oc.rad[t];
  const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
  const int lane = threadIdx.x & 63;
  const int nr = 2 * r + 3;
  for (int idx = lane; idx < 3 * nr; idx += 64) {
    const int rr = idx / 3, cc = idx - 3 * rr;
    const int yy = clampi(y - 1 - r + rr, 0, h - 1);
    const int xb = x - 1 + cc - r;
    double acc = 0.0;
    for (int i = 0; i <= 2 * r; ++i) acc = fma(wp[i], base_at(P, o, yy, clampi(xb + i, 0, w - 1)), acc);
    sh[idx] = acc;
  }
  __syncthreads();
  if (lane < 9) {
    const int a = lane / 3, cc = lane - 3 * a;
    double acc = 0.0;
    for (int j = 0; j <= 2 * r; ++j) acc = fma(wp[j], sh[(a + j) * 3 + cc], acc);
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
