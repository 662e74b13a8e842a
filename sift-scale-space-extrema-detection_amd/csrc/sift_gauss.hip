// Gaussian scale space + Difference-of-Gaussians for one octave (gfx950).
//
// Replaces background.js:71-237 (computeGaussianScaleSpace, whose hot loop is
// SIFT_blurMatrix2DChunk, sift.js:72-149) and background.js:258-354
// (computeDifferenceOfGaussians / SIFT_subtractMatrix2DChunk, sift.js:154-188).
//
// The reference convolves every scale of an octave with a full 2D kernel of
// the SAME octave base (the blur is not incremental, background.js:173-177).
// The 2D kernel is exactly separable (w(i) w(j), sift.js:22-67), so each
// 64x32 output tile runs, per scale, a vertical pass over the base straight
// from global memory (L1/L2: the base is re-read by every scale of the tile)
// into an fp64 LDS strip of 32 x (64+2r) columns, then a horizontal pass out
// of that strip, 8 independent rows per thread.  The epilogue writes L_s
// (fp32), the DoG L_{s-1} - L_s formed in fp64 and rounded once (fp32), and
// for s == S the fp64 subsample that seeds the next octave
// (background.js:114-118).  Octave 0's base is the 2x nearest-neighbour
// upsample of the input (background.js:84), read as img[y>>1][x>>1] and
// never materialised.
//
// Every output pixel runs the same operation sequence on its clamped
// neighbourhood (translation invariant, like the reference's 2D sum), so
// pixels with identical neighbourhoods get bit-identical values and fp32
// ties mean the same thing as the reference's fp64 ties.
//
// Roofline: HBM-bound on the plane stores: per octave pixel 4(S+3) + 4(S+2)
// bytes written (+2 for the fp64 seed) against 1 (octave 0) or 8 bytes of
// base read.  fp64 VALU work per pixel and scale is 2(2r+1) FMAs (+ the
// 8-row window's 7 zero taps and the 2r-column halo of the vertical pass).
#include "sift_common.h"
#include "sift_kernels.h"

namespace sift {

template <bool OCT0>
__global__ __launch_bounds__(256) void k_gauss_dog(const Pyramid P, const GaussLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[L.o];
  const int h = oc.h, w = oc.w, R = oc.rmax;
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ty = wv * kVT;
  const int VW = kTX + 2 * R;  // strip row stride (columns x0-R .. x0+63+R)
  double* sV = smem;
  const float* __restrict__ img = P.img;
  const double* __restrict__ seed = P.seeds + oc.seed_off;
  const long long plane = (long long)h * w;
  const int x = x0 + lane;

  double lprev[kVT];
#pragma unroll
  for (int t = 0; t < kVT; ++t) lprev[t] = 0.0;

  for (int s = 0; s < P.NS; ++s) {
    const int r = oc.rad[s];
    // Taps through the constant address space: wave-uniform scalar loads.
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);

    // Vertical pass: V[y][c] = sum_j w_j B(clamp(y - r + j), clamp(x0 - r + c))
    // for this wave's 8 rows and columns c = 0 .. 63+2r, an 8-row register
    // sliding window per column (zero-padded taps keep each output's fma
    // sequence j = 0..2r).
    for (int cb = 0; cb < kTX + 2 * r; cb += 64) {
      const int c = cb + lane;
      const int xx = clampi(x0 - r + c, 0, w - 1);
      double acc[kVT];
#pragma unroll
      for (int t = 0; t < kVT; ++t) acc[t] = 0.0;
      const int yb = y0 + ty - r;
#pragma unroll 4
      for (int j = 0; j < 2 * r + kVT; ++j) {
        const int yy = clampi(yb + j, 0, h - 1);
        const double v = OCT0 ? (double)img[(long long)(yy >> 1) * P.img_stride + (xx >> 1)]
                              : seed[(long long)yy * w + xx];
#pragma unroll
        for (int t = 0; t < kVT; ++t) acc[t] = fma(wp[j - t], v, acc[t]);
      }
      if (c < kTX + 2 * r) {
#pragma unroll
        for (int t = 0; t < kVT; ++t) sV[(ty + t) * VW + c + (R - r)] = acc[t];
      }
    }
    __syncthreads();

    // Horizontal pass: L[y][x] = sum_i w_i V[y][x - r + i], 8 independent rows.
    double acc[kVT];
#pragma unroll
    for (int t = 0; t < kVT; ++t) acc[t] = 0.0;
    const double* row = sV + ty * VW + lane + (R - r);
#pragma unroll 2
    for (int i = 0; i <= 2 * r; ++i) {
      const double wi = wp[i];
#pragma unroll
      for (int t = 0; t < kVT; ++t) acc[t] = fma(wi, row[t * VW + i], acc[t]);
    }
    __syncthreads();  // the strip is rewritten by the next scale

    if (x < w) {
#pragma unroll
      for (int t = 0; t < kVT; ++t) {
        const int y = y0 + ty + t;
        if (y < h) {
          const long long p = (long long)y * w + x;
          if (L.gauss) L.gauss[s * plane + p] = (float)acc[t];
          if (s > 0) L.dog[(s - 1) * plane + p] = (float)(lprev[t] - acc[t]);
          if (s == P.S && L.next_seed && !(y & 1) && !(x & 1))
            L.next_seed[(long long)(y >> 1) * L.next_w + (x >> 1)] = acc[t];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < kVT; ++t) lprev[t] = acc[t];
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

size_t gauss_lds_bytes(const Octave& oc) {
  return sizeof(double) * (size_t)kTY * (kTX + 2 * oc.rmax);
}

hipError_t launch_gauss_dog(const Pyramid& P, const GaussLaunch& L, hipStream_t st) {
  const Octave& oc = P.oct[L.o];
  dim3 grid((oc.w + kTX - 1) / kTX, (oc.h + kTY - 1) / kTY);
  const size_t lds = gauss_lds_bytes(oc);
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void*)k_gauss_dog<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_gauss_dog<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  if (L.o == 0) hipLaunchKernelGGL(k_gauss_dog<true>, grid, dim3(256), lds, st, P, L);
  else hipLaunchKernelGGL(k_gauss_dog<false>, grid, dim3(256), lds, st, P, L);
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
