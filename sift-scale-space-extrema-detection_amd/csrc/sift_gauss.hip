// Gaussian scale space + Difference-of-Gaussians for one octave (gfx950).
//
// Replaces background.js:71-237 (computeGaussianScaleSpace, whose hot loop is
// SIFT_blurMatrix2DChunk, sift.js:72-149) and background.js:258-354
// (computeDifferenceOfGaussians / SIFT_subtractMatrix2DChunk, sift.js:154-188).
//
// The reference convolves every scale of an octave with a full 2D kernel of
// the SAME octave base (the blur is not incremental, background.js:173-177).
// Here each 64x32 output tile stages that base once (replicated-edge region
// in LDS, fp64), then for every scale runs the separable form of the same
// kernel -- a horizontal pass into an fp64 LDS strip and a vertical pass with
// an 8-row register sliding window -- and writes L_s (fp32), the DoG
// L_{s-1} - L_s formed in fp64 and rounded once (fp32), and for s == S the
// fp64 subsample that seeds the next octave (background.js:114-118).
//
// Roofline: HBM-bound on the plane stores.  Per octave pixel the kernel
// writes 4(S+3) + 4(S+2) bytes (+8/4 for the seed) and reads 1 (octave 0:
// 4 bytes per 4 pixels) or 8/4 bytes of base.  fp64 VALU work per pixel is
// sum_s 2(2r_s+1) FMAs; it overlaps the store stream.
#include "sift_common.h"
#include "sift_kernels.h"

namespace sift {

template <bool BASE_LDS, bool OCT0>
__global__ __launch_bounds__(256) void k_gauss_dog(const Pyramid P, const GaussLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[L.o];
  const int h = oc.h, w = oc.w, R = oc.rmax;
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ty = wv * kVT;

  // Rows this tile can touch, clamped: the strip only holds distinct rows.
  const int lo_all = max(0, y0 - R), hi_all = min(h - 1, y0 + kTY - 1 + R);
  const int BW = kTX + 2 * R;
  double* sH = smem;
  double* sB = smem + (size_t)(hi_all - lo_all + 1) * kTX;
  const float* __restrict__ img = P.img;
  const double* __restrict__ seed = P.seeds + oc.seed_off;
  auto base = [&](int y, int x) -> double {  // y, x already clamped
    if (OCT0) return (double)img[(long long)(y >> 1) * P.img_stride + (x >> 1)];
    return seed[(long long)y * w + x];
  };

  if (BASE_LDS) {
    // Replicated-edge base region: rows lo_all..hi_all, columns x0-R ..
    // x0+kTX+R-1 with clamped sources.
    const int nr = hi_all - lo_all + 1;
    for (int idx = tid; idx < nr * BW; idx += 256) {
      const int rr = idx / BW, cc = idx - rr * BW;
      sB[idx] = base(lo_all + rr, clampi(x0 - R + cc, 0, w - 1));
    }
    __syncthreads();
  }

  const long long plane = (long long)h * w;
  const int x = x0 + lane;
  double lprev[kVT];
#pragma unroll
  for (int t = 0; t < kVT; ++t) lprev[t] = 0.0;

  for (int s = 0; s < P.NS; ++s) {
    const int r = oc.rad[s];
    // Taps through the constant address space: wave-uniform scalar loads.
    const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[s]);
    const int lo = max(0, y0 - r), hi = min(h - 1, y0 + kTY - 1 + r);
    const int nrows = hi - lo + 1;

    // Horizontal pass: sH[y - lo][c] = sum_i w_i * B(y, clamp(x0 + c - r + i)),
    // four independent rows per thread (wave rows wv*4 .. +3 of each group of 16).
    for (int rb = wv * 4; rb < nrows; rb += 16) {
      const int r0 = rb, r1 = min(rb + 1, nrows - 1), r2 = min(rb + 2, nrows - 1), r3 = min(rb + 3, nrows - 1);
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if (BASE_LDS) {
        const int cb = lane + R - r;
        const double* p0 = sB + (size_t)(lo + r0 - lo_all) * BW + cb;
        const double* p1 = sB + (size_t)(lo + r1 - lo_all) * BW + cb;
        const double* p2 = sB + (size_t)(lo + r2 - lo_all) * BW + cb;
        const double* p3 = sB + (size_t)(lo + r3 - lo_all) * BW + cb;
#pragma unroll 2
        for (int i = 0; i <= 2 * r; ++i) {
          const double wi = wp[i];
          a0 = fma(wi, p0[i], a0);
          a1 = fma(wi, p1[i], a1);
          a2 = fma(wi, p2[i], a2);
          a3 = fma(wi, p3[i], a3);
        }
      } else {
        const int xb = x0 + lane - r;
        for (int i = 0; i <= 2 * r; ++i) {
          const double wi = wp[i];
          const int xx = clampi(xb + i, 0, w - 1);
          a0 = fma(wi, base(lo + r0, xx), a0);
          a1 = fma(wi, base(lo + r1, xx), a1);
          a2 = fma(wi, base(lo + r2, xx), a2);
          a3 = fma(wi, base(lo + r3, xx), a3);
        }
      }
      sH[r0 * kTX + lane] = a0;
      if (rb + 1 < nrows) sH[r1 * kTX + lane] = a1;
      if (rb + 2 < nrows) sH[r2 * kTX + lane] = a2;
      if (rb + 3 < nrows) sH[r3 * kTX + lane] = a3;
    }
    __syncthreads();

    // Vertical pass, 8 outputs per thread: output row y0+ty+t reads strip
    // rows clamp(y0+ty+t-r+k), k = 0..2r.  Zero-padded taps keep the fma
    // sequence identical to a plain k = 0..2r sum for every t.
    double acc[kVT];
#pragma unroll
    for (int t = 0; t < kVT; ++t) acc[t] = 0.0;
    for (int j = 0; j < 2 * r + kVT; ++j) {
      const int yy = clampi(y0 + ty - r + j, 0, h - 1) - lo;
      const double v = sH[yy * kTX + lane];
#pragma unroll
      for (int t = 0; t < kVT; ++t) acc[t] = fma(wp[j - t], v, acc[t]);
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

size_t gauss_lds_bytes(const Octave& oc, bool base_lds) {
  const int R = oc.rmax;
  const int rows = std::min(oc.h, kTY + 2 * R);
  size_t b = (size_t)rows * kTX * sizeof(double);
  if (base_lds) b += (size_t)rows * (kTX + 2 * R) * sizeof(double);
  return b;
}

template <bool BL, bool O0>
static void set_lds_attr() {
  (void)hipFuncSetAttribute((const void*)k_gauss_dog<BL, O0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_gauss_dog(const Pyramid& P, const GaussLaunch& L, hipStream_t st) {
  const Octave& oc = P.oct[L.o];
  dim3 grid((oc.w + kTX - 1) / kTX, (oc.h + kTY - 1) / kTY);
  const size_t lds = gauss_lds_bytes(oc, L.base_lds);
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    set_lds_attr<true, true>();
    set_lds_attr<true, false>();
    set_lds_attr<false, true>();
    set_lds_attr<false, false>();
    attr_set = true;
  }
  const bool o0 = L.o == 0;
  if (L.base_lds && o0) hipLaunchKernelGGL((k_gauss_dog<true, true>), grid, dim3(256), lds, st, P, L);
  else if (L.base_lds) hipLaunchKernelGGL((k_gauss_dog<true, false>), grid, dim3(256), lds, st, P, L);
  else if (o0) hipLaunchKernelGGL((k_gauss_dog<false, true>), grid, dim3(256), lds, st, P, L);
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
