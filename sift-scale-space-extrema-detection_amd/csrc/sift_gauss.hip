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

// Octave 0, folded.  The octave-0 base is the 2x nearest-neighbour upsample
// of the input (background.js:84), so B[y][x] = I[y>>1][x>>1] and clamping
// commutes with the halving.  The horizontal sum depends on y only through
// q = y>>1, and both passes fold their 2r+1 taps onto r+1 input pixels with
// parity-dependent weights (sift_common.h, f0ofs): per output pixel and
// scale about (r+1)/2 + (r+4) FMAs instead of 2(2r+1), and the tile stages
// only the fp32 input region.  Same outputs as k_gauss_dog otherwise.
__global__ __launch_bounds__(256) void k_gauss_o0(const Pyramid P, const GaussLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Octave& oc = P.oct[0];
  const int h = oc.h, w = oc.w, H = P.H, W = P.W;
  const int cR = fold_half(oc.rmax);
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY;
  const int p0 = x0 >> 1, a0 = y0 >> 1;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  // Input region: rows qlo_all..qhi_all (distinct, clamped), columns
  // p0-cR .. p0+31+cR with replicated edges, as fp64.
  const int qlo_all = max(0, a0 - cR), qhi_all = min(H - 1, a0 + kTY / 2 - 1 + cR);
  const int IW = kTX / 2 + 2 * cR;
  double* sI = smem;
  double* sQ = smem + (size_t)(qhi_all - qlo_all + 1) * IW;
  {
    const float* __restrict__ img = P.img;
    const int n = (qhi_all - qlo_all + 1) * IW;
    for (int idx = tid; idx < n; idx += 256) {
      const int rr = idx / IW, cc = idx - rr * IW;
      sI[idx] = (double)img[(long long)(qlo_all + rr) * P.img_stride + clampi(p0 - cR + cc, 0, W - 1)];
    }
  }
  __syncthreads();

  const long long plane = (long long)h * w;
  const int x = x0 + lane;
  const int A = a0 + (wv * kVT) / 2;  // first input row of this wave's 8 output rows
  double lprev[kVT];
#pragma unroll
  for (int t = 0; t < kVT; ++t) lprev[t] = 0.0;

  for (int s = 0; s < P.NS; ++s) {
    const int r = oc.rad[s], c = fold_half(r);
    const int kmin0 = fold_kmin(0, r), kmin1 = fold_kmin(1, r);
    const cdouble* f0 = (const cdouble*)(P.wts + P.f0ofs[0][s]);
    const cdouble* f1 = (const cdouble*)(P.wts + P.f0ofs[1][s]);
    const int qlo = max(0, a0 - c), qhi = min(H - 1, a0 + kTY / 2 - 1 + c);
    const int nq = qhi - qlo + 1;

    // Horizontal: hq[q][2p+e] = sum_j fw_e[j] I[q][clamp(p + kmin_e + j)].
    // A unit is (row pair, parity): lanes 0-31 take row 2*pi, 32-63 row
    // 2*pi+1, column pair p = lane & 31; units u and u+4 share a parity, so
    // taps stay wave-uniform and two rows accumulate independently.
    {
      const int p = lane & 31, half = lane >> 5;
      const int units = ((nq + 1) >> 1) * 2;
      for (int u = wv; u < units; u += 8) {
        const int e = u & 1;
        const cdouble* fw = e ? f1 : f0;
        const int kmin = e ? kmin1 : kmin0;
        const int qa = qlo + 2 * (u >> 1) + half;
        const int u2 = u + 4;
        const bool has2 = u2 < units;
        const int qb = qlo + 2 * (u2 >> 1) + half;
        const int qa_c = min(qa, qhi), qb_c = min(qb, qhi);
        const double* ra = sI + (size_t)(qa_c - qlo_all) * IW + p + kmin + cR;
        const double* rb = sI + (size_t)(qb_c - qlo_all) * IW + p + kmin + cR;
        double a = 0.0, b = 0.0;
        for (int j = 0; j <= r; ++j) {
          const double fj = fw[j];
          a = fma(fj, ra[j], a);
          b = fma(fj, rb[j], b);
        }
        if (qa <= qhi) sQ[(qa - qlo) * kTX + 2 * p + e] = a;
        if (has2 && qb <= qhi) sQ[(qb - qlo) * kTX + 2 * p + e] = b;
      }
    }
    __syncthreads();

    // Vertical: L[2a+e][x] = sum_k fw_e[k] hq[clamp(a+k)][x] for a = A+m,
    // m = 0..3; strip row j holds input row clamp(A - c + j).  Zero-padded
    // taps keep each output's fma sequence k = kmin_e .. kmax_e.
    double acc[kVT];
#pragma unroll
    for (int t = 0; t < kVT; ++t) acc[t] = 0.0;
    for (int j = 0; j < 2 * c + 4; ++j) {
      const int qq = clampi(A - c + j, 0, H - 1) - qlo;
      const double v = sQ[qq * kTX + lane];
#pragma unroll
      for (int m = 0; m < kVT / 2; ++m) {
        const int k = j - c - m;
        acc[2 * m] = fma(f0[k - kmin0], v, acc[2 * m]);
        acc[2 * m + 1] = fma(f1[k - kmin1], v, acc[2 * m + 1]);
      }
    }
    __syncthreads();

    if (x < w) {
#pragma unroll
      for (int t = 0; t < kVT; ++t) {
        const int y = y0 + wv * kVT + t;
        if (y < h) {
          const long long pp = (long long)y * w + x;
          if (L.gauss) L.gauss[s * plane + pp] = (float)acc[t];
          if (s > 0) L.dog[(s - 1) * plane + pp] = (float)(lprev[t] - acc[t]);
          if (s == P.S && L.next_seed && !(y & 1) && !(x & 1))
            L.next_seed[(long long)(y >> 1) * L.next_w + (x >> 1)] = acc[t];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < kVT; ++t) lprev[t] = acc[t];
  }
}

size_t gauss_o0_lds_bytes(const Pyramid& P) {
  const int cR = fold_half(P.oct[0].rmax);
  const int rows = std::min(P.H, kTY / 2 + 2 * cR);
  return sizeof(double) * (size_t)rows * ((kTX / 2 + 2 * cR) + kTX);
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
    (void)hipFuncSetAttribute((const void*)k_gauss_o0, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const bool o0 = L.o == 0;
  if (o0 && !L.unfolded) {
    hipLaunchKernelGGL(k_gauss_o0, grid, dim3(256), gauss_o0_lds_bytes(P), st, P, L);
    return hipGetLastError();
  }
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
