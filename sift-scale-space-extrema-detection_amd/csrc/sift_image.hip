// Image products either side of the hot path (gfx950), SURVEY.md §8f rows 2-3.
//
// k_rgba_to_gray: ImageUtils_convertImageDataToMatrix2D with
//   convertToGrayscale / usePerceptualGrayscale (image-utils.js:27-152, as
//   main.js:98-103 calls it): gray = ((R*0.299) + (G*0.587) + (B*0.114)) / 255
//   and alpha = A / 255, in fp64 with the reference's operation order
//   (contraction off), rounded once into the ImageData-shaped Float32 gray
//   the path consumes.  Four pixels per lane: one 16-byte RGBA load, one
//   16-byte gray store (8 B/px of HBM traffic, 12 with alpha).
//
// k_plane_image: the preview ImageData the reference posts for every plane,
//   ImageUtils_convertMatrix2DToImageData(grayChannelMatrix) (image-utils.js:
//   171-217): p = Math.round(g*255) written as (p, p, p, 255) into a
//   Uint8ClampedArray (ToUint8Clamp: NaN and negatives -> 0, >255 -> 255), of
//     SIFT_DISPLAY_PLAIN    g = v                     Gaussian planes (background.js:139, :218)
//     SIFT_DISPLAY_SIGMOID  g = 1/(1+exp(c*(-1*v)))   Matrix2D_sigmoidNormalize (matrix2d.js:151),
//                                                     DoG chunks with c = 5 (background.js:303)
//     SIFT_DISPLAY_SAMPLED  g = (v-min)/(max-min)     Matrix2D_sampledNormalize (matrix2d.js:169),
//                                                     DoG images (background.js:336, :387)
//   All in fp64 from the fp32 plane values.  The plane min/max of the
//   sampled mode is a two-level reduction: k_minmax_partial writes one
//   (min, max) per block, every block of k_plane_image folds the partials
//   (<= 1024 pairs, L2-resident) before its pixels.
#include "sift_kernels.h"

#pragma clang fp contract(off)

namespace sift {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double js_round_d(double v) {
  const double f = floor(v);
  return (v - f >= 0.5) ? f + 1.0 : f;
}

__device__ __forceinline__ float gray_of(unsigned px) {
  const double r = (double)(px & 0xffu), g = (double)((px >> 8) & 0xffu), b = (double)((px >> 16) & 0xffu);
  const double v = (r * 0.299) + (g * 0.587) + (b * 0.114);  // image-utils.js:107
  return (float)(v / 255.0);                                 // image-utils.js:114
}

__device__ __forceinline__ float alpha_of(unsigned px) { return (float)((double)(px >> 24) / 255.0); }

// ToUint8Clamp of Math.round(g * 255) (image-utils.js:205, typed-array store).
__device__ __forceinline__ unsigned clamp_u8(double g) {
  const double p = js_round_d(g * 255.0);
  if (!(p > 0.0)) return 0u;  // NaN, -0, negatives
  if (p >= 255.0) return 255u;
  return (unsigned)p;
}

__device__ __forceinline__ unsigned rgba_of(unsigned p) { return p | (p << 8) | (p << 16) | 0xff000000u; }

// One lane per 4 pixels of a row; q = quad index within the row.
__global__ void __launch_bounds__(256) k_rgba_to_gray(const unsigned char* __restrict__ rgba, size_t stride_bytes,
                                                      int w, int h, int quads, float* __restrict__ gray,
                                                      float* __restrict__ alpha) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)quads * h) return;
  const int y = (int)(i / quads);
  const int x0 = (int)(i - (long long)y * quads) * 4;
  const unsigned char* row = rgba + (size_t)y * stride_bytes;
  float* grow = gray + (size_t)y * w;
  float* arow = alpha ? alpha + (size_t)y * w : nullptr;
  if (x0 + 4 <= w && ((((size_t)row) | ((size_t)grow)) & 15) == 0) {
    const uint4 px = *reinterpret_cast<const uint4*>(row + (size_t)x0 * 4);
    const f32x4 g = {gray_of(px.x), gray_of(px.y), gray_of(px.z), gray_of(px.w)};
    __builtin_nontemporal_store(g, reinterpret_cast<f32x4*>(grow + x0));
    if (arow) {
      if ((((size_t)arow) & 15) == 0) {
        float4 a;
        a.x = alpha_of(px.x);
        a.y = alpha_of(px.y);
        a.z = alpha_of(px.z);
        a.w = alpha_of(px.w);
        *reinterpret_cast<float4*>(arow + x0) = a;
      } else {
        arow[x0] = alpha_of(px.x);
        arow[x0 + 1] = alpha_of(px.y);
        arow[x0 + 2] = alpha_of(px.z);
        arow[x0 + 3] = alpha_of(px.w);
      }
    }
    return;
  }
  for (int x = x0; x < w && x < x0 + 4; ++x) {  // ragged tail or unaligned rows
    const unsigned px = *reinterpret_cast<const unsigned*>(row + (size_t)x * 4);
    grow[x] = gray_of(px);
    if (arow) arow[x] = alpha_of(px);
  }
}

constexpr int kMMThreads = 256;

__device__ __forceinline__ void wave_minmax(float& mn, float& mx) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, d, 64));
    mx = fmaxf(mx, __shfl_xor(mx, d, 64));
  }
}

// Block (min, max) of the block's share of the plane.  NaNs never win, as in
// the reference's `value < min` / `value > max` scan (matrix2d.js:176-186).
__global__ void __launch_bounds__(kMMThreads) k_minmax_partial(const float* __restrict__ v, long long n, int vec,
                                                               float2* __restrict__ part) {
  __shared__ float smn[kMMThreads / 64], smx[kMMThreads / 64];
  float mn = __builtin_inff(), mx = -__builtin_inff();
  const long long stride = (long long)gridDim.x * kMMThreads;
  long long i = (long long)blockIdx.x * kMMThreads + threadIdx.x;
  const long long n4 = vec ? n / 4 : 0;
  const float4* v4 = reinterpret_cast<const float4*>(v);
  for (long long k = i; k < n4; k += stride) {
    const float4 a = v4[k];
    mn = fminf(mn, fminf(fminf(a.x, a.y), fminf(a.z, a.w)));
    mx = fmaxf(mx, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
  }
  for (long long k = n4 * 4 + i; k < n; k += stride) {
    mn = fminf(mn, v[k]);
    mx = fmaxf(mx, v[k]);
  }
  wave_minmax(mn, mx);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[wv] = mn;
    smx[wv] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kMMThreads / 64; ++k) {
      mn = fminf(mn, smn[k]);
      mx = fmaxf(mx, smx[k]);
    }
    part[blockIdx.x] = make_float2(mn, mx);
  }
}

// One lane per 4 pixels of the plane (rows are contiguous: the plane is one
// w*h run).  mode: SIFT_DISPLAY_* (include/sift_hip.h).
__global__ void __launch_bounds__(256) k_plane_image(const float* __restrict__ v, long long n, int vec, int mode, double c,
                                                     const float2* __restrict__ part, int nparts,
                                                     unsigned* __restrict__ out) {
  double mn = 0.0, range = 1.0;
  if (mode == 2) {
    __shared__ float s_mn, s_mx;
    if (threadIdx.x < 64) {
      float a = __builtin_inff(), b = -__builtin_inff();
      for (int k = threadIdx.x; k < nparts; k += 64) {
        const float2 p = part[k];
        a = fminf(a, p.x);
        b = fmaxf(b, p.y);
      }
      wave_minmax(a, b);
      if (threadIdx.x == 0) {
        s_mn = a;
        s_mx = b;
      }
    }
    __syncthreads();
    mn = (double)s_mn;
    range = (double)s_mx - mn;  // matrix2d.js:192: (v - min) / (max - min)
  }
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long x0 = q * 4;
  if (x0 >= n) return;
  unsigned px[4];
  float vv[4];
  const bool full = vec && x0 + 4 <= n;
  if (full) {
    const float4 a = reinterpret_cast<const float4*>(v)[q];
    vv[0] = a.x;
    vv[1] = a.y;
    vv[2] = a.z;
    vv[3] = a.w;
  } else {
    for (int k = 0; k < 4; ++k) vv[k] = x0 + k < n ? v[x0 + k] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double x = (double)vv[k];
    double g;
    if (mode == 1)
      g = 1.0 / (1.0 + exp(c * (-1.0 * x)));  // matrix2d.js:156
    else if (mode == 2)
      g = (x - mn) / range;
    else
      g = x;
    px[k] = rgba_of(clamp_u8(g));
  }
  if (full) {
    const u32x4 o4 = {px[0], px[1], px[2], px[3]};
    __builtin_nontemporal_store(o4, reinterpret_cast<u32x4*>(out) + q);
  } else {
    for (int k = 0; k < 4 && x0 + k < n; ++k) out[x0 + k] = px[k];
  }
}

}  // namespace

hipError_t launch_rgba_to_gray(const unsigned char* rgba, size_t stride_bytes, int w, int h, float* gray,
                               float* alpha, hipStream_t st) {
  const int quads = (w + 3) / 4;
  const long long lanes = (long long)quads * h;
  if (lanes == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((lanes + 255) / 256);
  hipLaunchKernelGGL(k_rgba_to_gray, dim3(blocks), dim3(256), 0, st, rgba, stride_bytes, w, h, quads, gray, alpha);
  return hipGetLastError();
}

int plane_image_parts(long long n) {
  const long long want = (n / 4 + kMMThreads * 8 - 1) / (kMMThreads * 8);  // >= 8 float4 per lane
  return (int)std::max(1LL, std::min(1024LL, want));
}

hipError_t launch_plane_image(const float* plane, long long n, int mode, double coefficient, float2* parts,
                              unsigned* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const int vin = (((size_t)plane) & 15) == 0;
  const int vec = vin && (((size_t)out) & 15) == 0;
  int nparts = 0;
  if (mode == 2) {
    nparts = plane_image_parts(n);
    hipLaunchKernelGGL(k_minmax_partial, dim3(nparts), dim3(kMMThreads), 0, st, plane, n, vin, parts);
  }
  const long long lanes = (n + 3) / 4;
  hipLaunchKernelGGL(k_plane_image, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, plane, n, vec, mode,
                     coefficient, (const float2*)parts, nparts, out);
  return hipGetLastError();
}

}  // namespace sift
