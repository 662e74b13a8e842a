// fp64 FMA issue probes for the Gaussian passes (gfx950).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/calib/fma_probe tools/calib/fma_probe.hip
// (a) NA independent fma chains per lane, taps in SGPRs: dependent-issue
//     latency and the waves per SIMD needed to fill the fp64 pipe;
// (b) the vertical pass's shape: 2 columns per lane, NO output rows, a
//     window of 2R + NO rows of 16-byte loads from an fp64 plane in L2 /
//     Infinity Cache, PF rows in flight; reports fma issue rate.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__device__ __forceinline__ void pin(double (&a)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i])::"memory");
}

template <int NA>
__global__ __launch_bounds__(256) void k_chain(double* out, const double* taps, int iters) {
  double a[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double t0 = taps[0], t1 = taps[1];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int i = 0; i < NA; ++i) a[i] = fma(t0, a[i], t1);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NA; ++i) s += a[i];
  if (s == 1.2345) out[threadIdx.x] = s;
}

// NA chains, each fma reading a second VGPR pair (the convolution's shape:
// acc = fma(tap_sgpr, value_vgpr, acc)); NB distinct values.
template <int NA, int NB>
__global__ __launch_bounds__(256) void k_chain2(double* out, const double* taps, int iters) {
  double a[NA], b[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) a[i] = threadIdx.x * 1e-3 + i;
#pragma unroll
  for (int i = 0; i < NB; ++i) b[i] = threadIdx.x * 1e-4 + 2 * i;
  const double t0 = taps[0];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int i = 0; i < NA; ++i) a[i] = fma(t0, b[(i + u) % NB], a[i]);
    }
    pin(b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NA; ++i) s += a[i];
  if (s == 1.2345) out[threadIdx.x] = s;
}
// the same with the multiplier in a VGPR too (three VGPR pairs per fma)
template <int NA, int NB>
__global__ __launch_bounds__(256) void k_chain3(double* out, const double* taps, int iters) {
  double a[NA], b[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) a[i] = threadIdx.x * 1e-3 + i;
#pragma unroll
  for (int i = 0; i < NB; ++i) b[i] = threadIdx.x * 1e-4 + 2 * i;
  double t0 = taps[0] + threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int i = 0; i < NA; ++i) a[i] = fma(t0, b[(i + u) % NB], a[i]);
    }
    pin(b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NA; ++i) s += a[i];
  if (s == 1.2345) out[threadIdx.x] = s;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// One wave = one 128-column x NO-row strip of one "scale": window rows
// y0 - R .. y0 + NO - 1 + R of the plane, repeated for `scales` strips
// (different row bands, so the loads are not L1 hits of the previous one).
template <int R, int NO, int PF>
__global__ __launch_bounds__(256) void k_vpass(const double* base, double* out, int h, int w, int scales) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nx = w / 128;
  const int tx = wv % nx, ty = wv / nx;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, h * w * 8, 0x00020000);
  const int xoff = (tx * 128 + 2 * lane) * 8;
  double tot = 0;
  constexpr int NJ = 2 * R + NO;
  constexpr int P = NJ < PF ? NJ : PF;
  for (int s = 0; s < scales; ++s) {
    int yy = __builtin_amdgcn_readfirstlane(((ty * scales + s) * NO) % (h - NJ));
    double a0[NO], a1[NO];
    double2 v[NJ];
#pragma unroll
    for (int t = 0; t < NO; ++t) a0[t] = a1[t] = 0.0;
    auto ld = [&]() -> double2 {
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, xoff, yy * w * 8, 0);
      asm volatile("" : "+s"(yy));
      yy += 1;
      return __builtin_bit_cast(double2, q);
    };
#pragma unroll
    for (int j = 0; j < P; ++j) v[j] = ld();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j + P < NJ) v[j + P] = ld();
#pragma unroll
      for (int t = 0; t < NO; ++t) {
        const int k = j - t;
        if (k >= 0 && k <= 2 * R) {
          const double wk = 0.01 * (k + 1);
          a0[t] = fma(wk, v[j].x, a0[t]);
          a1[t] = fma(wk, v[j].y, a1[t]);
        }
      }
      pin(a0);
      pin(a1);
    }
#pragma unroll
    for (int t = 0; t < NO; ++t) tot += a0[t] * a1[t];
  }
  if (tot == 1.2345) out[threadIdx.x] = tot;
}

// The same loop with the window rows read from LDS (a wave-private 128-column
// window of NJ rows staged once per scale): no L1/L2 traffic in the loop.
template <int R, int NO, int PF>
__global__ __launch_bounds__(256) void k_vpass_lds(double* out, int scales) {
  constexpr int NJ = 2 * R + NO;
  __shared__ double2 win[4][NJ][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int j = 0; j < NJ; ++j) win[wv][j][lane] = make_double2(lane * 1e-3 + j, j * 1e-3);
  __syncthreads();
  constexpr int P = NJ < PF ? NJ : PF;
  double tot = 0;
  for (int s = 0; s < scales; ++s) {
    double a0[NO], a1[NO];
    double2 v[NJ];
    int jj = 0;
    asm volatile("" : "+v"(jj));
#pragma unroll
    for (int t = 0; t < NO; ++t) a0[t] = a1[t] = 0.0;
#pragma unroll
    for (int j = 0; j < P; ++j) v[j] = win[wv][j + jj][lane];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j + P < NJ) v[j + P] = win[wv][j + P + jj][lane];
#pragma unroll
      for (int t = 0; t < NO; ++t) {
        const int k = j - t;
        if (k >= 0 && k <= 2 * R) {
          const double wk = 0.01 * (k + 1);
          a0[t] = fma(wk, v[j].x, a0[t]);
          a1[t] = fma(wk, v[j].y, a1[t]);
        }
      }
      pin(a0);
      pin(a1);
    }
#pragma unroll
    for (int t = 0; t < NO; ++t) tot += a0[t] * a1[t];
  }
  if (tot == 1.2345) out[threadIdx.x] = tot;
}

int main() {
  double *b, *out, *taps;
  const int h = 2160, w = 3840;  // an octave-1 base: 66 MB fp64
  if (hipMalloc(&b, (size_t)h * w * 8) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  hipMemset(b, 0, (size_t)h * w * 8);
  hipMalloc(&taps, 64);
  double ht[2] = {0.999999, 1e-7};
  hipMemcpy(taps, ht, 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, int a1, int a2, auto f, double fmas) {
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int it = 5;
    for (int i = 0; i < it; ++i) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    // fraction of the 78.6 TFLOP/s fp64 vector peak (39.3 T fma/s)
    printf("%-28s %4d %4d %8.3f ms  %6.1f Tfma/s  %.3f of peak\n", name, a1, a2, ms, fmas / ms / 1e9,
           fmas / ms / 1e9 / 39.3);
  };
  const int iters = 256;
  for (int wps : {1, 2, 4}) {
    const int blocks = 256 * wps;
#define CH(NA)                                                                                        \
  run("chain acc (sgpr operands)", NA, wps, [&] { k_chain<NA><<<blocks, 256>>>(out, taps, iters); },  \
      (double)NA * 16 * iters * blocks * 256.0);
#define CH2(NA, NB)                                                                                   \
  run("chain2 acc (vgpr value)", NA * 100 + NB, wps, [&] { k_chain2<NA, NB><<<blocks, 256>>>(out, taps, iters); }, \
      (double)NA * 16 * iters * blocks * 256.0);
#define CH3(NA, NB)                                                                                   \
  run("chain3 acc (vgpr tap+value)", NA * 100 + NB, wps, [&] { k_chain3<NA, NB><<<blocks, 256>>>(out, taps, iters); }, \
      (double)NA * 16 * iters * blocks * 256.0);
    CH(8) CH(16) CH2(8, 8) CH2(8, 16) CH2(16, 8) CH3(8, 8) CH3(16, 8)
#undef CH
#undef CH2
#undef CH3
  }
  return 0;
}
