// Does v_mfma_f64_16x16x4_f64 accumulate like a chain of fp64 fmas?
//
// The Gaussian vertical pass is V[y] = sum_k w_k B[y - r + k], an fma chain
// in increasing k from 0.0 (the order every plane is pinned to).  As a
// band-Toeplitz product on the matrix cores, each MFMA adds 4 taps to the
// accumulator.  The planes stay bit-identical only if D = A B + C is
// evaluated as fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, c)))) per
// element.  This probe compares the MFMA against that chain (and against the
// reverse chain and a plain rounded-product sum) over random inputs chained
// through many MFMAs, counting bit mismatches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib/mfma_f64_probe tools/calib/mfma_f64_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double double4_t __attribute__((ext_vector_type(4)));

// One wave: NSTEP chained MFMAs; A[16][4], B[4][16] per step, C the running D.
// Layout (MI355X_MICROARCH.md): A lane l -> A[l % 16][l / 16]; B lane l ->
// B[l / 16][l % 16]; C/D reg q of lane l -> D[(l >> 4) + 4 q][l & 15].
__global__ void k_probe(const double* A, const double* B, int nstep, double* d_mfma, double* d_fwd,
                        double* d_rev, double* d_sum) {
  const int l = threadIdx.x;
  double4_t acc = {0.0, 0.0, 0.0, 0.0};
  double fwd[4] = {0, 0, 0, 0}, rev[4] = {0, 0, 0, 0}, sum[4] = {0, 0, 0, 0};
  const int col = l & 15;
  for (int t = 0; t < nstep; ++t) {
    const double* At = A + t * 64;  // [16][4] row-major
    const double* Bt = B + t * 64;  // [4][16] row-major
    const double a = At[(l % 16) * 4 + l / 16];
    const double b = Bt[(l / 16) * 16 + l % 16];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (l >> 4) + 4 * q;
      double f = fwd[q], r = rev[q];
      for (int k = 0; k < 4; ++k) f = fma(At[row * 4 + k], Bt[k * 16 + col], f);
      for (int k = 3; k >= 0; --k) r = fma(At[row * 4 + k], Bt[k * 16 + col], r);
      double p = 0.0;
      for (int k = 0; k < 4; ++k) p += At[row * 4 + k] * Bt[k * 16 + col];
      fwd[q] = f;
      rev[q] = r;
      sum[q] = sum[q] + p;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = ((l >> 4) + 4 * q) * 16 + col;
    d_mfma[idx] = acc[q];
    d_fwd[idx] = fwd[q];
    d_rev[idx] = rev[q];
    d_sum[idx] = sum[q];
  }
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 200, nstep = argc > 2 ? atoi(argv[2]) : 24;
  srand(12345);
  double *A, *B, *o[4];
  hipMalloc(&A, 64 * nstep * sizeof(double));
  hipMalloc(&B, 64 * nstep * sizeof(double));
  for (int i = 0; i < 4; ++i) hipMalloc(&o[i], 256 * sizeof(double));
  std::vector<double> ha(64 * nstep), hb(64 * nstep), h[4];
  for (int i = 0; i < 4; ++i) h[i].resize(256);
  long long n = 0, mis_fwd = 0, mis_rev = 0, mis_sum = 0;
  for (int t = 0; t < trials; ++t) {
    // taps in (0, 1) like normalised Gaussian weights, values like fp64 plane data in [0, 1]
    for (auto& v : ha) v = (double)rand() / RAND_MAX * (t & 1 ? 0.25 : 1.0);
    for (auto& v : hb) v = (double)rand() / RAND_MAX;
    hipMemcpy(A, ha.data(), ha.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(B, hb.data(), hb.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, A, B, nstep, o[0], o[1], o[2], o[3]);
    for (int i = 0; i < 4; ++i) hipMemcpy(h[i].data(), o[i], 256 * 8, hipMemcpyDeviceToHost);
    for (int e = 0; e < 256; ++e, ++n) {
      mis_fwd += h[0][e] != h[1][e];
      mis_rev += h[0][e] != h[2][e];
      mis_sum += h[0][e] != h[3][e];
    }
  }
  printf("v_mfma_f64_16x16x4_f64, %d chained MFMAs, %lld outputs: mismatches vs fma chain k=0..3: %lld, "
         "vs k=3..0: %lld, vs c + rounded products: %lld\n", nstep, n, mis_fwd, mis_rev, mis_sum);
  printf("%s\n", mis_fwd == 0 ? "MFMA == increasing-k fma chain (bit-exact)" : "MFMA differs from the increasing-k fma chain");
  return 0;
}
