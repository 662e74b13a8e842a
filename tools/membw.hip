// Store-bandwidth probes for the Gaussian kernel's write pattern (gfx950).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/membw tools/membw.hip
// (a) linear float4 stream, (b) TXxTY tiles x NP planes (the k_gauss_dog
// epilogue pattern, no compute), (c) linear copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_write_lin(float4* p, long long n4) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
    p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ void k_copy_lin(const float4* a, float4* b, long long n4) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) b[i] = a[i];
}

// one block per TX x 32 tile; lane -> 4 columns; NP planes written in turn
template <int TX>
__global__ void k_write_tiles(float* p, int h, int w, int np, int spin) {
  constexpr int CG = TX / 4, RS = 256 / CG, NR = 32 / RS;
  const int x0 = blockIdx.x * TX, y0 = blockIdx.y * 32;
  const int cg = threadIdx.x % CG, rs = threadIdx.x / CG;
  const long long plane = (long long)h * w;
  float acc = threadIdx.x;
  for (int s = 0; s < np; ++s) {
    for (int k = 0; k < spin; ++k) acc = acc * 1.0001f + 0.5f;
    for (int i = 0; i < NR; ++i) {
      const int y = y0 + rs + RS * i, x = x0 + 4 * cg;
      if (y < h && x < w)
        *reinterpret_cast<float4*>(p + s * plane + (long long)y * w + x) = make_float4(acc, acc, acc, acc);
    }
  }
}

// fp64 FMA throughput: NA independent accumulators per lane, tap from an SGPR.
template <int NA>
__global__ void k_fma64(double* out, const double* taps, int iters) {
  double a[NA];
  for (int i = 0; i < NA; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double t0 = taps[0], t1 = taps[1];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NA; ++i) a[i] = fma(t0, a[i], t1);
  }
  double s = 0;
  for (int i = 0; i < NA; ++i) s += a[i];
  if (s == 1.2345) out[threadIdx.x] = s;
}

int main() {
  const int h = 4320, w = 7680, np = 15;
  const long long n = (long long)h * w * np;
  float *a, *b;
  if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, int arg, auto f, double bytes) {
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int it = 10;
    for (int i = 0; i < it; ++i) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("%-34s %6d %8.3f ms  %7.1f GB/s\n", name, arg, ms, bytes / ms / 1e6);
  };
  for (int g : {1024, 2048, 4096, 8192, 16384})
    run("write linear, grid", g, [&] { k_write_lin<<<g, 256>>>((float4*)a, n / 4); }, n * 4.0);
  run("copy linear, grid", 8192, [&] { k_copy_lin<<<8192, 256>>>((const float4*)a, (float4*)b, n / 8); }, n * 4.0);
  for (int spin : {0, 64, 256}) {
    run("tiles 64x32 x15 planes, spin", spin,
        [&] { k_write_tiles<64><<<dim3(w / 64, h / 32), 256>>>(a, h, w, np, spin); }, n * 4.0);
    run("tiles 128x32 x15 planes, spin", spin,
        [&] { k_write_tiles<128><<<dim3(w / 128, h / 32), 256>>>(a, h, w, np, spin); }, n * 4.0);
    run("tiles 256x32 x15 planes, spin", spin,
        [&] { k_write_tiles<256><<<dim3(w / 256, h / 32), 256>>>(a, h, w, np, spin); }, n * 4.0);
  }
  double* taps;
  hipMalloc(&taps, 64);
  double ht[2] = {0.999999, 1e-7};
  hipMemcpy(taps, ht, 16, hipMemcpyHostToDevice);
  const int iters = 4096;
  for (int wpc : {4, 8, 16}) {
    const int blocks = 256 * wpc / 4;
    const double flops = 2.0 * 8 * iters * blocks * 256.0;
    run("fp64 fma 8 acc, waves/CU", wpc, [&] { k_fma64<8><<<blocks, 256>>>((double*)b, taps, iters); }, flops / 1e3);
  }
  for (int wpc : {4, 8, 16}) {
    const int blocks = 256 * wpc / 4;
    const double flops = 2.0 * 4 * iters * blocks * 256.0;
    run("fp64 fma 4 acc, waves/CU", wpc, [&] { k_fma64<4><<<blocks, 256>>>((double*)b, taps, iters); }, flops / 1e3);
  }
  printf("(fp64 rows: the GB/s column is GFLOP/s / 1000 = TFLOP/s)\n");
  return 0;
}
