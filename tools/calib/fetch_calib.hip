// FETCH_SIZE calibration on gfx950 for the access widths this path uses
// (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B-per-lane
// streaming reads).  Each kernel reads a known number of bytes from a 1 GiB
// buffer (far beyond the 256 MiB Infinity Cache) once; rocprofv3 --pmc
// FETCH_SIZE over this program gives the counter's bytes per kernel:
//   k_stream<1|2|4>  coalesced streaming reads of 4 / 8 / 16 B per lane
//   k_gather_line    one 4-B read per 128-B line (every lane a different line)
//   k_gather_row3    three consecutive floats per lane at random rows (the
//                    refinement's patch-row reads)
// usage: fetch_calib  (prints the algorithmic bytes of each kernel)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;

template <int W>
__global__ void k_stream(const unsigned* __restrict__ src, size_t n_vec, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_vec; i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (W == 1) acc ^= src[i];
    if constexpr (W == 2) { const uint2 v = reinterpret_cast<const uint2*>(src)[i]; acc ^= v.x ^ v.y; }
    if constexpr (W == 4) { const uint4 v = reinterpret_cast<const uint4*>(src)[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__device__ __forceinline__ size_t hash_line(size_t i, size_t n_lines) {
  return (i * 2654435761ull + 12345) % n_lines;
}

__global__ void k_gather_line(const unsigned* __restrict__ src, size_t n, size_t n_lines, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[hash_line(i, n_lines) * 32];
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ void k_gather_row3(const float* __restrict__ src, size_t n, size_t n_rows, int w, float* __restrict__ out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = hash_line(i, n_rows);
    const float* p = src + r * w + (i * 37) % (w - 3);
    acc += p[0] + p[1] + p[2];
  }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  unsigned* buf;
  unsigned* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(buf, 1, kBytes);
  hipDeviceSynchronize();
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream<1>, dim3(grid), dim3(block), 0, 0, buf, kBytes / 4, out);
    hipLaunchKernelGGL(k_stream<2>, dim3(grid), dim3(block), 0, 0, buf, kBytes / 8, out);
    hipLaunchKernelGGL(k_stream<4>, dim3(grid), dim3(block), 0, 0, buf, kBytes / 16, out);
    const size_t n_lines = kBytes / 128, n_g = size_t(1) << 22;  // 4 Mi distinct-line reads
    hipLaunchKernelGGL(k_gather_line, dim3(grid), dim3(block), 0, 0, buf, n_g, n_lines, out);
    const int w = 15360;  // a 4K octave-0 row (floats)
    hipLaunchKernelGGL(k_gather_row3, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const float*>(buf), n_g,
                       kBytes / 4 / w - 1, w, reinterpret_cast<float*>(out));
  }
  hipDeviceSynchronize();
  std::printf("k_stream<1> k_stream<2> k_stream<4>: %zu bytes each\n", kBytes);
  std::printf("k_gather_line: %zu reads of 4 B, one per 128-B line (%zu B of lines)\n", size_t(1) << 22,
              (size_t(1) << 22) * 128);
  std::printf("k_gather_row3: %zu reads of 12 B at random rows (%zu B of 128-B lines if each hits 1 line)\n",
              size_t(1) << 22, (size_t(1) << 22) * 128);
  return 0;
}
