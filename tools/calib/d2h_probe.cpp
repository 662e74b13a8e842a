// Device -> host copy rates into the kinds of host memory a caller hands
// sift_get_plane (JS: a fresh Float32Array), to place the stage chain's
// plane reads: fresh pageable pages (first touch faults), touched pageable,
// huge-page advised, pinned; and the staged path (pinned chunks + threaded
// memcpy).  usage: d2h_probe [MB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

static void par_copy(char* d, const char* s, size_t n, int nt) {
  std::vector<std::thread> th;
  size_t per = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    size_t a = std::min(n, t * per), b = std::min(n, (t + 1) * per);
    if (a < b) th.emplace_back([=] { std::memcpy(d + a, s + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoi(argv[1]) : 512;
  const size_t n = mb << 20;
  void* dsrc;
  CK(hipMalloc(&dsrc, n));
  CK(hipMemset(dsrc, 1, n));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto rate = [&](const char* what, double t) { std::printf("%-58s %8.2f GB/s  (%.1f ms)\n", what, n / t / 1e9, t * 1e3); };
  // 1. fresh pageable (malloc -> mmap, untouched)
  for (int rep = 0; rep < 2; ++rep) {
    char* h = (char*)std::malloc(n);
    double t0 = now();
    CK(hipMemcpyAsync(h, dsrc, n, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    rate("hipMemcpy D2H -> fresh pageable", now() - t0);
    t0 = now();
    CK(hipMemcpyAsync(h, dsrc, n, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    rate("hipMemcpy D2H -> touched pageable", now() - t0);
    std::free(h);
  }
  // 2. first-touch cost alone
  {
    char* h = (char*)std::malloc(n);
    double t0 = now();
    std::memset(h, 0, n);
    rate("memset fresh pageable (1 thread: page faults + zeroing)", now() - t0);
    std::free(h);
    h = (char*)std::malloc(n);
    t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t) th.emplace_back([=] { std::memset(h + t * (n / 8), 0, n / 8); });
    for (auto& x : th) x.join();
    rate("memset fresh pageable (8 threads)", now() - t0);
    std::free(h);
    void* p = nullptr;
    if (posix_memalign(&p, 2 << 20, n) == 0) {
      madvise(p, n, MADV_HUGEPAGE);
      t0 = now();
      std::memset(p, 0, n);
      rate("memset fresh MADV_HUGEPAGE (1 thread)", now() - t0);
      std::free(p);
    }
  }
  // 3. pinned
  {
    void* h;
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    for (int rep = 0; rep < 2; ++rep) {
      double t0 = now();
      CK(hipMemcpyAsync(h, dsrc, n, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      rate("hipMemcpy D2H -> pinned", now() - t0);
    }
    // 4. staged: pinned -> pageable, threads
    for (int nt : {1, 4, 8, 16}) {
      char* h2 = (char*)std::malloc(n);
      double t0 = now();
      par_copy(h2, (char*)h, n, nt);
      char name[96];
      std::snprintf(name, sizeof name, "memcpy pinned -> fresh pageable, %d threads", nt);
      rate(name, now() - t0);
      t0 = now();
      par_copy(h2, (char*)h, n, nt);
      std::snprintf(name, sizeof name, "memcpy pinned -> touched pageable, %d threads", nt);
      rate(name, now() - t0);
      std::free(h2);
    }
    CK(hipHostFree(h));
  }
  std::printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
  return 0;
}
