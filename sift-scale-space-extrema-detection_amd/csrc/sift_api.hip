// C ABI of libsift_hip.so (include/sift_hip.h): context, schedule, stage
// orchestration on one HIP stream.  The stage functions mirror the
// reference's worker stages (background.js:71 / :258 / :359 / :455).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/sift_hip.h"
#include "sift_kernels.h"

using namespace sift;

namespace {

// Grow-only device buffer.
struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t need) {
    if (need <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    size_t want = need + need / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Grow-only pinned host buffer (staging of host images and keypoint records).
struct HBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t need) {
    if (need <= bytes) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    size_t want = need + need / 4 + 256;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// Row copy between host buffers on up to `nt` threads (host memory bandwidth
// of one core is well below what the DMA engines take from pinned memory).
void par_copy_rows(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows, int nt) {
  auto part = [&](size_t r0, size_t r1) {
    for (size_t r = r0; r < r1; ++r)
      std::memcpy((char*)dst + r * dpitch, (const char*)src + r * spitch, width);
  };
  if (nt <= 1 || rows * width < ((size_t)4 << 20)) {
    part(0, rows);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (rows + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) {
    const size_t r0 = std::min(rows, t * per), r1 = std::min(rows, (t + 1) * per);
    if (r0 < r1) th.emplace_back(part, r0, r1);
  }
  part(0, std::min(rows, per));
  for (auto& x : th) x.join();
}

// Host rows -> pinned staging -> device, pipelined: each of nt host threads
// copies its share of the rows in ~2 MiB pieces and queues each piece's DMA on
// `st` as soon as it is staged (disjoint ranges: their order does not matter;
// the caller's later launches on `st` follow every piece).
hipError_t h2d_rows_staged(void* dev, void* stage, const void* src, size_t spitch, size_t width, size_t rows, int nt,
                           hipStream_t st) {
  std::atomic<int> err{0};
  auto part = [&](size_t r0, size_t r1) {
    const size_t piece = std::max<size_t>(1, ((size_t)2 << 20) / width);
    for (size_t a = r0; a < r1; a += piece) {
      const size_t b = std::min(r1, a + piece);
      for (size_t r = a; r < b; ++r) std::memcpy((char*)stage + r * width, (const char*)src + r * spitch, width);
      if (hipMemcpyAsync((char*)dev + a * width, (const char*)stage + a * width, (b - a) * width,
                         hipMemcpyHostToDevice, st) != hipSuccess)
        err = 1;
    }
  };
  if (nt <= 1 || rows * width < ((size_t)4 << 20)) {
    part(0, rows);
  } else {
    std::vector<std::thread> th;
    const size_t per = (rows + nt - 1) / nt;
    for (int t = 1; t < nt; ++t) {
      const size_t r0 = std::min(rows, t * per), r1 = std::min(rows, (t + 1) * per);
      if (r0 < r1) th.emplace_back(part, r0, r1);
    }
    part(0, std::min(rows, per));
    for (auto& x : th) x.join();
  }
  return err ? hipErrorUnknown : hipSuccess;
}

// Host threads of the library's own copies (image staging, keypoint split,
// plane read-back): min(4, cores); SIFT_HOST_THREADS=n in experiments builds
// (1, 2 and 4 measured under the N-API pool: 4 is best).
int host_threads() {
  static const int n = [] {
    const int v = exp_knob("SIFT_HOST_THREADS", 0);
    if (v >= 1 && v <= 64) return v;
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(4u, h ? h : 1u));
  }();
  return n;
}

double js_round(double x) {
  double f = std::floor(x);
  return (x - f >= 0.5) ? f + 1.0 : f;
}

enum DogSource { kNone = 0, kNative = 1, kForeign = 2 };

// Device counter slots: 0..31 extrema / refinement counts (see below), then
// the kept keypoints per (octave, scale) block from kBlk on.
constexpr int kBlk = 64;
constexpr int kCntAll = kBlk + kBlkWords;  // per-block counts, block starts, order flag (sift_kernels.h)

}  // namespace

struct sift_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;          // false: the stream of another context (sift_ctx_create_shared)
  std::string err;
  sift_params p{};
  int W = 0, H = 0;
  std::vector<int> dims;           // 2*O
  std::vector<double> blur, sigma; // O*NS
  Pyramid P{};
  int dog_source = kNone;
  bool have_gauss = false;
  bool have_cand = false;
  size_t n_cand = 0, n_low = 0, n_kp = 0, n_sing = 0, n_exact = 0;
  size_t n_slots = 0;       // candidate slots (n_cand + entries dropped by the exact pass)
  bool want_low = false;    // this extrema stage lists the low-contrast extrema
  bool have_low = false;    // the last extrema stage did (sift_copy_low_contrast)
  unsigned low_cap = 0;     // slots of the ordered low-contrast list
  size_t n_low_sure = 0, n_low_late = 0;  // ordered (certain) and exact-pass (late) low-contrast entries
  unsigned cand_cap = 0;    // capacity of the candidate slot arrays (extrema path)
  unsigned amb_cap = 0;     // capacity of the ambiguous-key list
  int slot_cap = 0;         // slots the refinement runs over
  bool ext_pending = false; // extrema launched, counts not yet read back
  bool has_keep = false;    // slots carry keep flags
  bool slots_rows = false;  // slots are the extrema stage's emission (row offsets in rowoff): band order applies
  bool counters_zeroed = false;  // extrema_prepare zeroed the refinement counters too
  bool detect_pending = false;   // sift_detect_device_async enqueued, sift_detect_wait not yet called
  bool begin_pending = false;    // sift_detect_begin_async enqueued, sift_detect_end_async not yet called
  bool detect_host_img = false;
  ExtremaLaunch xl{};       // extrema launch state between prepare / scan / finish
  int o_first = 0;          // first octave of the pyramid in use (sift_detect_from_seed: > 0)
  int scan_first = 0;       // first octave the extrema stage scans (>= o_first; sift_detect_from_seed_range)
  int planes_first = 0;     // first octave with Gaussian / DoG planes (below: only its successor's base)
  int row0 = 0;             // sift_set_row_origin: input row of the image's first row
  int xseed_h = 0, xseed_w = 0;  // SIFT_F_EXPORT_NEXT_SEED: the base of octave O
  bool has_xseed = false;
  bool has_origins = false; // kp_key holds the candidate key of every keypoint
  std::vector<long long> x_word_off, x_row_off;
  std::vector<int> x_nw, x_ww, x_woff;  // bitmap words per row, columns per word, column of bit 0
  long long x_rows = 0;
  int x_nf = 0;             // leading octaves whose extrema decisions run fused into the Gaussian pass
  bool x_prepared = false;  // extrema_prepare already ran for this detection (fused octaves)
  // device memory
  DBuf img, seeds, gauss, dog, wts;
  DBuf base0;                                  // materialised octave-0 base (large radii only)
  DBuf l64;                                    // fp64 Gaussian planes of the large-radius octaves
  DBuf vsplit;                                 // vertical-sum scratch of the split-pass octaves (one at a time)
  DBuf seedv;                                  // vertical sums of the seed-only octaves (launch_seed_only)
  long long vsplit_pi = 0;                     // ... doubles per image of a batch
  std::vector<double> wts_host;                // taps last uploaded to wts
  // Taps of the deepest schedule built so far (setup_geometry): per-(octave,
  // scale) sigma, the padded tap vector, its length after each octave, and
  // every scale's radius and tap offset.  Sigma does not depend on the octave
  // count, so a schedule whose sigmas are a prefix of these reuses a prefix
  // of the taps instead of ~3 K exp() per call (8K O6 S5: ~35 us).
  struct TapCache {
    int NS = 0;
    std::vector<double> sigma, w;
    std::vector<size_t> oct_end;
    std::vector<int> rad, wofs;
  } taps;
  DBuf bitmap, rowcount, rowoff, amb_keys;     // extrema scan
  DBuf ambbitmap;                              // ambiguous words (k_exact_words)
  bool x_words = false;                        // this extrema stage lists ambiguous words, not keys
  DBuf cand_key, cand_val, cand_keep;          // ordered candidates
  DBuf patch, wslot, cand_patch;               // first-step patches captured by the scan (ExtremaLaunch.patch)
  DBuf pre;                                    // the scan's first refinement steps (ExtremaLaunch.pre, SIFT_XREFINE)
  bool x_patch = false;                        // this extrema stage captures patches
  bool has_patch = false;                      // cand_patch indexes the current slots
  DBuf lowbitmap, lowrowcount, lowrowoff;      // low-contrast list (SIFT_F_LOW_CONTRAST_LIST)
  DBuf low_key, low_val, late_key, late_val;
  DBuf keep, pos;                              // keypoint compaction
  DBuf keep_tile;                              // ... its per-tile counts (launch_keep_compact)
  DBuf band_cnt, band_first, band_start, perm;  // refinement band order
  DBuf status, kp_tmp, kp, uncertain;          // refinement
  DBuf kp_soa;                                 // keypoint field arrays for a DMA into registered host arrays
  DBuf xseed, kp_key;                          // next-octave base, keypoint origins
  DBuf merge_tab;                              // sift_merge_keypoint_blocks_device tables
  DBuf counters, temp;
  DBuf rgba, alpha, display, mm_parts;         // image products (sift_image.hip)
  unsigned* h_counters = nullptr;              // pinned mirror of counters (+ per-block keypoint counts at kBlk)
  int own_lo = -1, own_hi = -1;                // sift_set_owned_rows
  std::vector<long long> blk_counts;           // kept keypoints per (octave, scale) of the last refinement
  HBuf himg, hkp;                  // pinned staging: host images in, keypoint records out
  hipEvent_t ev_himg = nullptr;    // the DMA out of himg is done (himg may be refilled)
  HBuf hpl;                        // pinned staging of plane reads: two halves, double-buffered
  hipEvent_t ev_pl[2] = {nullptr, nullptr};
  hipEvent_t ev[8]{};
  hipEvent_t ev_heavy = nullptr;  // after the last bandwidth-heavy kernel of a detection (sift_order_after)
  hipEvent_t ev_go[kMaxOctaves]{}; // after octave o's Gaussian+DoG launch (per-octave timings)
  sift_timings tm{};
  std::vector<double> oct_ms;      // per-octave Gaussian+DoG launch time of the last build
  std::vector<std::string> pass_kn; // per-octave pass kernels of the last build (sift_last_pass_kernels)
};

#define HIPCHK(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);                         \
      return SIFT_E_HIP;                                                                    \
    }                                                                                       \
  } while (0)

static int set_err(sift_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

static int check_params(const sift_params* p) {
  if (!p) return SIFT_E_ARG;
  if (p->num_octaves < 1 || p->num_octaves > kMaxOctaves) return SIFT_E_UNSUPPORTED;
  if (p->scales_per_octave < 1 || p->scales_per_octave + 3 > kMaxScales) return SIFT_E_UNSUPPORTED;
  if (!(p->min_blur > 0) || !(p->assumed_blur >= 0) || !(p->min_interpixel_distance > 0)) return SIFT_E_ARG;
  return SIFT_OK;
}

// Device -> pageable host copy through pinned staging: chunks alternate
// between the two halves of ctx->hpl, so the DMA of chunk i+1 overlaps the
// (multi-threaded) host copy of chunk i.  A plain hipMemcpy into pageable
// memory runs at a fraction of the link rate; this keeps the link busy.
// Host ranges page-locked through sift_host_register: the runtime DMAs into
// them directly; anything else is treated as pageable.  Tracked here rather
// than probed with hipPointerGetAttributes, whose failure on pageable memory
// would have to be cleared with hipGetLastError -- and that would also
// swallow an earlier asynchronous error still pending on the thread.
static std::mutex g_reg_mu;
static std::map<uintptr_t, size_t> g_reg_ranges;  // start -> bytes

static bool host_registered(const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg_ranges.upper_bound(a);
  if (it == g_reg_ranges.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

static hipError_t d2h_staged(sift_ctx* ctx, void* dst, const void* src, size_t bytes) {
  constexpr size_t kChunk = (size_t)8 << 20;
  if (bytes < ((size_t)1 << 20) || host_registered(dst, bytes)) {  // small or page-locked: one DMA straight into it
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
  }
  hipError_t e = ctx->hpl.ensure(2 * kChunk);
  for (int i = 0; i < 2 && e == hipSuccess; ++i)
    if (!ctx->ev_pl[i]) e = hipEventCreateWithFlags(&ctx->ev_pl[i], hipEventDisableTiming);
  if (e != hipSuccess) return e;
  char* half[2] = {(char*)ctx->hpl.p, (char*)ctx->hpl.p + kChunk};
  const size_t n = (bytes + kChunk - 1) / kChunk;
  auto len = [&](size_t i) { return std::min(kChunk, bytes - i * kChunk); };
  auto issue = [&](size_t i) {
    hipError_t r = hipMemcpyAsync(half[i & 1], (const char*)src + i * kChunk, len(i), hipMemcpyDeviceToHost,
                                  ctx->stream);
    return r != hipSuccess ? r : hipEventRecord(ctx->ev_pl[i & 1], ctx->stream);
  };
  for (size_t i = 0; i < std::min<size_t>(n, 2) && e == hipSuccess; ++i) e = issue(i);
  for (size_t i = 0; i < n && e == hipSuccess; ++i) {
    e = hipEventSynchronize(ctx->ev_pl[i & 1]);
    if (e != hipSuccess) break;
    const size_t piece = 256 << 10, l = len(i), rows = l / piece;  // 256 KB rows split over the threads
    par_copy_rows((char*)dst + i * kChunk, piece, half[i & 1], piece, piece, rows, host_threads());
    if (l > rows * piece) std::memcpy((char*)dst + i * kChunk + rows * piece, half[i & 1] + rows * piece, l - rows * piece);
    if (i + 2 < n) e = issue(i + 2);
  }
  if (e != hipSuccess) (void)hipStreamSynchronize(ctx->stream);  // nothing left writing into hpl
  return e;
}

extern "C" {

int sift_abi_version(void) { return SIFT_ABI_VERSION; }

int sift_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return SIFT_E_ARG;
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) return SIFT_E_HIP;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  g_reg_ranges[reinterpret_cast<uintptr_t>(p)] = bytes;
  return SIFT_OK;
}

int sift_host_unregister(void* p) {
  if (!p) return SIFT_E_ARG;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg_ranges.erase(reinterpret_cast<uintptr_t>(p));
  }
  return hipHostUnregister(p) == hipSuccess ? SIFT_OK : SIFT_E_HIP;
}

int sift_params_default(sift_params* p) {
  if (!p) return SIFT_E_ARG;
  p->num_octaves = 5;         // worker.js:33
  p->scales_per_octave = 3;   // worker.js:34
  p->min_blur = 0.8;          // worker.js:35
  p->assumed_blur = 0.5;      // worker.js:36
  p->min_interpixel_distance = 0.5;  // worker.js:88
  p->flags = 0;
  return SIFT_OK;
}

int sift_octave_dims(int width, int height, int num_octaves, int* dims) {
  if (width < 1 || height < 1 || num_octaves < 1 || !dims) return SIFT_E_ARG;
  int h = 2 * height, w = 2 * width;  // background.js:84 (2x upsample)
  for (int o = 0; o < num_octaves; ++o) {
    if (o > 0) { h = (h + 1) / 2; w = (w + 1) / 2; }  // background.js:118
    dims[2 * o] = h;
    dims[2 * o + 1] = w;
  }
  return SIFT_OK;
}

int sift_schedule(const sift_params* p, double* blur, double* sigma) {
  int rc = check_params(p);
  if (rc) return rc;
  if (!blur || !sigma) return SIFT_E_ARG;
  // background.js:89-177
  const int S = p->scales_per_octave, NS = S + 3;
  const double k = std::pow(2.0, 1.0 / S);
  double base_blur = p->min_blur;
  for (int o = 0; o < p->num_octaves; ++o) {
    for (int s = 0; s < NS; ++s) {
      if (o > 0 && s == 0) {
        base_blur = blur[(o - 1) * NS + S];
        blur[o * NS] = base_blur;
        sigma[o * NS] = 0.0;
      } else {
        const double target = base_blur * std::pow(k, (double)s);
        const double from = o == 0 ? p->assumed_blur : base_blur;
        blur[o * NS + s] = target;
        sigma[o * NS + s] = std::sqrt((target * target) - (from * from));
      }
    }
  }
  return SIFT_OK;
}

static int ctx_create(int device, sift_ctx* share, sift_ctx** out) {
  if (!out) return SIFT_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return SIFT_E_HIP;
  if (device < 0 || device >= n) return SIFT_E_ARG;
  sift_ctx* ctx = new sift_ctx();
  ctx->device = device;
  ctx->own_stream = share == nullptr;
  if (hipSetDevice(device) != hipSuccess ||
      (share ? (ctx->stream = share->stream, false)
             : hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) ||
      hipHostMalloc((void**)&ctx->h_counters, kCntAll * sizeof(unsigned), hipHostMallocDefault) != hipSuccess ||
      ctx->counters.ensure(kCntAll * sizeof(unsigned)) != hipSuccess) {
    delete ctx;
    return SIFT_E_HIP;
  }
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  for (auto& e : ctx->ev_go) (void)hipEventCreate(&e);
  (void)hipEventCreateWithFlags(&ctx->ev_heavy, hipEventDisableTiming);
  *out = ctx;
  return SIFT_OK;
}

int sift_ctx_create(int device, sift_ctx** out) { return ctx_create(device, nullptr, out); }

int sift_ctx_create_shared(sift_ctx* share, sift_ctx** out) {
  if (!share || !out) return SIFT_E_ARG;
  return ctx_create(share->device, share, out);
}

int sift_ctx_destroy(sift_ctx* ctx) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  DBuf* bufs[] = {&ctx->ambbitmap, &ctx->img, &ctx->seeds, &ctx->base0, &ctx->l64, &ctx->vsplit, &ctx->gauss, &ctx->dog, &ctx->wts, &ctx->bitmap,
                  &ctx->rowcount, &ctx->rowoff, &ctx->amb_keys, &ctx->keep, &ctx->pos,
                  &ctx->cand_keep, &ctx->cand_key, &ctx->cand_val, &ctx->status,
                  &ctx->kp_tmp, &ctx->kp, &ctx->uncertain, &ctx->xseed, &ctx->kp_key, &ctx->counters,
                  &ctx->temp, &ctx->rgba, &ctx->alpha, &ctx->display, &ctx->mm_parts, &ctx->merge_tab,
                  &ctx->lowbitmap, &ctx->lowrowcount, &ctx->lowrowoff, &ctx->low_key, &ctx->low_val,
                  &ctx->late_key, &ctx->late_val, &ctx->band_cnt, &ctx->band_first, &ctx->band_start,
                  &ctx->perm, &ctx->patch, &ctx->wslot, &ctx->cand_patch, &ctx->pre, &ctx->kp_soa, &ctx->keep_tile};
  for (DBuf* b : bufs) b->release();
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->ev_go)
    if (e) (void)hipEventDestroy(e);
  if (ctx->ev_heavy) (void)hipEventDestroy(ctx->ev_heavy);
  ctx->himg.release();
  ctx->hkp.release();
  if (ctx->ev_himg) (void)hipEventDestroy(ctx->ev_himg);
  ctx->hpl.release();
  for (auto& e : ctx->ev_pl)
    if (e) (void)hipEventDestroy(e);
  if (ctx->h_counters) (void)hipHostFree(ctx->h_counters);
  ctx->seedv.release();
  if (ctx->stream && ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return SIFT_OK;
}

const char* sift_last_error(sift_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* sift_stream(sift_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int sift_synchronize(sift_ctx* ctx) {
  if (!ctx) return SIFT_E_ARG;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Geometry, schedule and weights (host), background.js:71-177 + sift.js:31-67.
// ---------------------------------------------------------------------------
static int setup_geometry(sift_ctx* ctx, int W, int H, const sift_params* p, const double* sig_in,
                          bool need_weights) {
  int rc = check_params(p);
  if (rc) return set_err(ctx, rc, "invalid or unsupported parameters");
  if (W < 1 || H < 1) return set_err(ctx, SIFT_E_ARG, "empty image");
  const int O = p->num_octaves, S = p->scales_per_octave, NS = S + 3, ND = S + 2;
  ctx->p = *p;
  ctx->scan_first = 0;
  ctx->planes_first = 0;
  ctx->has_patch = false;
  ctx->P.vsum = nullptr;
  ctx->P.vsum_oct = -1;
  ctx->W = W;
  ctx->H = H;
  ctx->dims.assign(2 * O, 0);
  sift_octave_dims(W, H, O, ctx->dims.data());
  ctx->blur.assign(O * NS, 0.0);
  ctx->sigma.assign(O * NS, 0.0);
  sift_schedule(p, ctx->blur.data(), ctx->sigma.data());
  if (sig_in) {
    for (int i = 0; i < O * NS; ++i) ctx->sigma[i] = sig_in[i];
  }
  Pyramid& P = ctx->P;
  std::memset(&P, 0, sizeof(P));
  P.O = O; P.S = S; P.NS = NS; P.ND = ND;
  P.W = W; P.H = H;
  const double thr = ((std::pow(2.0, 1.0 / S) - 1) / (std::pow(2.0, 1.0 / 3) - 1)) * 0.015;
  P.thr = thr;             // background.js:572
  P.row0 = ctx->row0;
  P.pix_thr = thr * 0.8;   // sift.js:285-294
  std::vector<double> w;
  long long goff = 0, doff = 0, soff = 0;
  unsigned long long koff = 0;
  sift_ctx::TapCache& tc = ctx->taps;
  const bool taps_hit = need_weights && tc.NS == NS && tc.sigma.size() >= (size_t)O * NS &&
                        std::equal(ctx->sigma.begin(), ctx->sigma.end(), tc.sigma.begin());
  if (taps_hit) w.assign(tc.w.begin(), tc.w.begin() + (std::ptrdiff_t)tc.oct_end[O - 1]);
  std::vector<size_t> oct_end;
  for (int o = 0; o < O; ++o) {
    Octave& oc = P.oct[o];
    oc.h = ctx->dims[2 * o];
    oc.w = ctx->dims[2 * o + 1];
    const long long plane = (long long)oc.h * oc.w;
    oc.gauss_off = goff;
    oc.dog_off = doff;
    oc.seed_off = o > 0 ? soff : 0;
    if (o > 0) soff += plane;
    if (koff > 0xffffffffull) return set_err(ctx, SIFT_E_UNSUPPORTED, "image too large for 32-bit keys");
    oc.key_off = (unsigned)koff;
    koff += (unsigned long long)S * plane;
    goff += NS * plane;
    doff += ND * plane;
    oc.rmax = 0;
    oc.l64_off = -1;
    if (taps_hit) {
      for (int s = 0; s < NS; ++s) {
        oc.rad[s] = tc.rad[o * NS + s];
        oc.wofs[s] = tc.wofs[o * NS + s];
        oc.rmax = std::max(oc.rmax, oc.rad[s]);
      }
      continue;
    }
    for (int s = 0; s < NS; ++s) {
      const double sg = ctx->sigma[o * NS + s];
      int r = 0;
      for (int z = 0; z < kWPad; ++z) w.push_back(0.0);
      oc.wofs[s] = (int)w.size();
      if (o > 0 && s == 0) {
        w.push_back(1.0);  // the un-blurred seed: exact copy
      } else {
        // sift.js:38-44: r = Math.round(3 sigma); the 2D kernel
        // exp(((i^2+j^2)/s^2)*-0.5)/(2 pi s^2) / sum factors as w(i) w(j)
        // with w(i) = exp((i^2/s^2)*-0.5) / sum_i exp(...).
        r = (int)js_round(3.0 * sg);
        std::vector<double> g(2 * r + 1);
        double sum = 0.0;
        for (int i = 0; i <= 2 * r; ++i) {
          const double a = i - r;
          g[i] = std::exp(((a * a) / (sg * sg)) * -0.5);
          sum += g[i];
        }
        for (int i = 0; i <= 2 * r; ++i) w.push_back(g[i] / sum);
      }
      for (int z = 0; z < kWPad; ++z) w.push_back(0.0);
      oc.rad[s] = r;
      oc.rmax = std::max(oc.rmax, r);
    }
    oct_end.push_back(w.size());
  }
  if (koff > 0xffffffffull) return set_err(ctx, SIFT_E_UNSUPPORTED, "image too large for 32-bit keys");
  if (need_weights && !taps_hit && (tc.NS != NS || O * NS >= (int)tc.sigma.size())) {
    // a miss at this depth or deeper replaces the cache; a shallower miss
    // (another schedule) leaves a deeper one in place
    tc.NS = NS;
    tc.sigma = ctx->sigma;
    tc.w = w;
    tc.oct_end = oct_end;
    tc.rad.assign((size_t)O * NS, 0);
    tc.wofs.assign((size_t)O * NS, 0);
    for (int o = 0; o < O; ++o)
      for (int s = 0; s < NS; ++s) {
        tc.rad[o * NS + s] = P.oct[o].rad[s];
        tc.wofs[o * NS + s] = P.oct[o].wofs[s];
      }
  }
  P.nimg = 1;  // one image (build_common sets a batch)
  P.kpi = (unsigned)koff;
  // LDS feasibility of the Gaussian kernel (two strips of 32 rows x (76 + 2R) fp64).
  for (int o = 0; o < O; ++o)
    if (gauss_lds_bytes(P, o) > 160 * 1024)
      return set_err(ctx, SIFT_E_UNSUPPORTED, "blur radius too large for one LDS strip");
  if (need_weights) {
    // Upload only when the taps changed (the same schedule image after image).
    // The taps are laid out octave after octave, so a schedule with fewer
    // octaves is a prefix of a deeper one: a context that alternates row bands
    // (octaves 0..K) and tail pieces (octaves 0..t) keeps the deepest taps
    // and uploads (a blocking copy) only when a deeper schedule arrives.
    const bool prefix = w.size() <= ctx->wts_host.size() &&
                        std::equal(w.begin(), w.end(), ctx->wts_host.begin());
    if (!prefix || !ctx->wts.p) {
      if (ctx->wts.ensure(w.size() * sizeof(double)) != hipSuccess)
        return set_err(ctx, SIFT_E_HIP, "hipMalloc weights");
      if (hipMemcpy(ctx->wts.p, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
        return set_err(ctx, SIFT_E_HIP, "upload weights");
      ctx->wts_host = w;
    }
    P.wts = ctx->wts.as<double>();
  }
  (void)soff;
  return SIFT_OK;
}

static long long total_plane_px(const sift_ctx* ctx) {
  long long t = 0;
  for (int o = 0; o < ctx->P.O; ++o) t += (long long)ctx->P.oct[o].h * ctx->P.oct[o].w;
  return t;
}

static int extrema_prepare(sift_ctx* ctx, hipStream_t st, int nf = 0);
static int extrema_scan(sift_ctx* ctx, int o0, int o1, hipStream_t st);

// Fused extrema decisions (k_gauss_dog, XF): SIFT_F_FUSED_EXTREMA, or
// SIFT_FUSE=1 for every detection (experiments).
static bool fuse_enabled(const sift_params* p) {
  static const bool env = exp_knob("SIFT_FUSE", 0) != 0;
  return env || (p->flags & SIFT_F_FUSED_EXTREMA);
}

// o_first > 0 (sift_detect_from_seed): no image; the fp64 base of octave
// o_first is seed_host / seed_dev and octaves o_first .. O-1 are built.
// fuse_extrema: a detection -- octave 0's extrema decisions run inside its
// Gaussian+DoG launch (the extrema stage then scans octaves >= 1 only).
// nimg > 1: a batch of nimg device images of one geometry, image b at
// img_dev + b * img_bstride (sift_detect_batch_device): one launch per stage
// over all of them, planes and seeds image-major.
static int build_common(sift_ctx* ctx, const float* img_host, const float* img_dev, int W, int H,
                        size_t stride, const sift_params* p, const double* sig,
                        int o_first = 0, const double* seed_host = nullptr, const double* seed_dev = nullptr,
                        bool fuse_extrema = false, int nimg = 1, size_t img_bstride = 0, int seed_only_below = 0) {
  if (!ctx) return SIFT_E_ARG;
  if (o_first == 0 && !img_host && !img_dev) return set_err(ctx, SIFT_E_ARG, "null image");
  if (o_first > 0 && !seed_host && !seed_dev) return set_err(ctx, SIFT_E_ARG, "null seed");
  if (o_first == 0 && stride < (size_t)W) return set_err(ctx, SIFT_E_ARG, "stride < width");
  HIPCHK(hipSetDevice(ctx->device));
  int rc = setup_geometry(ctx, W, H, p, sig, true);
  if (rc) return rc;
  Pyramid& P = ctx->P;
  if (o_first < 0 || o_first >= P.O) return set_err(ctx, SIFT_E_ARG, "octave_first out of range");
  ctx->o_first = o_first;
  ctx->scan_first = o_first;
  // Octaves [o_first, so_end) only feed their successor's base (a range
  // detection scans from so_end): launch_seed_only, no planes.
  const int so_end = std::min(std::max(o_first, seed_only_below), P.O - 1);
  if (so_end > o_first && (nimg > 1 || fuse_extrema))
    return set_err(ctx, SIFT_E_UNSUPPORTED, "seed-only octaves: single image, no fused decisions");
  ctx->planes_first = so_end;
  ctx->has_xseed = false;
  const long long tot = total_plane_px(ctx);
  const bool keep_gauss = !(p->flags & SIFT_F_SKIP_GAUSS_PLANES);
  if (nimg > 1) {
    if (o_first != 0 || (!img_host && !img_dev) || fuse_extrema || gauss_needs_base0(P) || ctx->row0 != 0 ||
        ctx->own_lo >= 0 ||
        (p->flags & (SIFT_F_EXPORT_NEXT_SEED | SIFT_F_LOW_CONTRAST_LIST | SIFT_F_FUSED_EXTREMA |
                     SIFT_F_KEYPOINT_ORIGINS)))  // origins carry no image index
      return set_err(ctx, SIFT_E_UNSUPPORTED, "batch: whole device images, plain detection only");
    if ((unsigned long long)P.kpi * (unsigned long long)nimg > 0xffffffffull ||
        (long long)nimg * P.O * P.S > kBlkN)
      return set_err(ctx, SIFT_E_UNSUPPORTED, "batch too large for 32-bit keys / block counts");
  }
  const long long seeds_pi = std::max<long long>(1, tot - (long long)P.oct[0].h * P.oct[0].w);
  P.nimg = nimg;
  P.img_bstride = nimg > 1 ? (long long)img_bstride : 0;
  P.seed_bstride = seeds_pi;
  P.dog_bstride = tot * P.ND;
  HIPCHK(ctx->dog.ensure((size_t)tot * P.ND * nimg * sizeof(float)));
  if (keep_gauss) HIPCHK(ctx->gauss.ensure((size_t)tot * P.NS * nimg * sizeof(float)));
  HIPCHK(ctx->seeds.ensure((size_t)seeds_pi * nimg * sizeof(double)));
  HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  if (o_first > 0) {
    const Octave& of = P.oct[o_first];
    HIPCHK(hipMemcpyAsync(ctx->seeds.as<double>() + of.seed_off, seed_host ? (const void*)seed_host : seed_dev,
                          (size_t)of.h * of.w * sizeof(double),
                          seed_host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice, ctx->stream));
    P.img = nullptr;
    P.img_stride = 0;
  } else if (img_host) {  // (a batch: image b from img_host + b * img_bstride, dense on the device)
    // Through the context's pinned staging: the rows are copied on several
    // host threads, then one DMA (the runtime's pageable path stages them on
    // one thread).  The staging is refilled only after the previous DMA out
    // of it has completed.
    const size_t img_bytes = (size_t)W * H * nimg * sizeof(float);
    HIPCHK(ctx->img.ensure(img_bytes));
    const bool dense = stride == (size_t)W && (nimg == 1 || img_bstride == (size_t)W * H);
    if (dense && host_registered(img_host, img_bytes)) {
      // page-locked caller memory (sift_host_register): one DMA straight from
      // it -- every host-image entry point synchronises before it returns
      HIPCHK(hipMemcpyAsync(ctx->img.p, img_host, img_bytes, hipMemcpyHostToDevice, ctx->stream));
    } else {
      if (!ctx->ev_himg) HIPCHK(hipEventCreateWithFlags(&ctx->ev_himg, hipEventDisableTiming));
      else HIPCHK(hipEventSynchronize(ctx->ev_himg));
      HIPCHK(ctx->himg.ensure(img_bytes));
#ifndef SIFT_H2D_PIPE
#define SIFT_H2D_PIPE 1
#endif
      if (!SIFT_H2D_PIPE) {
        for (int b = 0; b < nimg; ++b)
          par_copy_rows((float*)ctx->himg.p + (size_t)b * W * H, W * sizeof(float), img_host + (size_t)b * img_bstride,
                        stride * sizeof(float), W * sizeof(float), H, host_threads());
        HIPCHK(hipMemcpyAsync(ctx->img.p, ctx->himg.p, img_bytes, hipMemcpyHostToDevice, ctx->stream));
      } else
      for (int b = 0; b < nimg; ++b)
        HIPCHK(h2d_rows_staged(ctx->img.as<float>() + (size_t)b * W * H, (float*)ctx->himg.p + (size_t)b * W * H,
                               img_host + (size_t)b * img_bstride, stride * sizeof(float), W * sizeof(float), H,
                               host_threads(), ctx->stream));
      HIPCHK(hipEventRecord(ctx->ev_himg, ctx->stream));
    }
    P.img = ctx->img.as<float>();
    P.img_stride = W;
    P.img_bstride = nimg > 1 ? (long long)W * H : 0;
  } else {
    P.img = img_dev;
    P.img_stride = (int)stride;
  }
  P.seeds = ctx->seeds.as<double>();
  P.dog = ctx->dog.as<float>();
  {  // large-radius octaves keep their fp64 Gaussian planes (the exact passes read them)
    long long l64 = 0;
    for (int o = so_end; o < P.O; ++o)
      if (gauss_keep_l64(P, o)) {
        P.oct[o].l64_off = l64;
        l64 += (long long)P.NS * P.oct[o].h * P.oct[o].w;
      }
    if (l64) HIPCHK(ctx->l64.ensure((size_t)l64 * nimg * sizeof(double)));
    P.l64 = l64 ? ctx->l64.as<double>() : nullptr;
    P.l64_bstride = l64;
    size_t vs = 0;  // the split-pass octaves run in turn on this stream: one scratch (per image)
    for (int o = so_end; o < P.O; ++o)
      if (gauss_vsplit(P, o)) vs = std::max(vs, (size_t)P.NS * P.oct[o].h * P.oct[o].w);
    size_t sv = 0;
    for (int o = o_first; o < so_end; ++o) sv = std::max(sv, seed_only_scratch(P, o));
    if (sv) HIPCHK(ctx->seedv.ensure(sv * sizeof(double)));
    if (vs) HIPCHK(ctx->vsplit.ensure(vs * nimg * sizeof(double)));
    ctx->vsplit_pi = (long long)vs;
    // after the pass the scratch holds the last split octave's sums (octaves run in order)
    P.vsum_oct = -1;
    for (int o = so_end; o < P.O; ++o)
      if (gauss_vsplit(P, o)) P.vsum_oct = o;
    static const int vsum_exact = exp_knob("SIFT_VSUM_EXACT", 1);  // 0: the exact passes recompute (A/B)
    if (!vsum_exact) P.vsum_oct = -1;
    P.vsum = P.vsum_oct >= 0 ? ctx->vsplit.as<double>() : nullptr;
    P.vsum_bstride = ctx->vsplit_pi;
  }
  HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
  const double* base0 = nullptr;
  if (o_first == 0 && gauss_needs_base0(P)) {
    HIPCHK(ctx->base0.ensure((size_t)P.oct[0].h * P.oct[0].w * sizeof(double)));
    HIPCHK(launch_upsample_base(P, ctx->base0.as<double>(), ctx->stream));
    base0 = ctx->base0.as<double>();
  }
  ctx->x_prepared = false;
  const int nf = (fuse_extrema && o_first == 0 && fuse_enabled(p) && gauss_can_fuse(P, 0) &&
                  !(p->flags & SIFT_F_LOW_CONTRAST_LIST)) ? 1 : 0;
  if (nf) {  // bitmap geometry, counter resets: before the fused launch writes them
    ctx->dog_source = kNative;
    rc = extrema_prepare(ctx, ctx->stream, nf);
    if (rc) return rc;
    ctx->x_prepared = true;
  }
  const bool xseed = (p->flags & SIFT_F_EXPORT_NEXT_SEED) != 0;
  if (xseed) {
    ctx->xseed_h = (P.oct[P.O - 1].h + 1) / 2;  // background.js:118
    ctx->xseed_w = (P.oct[P.O - 1].w + 1) / 2;
    HIPCHK(ctx->xseed.ensure((size_t)ctx->xseed_h * ctx->xseed_w * sizeof(double)));
  }
  ctx->pass_kn.assign(P.O, std::string());
  for (int o = o_first; o < P.O; ++o) {
    const Octave& oc = P.oct[o];
    hipStream_t ost = ctx->stream;
    if (o < so_end) {
      ctx->pass_kn[o] = "k_seed_vert + k_seed_horz (next base only)";
      HIPCHK(launch_seed_only(P, o, ctx->seeds.as<double>() + oc.seed_off, ctx->seedv.as<double>(),
                              ctx->seeds.as<double>() + P.oct[o + 1].seed_off, ctx->stream));
      if (o == o_first) HIPCHK(hipEventRecord(ctx->ev[7], ctx->stream));
      HIPCHK(hipEventRecord(ctx->ev_go[o], ctx->stream));
      continue;
    }
    GaussLaunch L{};
    L.o = o;
    L.base = o == 0 ? base0 : ctx->seeds.as<double>() + oc.seed_off;
    L.gauss = keep_gauss ? ctx->gauss.as<float>() + oc.gauss_off : nullptr;
    L.dog = ctx->dog.as<float>() + oc.dog_off;
    L.next_seed = (o + 1 < P.O) ? ctx->seeds.as<double>() + P.oct[o + 1].seed_off
                                : (xseed ? ctx->xseed.as<double>() : nullptr);
    L.next_w = (o + 1 < P.O) ? P.oct[o + 1].w : (xseed ? ctx->xseed_w : 0);
    if (o < nf) {
      const ExtremaLaunch& XL = ctx->xl;
      L.fuse = 1;
      L.X.bitmap = XL.bitmap + XL.word_off[o];
      L.X.rowcount = XL.rowcount + XL.row_off[o];
      L.X.nw = ctx->x_nw[o];
      L.X.amb_keys = XL.amb_keys;
      L.X.counters = XL.counters;
      L.X.amb_cap = XL.amb_cap;
      L.X.c_lo = XL.c_lo;
      L.X.c_hi = XL.c_hi;
    }
    L.l64 = P.oct[o].l64_off >= 0 ? ctx->l64.as<double>() + P.oct[o].l64_off : nullptr;
    L.vsplit = gauss_vsplit(P, o) ? ctx->vsplit.as<double>() : nullptr;
    L.nimg = nimg;
    L.gauss_bs = tot * P.NS;
    L.dog_bs = tot * P.ND;
    L.seed_bs = seeds_pi;
    L.base_bs = o == 0 ? 0 : seeds_pi;
    L.l64_bs = P.l64_bstride;
    L.vsplit_bs = ctx->vsplit_pi;
    const char* kn = nullptr;
    HIPCHK(launch_gauss_dog(P, L, ost, 0, -1, &kn));
    ctx->pass_kn[o] = std::string(o == 0 && base0 ? "k_upsample_base + " : "") + (kn ? kn : "?");
    if (o == o_first) HIPCHK(hipEventRecord(ctx->ev[7], ost));
    HIPCHK(hipEventRecord(ctx->ev_go[o], ost));
  }
  HIPCHK(hipEventRecord(ctx->ev[2], ctx->stream));
  ctx->dog_source = kNative;
  ctx->have_gauss = keep_gauss;
  ctx->have_cand = false;
  ctx->has_xseed = xseed;
  return SIFT_OK;
}

// Gaussian+DoG timings of the last build (its events must have completed):
// the whole pass, octave 0's launch and every octave's launch.
static void read_gauss_times(sift_ctx* ctx) {
  float b = 0;
  if (hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[2]) == hipSuccess) ctx->tm.gauss_dog_ms = b;
  if (hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[7]) == hipSuccess) ctx->tm.gauss_oct0_ms = b;
  ctx->oct_ms.assign(ctx->P.O, 0.0);
  hipEvent_t prev = ctx->ev[1];
  for (int o = ctx->o_first; o < ctx->P.O; ++o) {
    if (hipEventElapsedTime(&b, prev, ctx->ev_go[o]) == hipSuccess) ctx->oct_ms[o] = b;
    prev = ctx->ev_go[o];
  }
}

// A page-locked caller image is uploaded by one DMA straight from the
// caller's memory (build_common), which every host-image entry point waits
// for before it returns -- on its error exits too, so the caller
// may free or overwrite the image as soon as the call returns.
static int host_image_exit(sift_ctx* ctx, int rc) {
  if (rc != SIFT_OK && ctx && ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  return rc;
}

extern "C" {

int sift_build_scale_space(sift_ctx* ctx, const float* img, int width, int height, size_t stride_px,
                           const sift_params* p, const double* sig) {
  int rc = build_common(ctx, img, nullptr, width, height, stride_px, p, sig);
  if (rc) return host_image_exit(ctx, rc);
  HIPCHK(hipStreamSynchronize(ctx->stream));
  float a = 0;
  (void)hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]);
  ctx->tm.h2d_ms = a;
  read_gauss_times(ctx);
  return SIFT_OK;
}

int sift_build_scale_space_device(sift_ctx* ctx, const float* d_img, int width, int height,
                                  size_t stride_px, const sift_params* p, const double* sig) {
  int rc = build_common(ctx, nullptr, d_img, width, height, stride_px, p, sig);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->tm.h2d_ms = 0;
  read_gauss_times(ctx);
  return SIFT_OK;
}

int sift_get_dims(sift_ctx* ctx, int o, int* rows, int* cols) {
  if (!ctx || !rows || !cols) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no pyramid");
  if (o < 0 || o >= ctx->P.O) return set_err(ctx, SIFT_E_ARG, "octave out of range");
  *rows = ctx->P.oct[o].h;
  *cols = ctx->P.oct[o].w;
  return SIFT_OK;
}

int sift_get_blur_level(sift_ctx* ctx, int kind, int o, int s, double* blur) {
  if (!ctx || !blur) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no pyramid");
  const int lim = kind == SIFT_PLANE_GAUSS ? ctx->P.NS : ctx->P.ND;
  if (o < 0 || o >= ctx->P.O || s < 0 || s >= lim) return set_err(ctx, SIFT_E_ARG, "index out of range");
  // DoG[s] carries L[s-1+1-1] = L[s].blurLevel (background.js:326-329).
  *blur = ctx->blur[o * ctx->P.NS + s];
  return SIFT_OK;
}

int sift_get_plane(sift_ctx* ctx, int kind, int o, int s, float* dst, size_t cap_px) {
  if (!ctx || !dst) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no pyramid");
  const Pyramid& P = ctx->P;
  if (o < 0 || o >= P.O) return set_err(ctx, SIFT_E_ARG, "octave out of range");
  if (o < ctx->planes_first) return set_err(ctx, SIFT_E_STATE, "octave not built (sift_detect_from_seed[_range])");
  const Octave& oc = P.oct[o];
  const size_t plane = (size_t)oc.h * oc.w;
  if (cap_px < plane) return set_err(ctx, SIFT_E_CAPACITY, "destination too small");
  const float* src = nullptr;
  if (kind == SIFT_PLANE_GAUSS) {
    if (!ctx->have_gauss) return set_err(ctx, SIFT_E_STATE, "Gaussian planes not materialised");
    if (s < 0 || s >= P.NS) return set_err(ctx, SIFT_E_ARG, "scale out of range");
    src = ctx->gauss.as<float>() + oc.gauss_off + (size_t)s * plane;
  } else if (kind == SIFT_PLANE_DOG) {
    if (s < 0 || s >= P.ND) return set_err(ctx, SIFT_E_ARG, "scale out of range");
    src = ctx->dog.as<float>() + oc.dog_off + (size_t)s * plane;
  } else {
    return set_err(ctx, SIFT_E_ARG, "bad plane kind");
  }
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(d2h_staged(ctx, dst, src, plane * sizeof(float)));
  return SIFT_OK;
}

int sift_load_dog(sift_ctx* ctx, const float* planes, int width, int height, const sift_params* p) {
  if (!ctx || !planes) return SIFT_E_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  int rc = setup_geometry(ctx, width, height, p, nullptr, false);
  if (rc) return rc;
  const long long tot = total_plane_px(ctx);
  HIPCHK(ctx->dog.ensure((size_t)tot * ctx->P.ND * sizeof(float)));
  HIPCHK(hipMemcpyAsync(ctx->dog.p, planes, (size_t)tot * ctx->P.ND * sizeof(float),
                        hipMemcpyHostToDevice, ctx->stream));
  ctx->P.dog = ctx->dog.as<float>();
  ctx->P.img = nullptr;
  ctx->P.seeds = nullptr;
  ctx->dog_source = kForeign;
  ctx->o_first = 0;
  ctx->scan_first = 0;
  ctx->planes_first = 0;
  ctx->have_gauss = false;
  ctx->have_cand = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_load_scale_space(sift_ctx* ctx, const float* planes, int width, int height,
                          const sift_params* p) {
  if (!ctx || !planes) return SIFT_E_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  int rc = setup_geometry(ctx, width, height, p, nullptr, false);
  if (rc) return rc;
  const Pyramid& P = ctx->P;
  const long long tot = total_plane_px(ctx);
  HIPCHK(ctx->gauss.ensure((size_t)tot * P.NS * sizeof(float)));
  HIPCHK(ctx->dog.ensure((size_t)tot * P.ND * sizeof(float)));
  HIPCHK(hipMemcpyAsync(ctx->gauss.p, planes, (size_t)tot * P.NS * sizeof(float),
                        hipMemcpyHostToDevice, ctx->stream));
  for (int o = 0; o < P.O; ++o) {
    const Octave& oc = P.oct[o];
    HIPCHK(launch_dog_from_gauss(ctx->gauss.as<float>() + oc.gauss_off, ctx->dog.as<float>() + oc.dog_off,
                                 (long long)oc.h * oc.w, P.ND, ctx->stream));
  }
  ctx->P.dog = ctx->dog.as<float>();
  ctx->P.img = nullptr;
  ctx->P.seeds = nullptr;
  ctx->dog_source = kForeign;
  ctx->o_first = 0;
  ctx->scan_first = 0;
  ctx->planes_first = 0;
  ctx->have_gauss = true;
  ctx->have_cand = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Extrema: scan -> sort by (octave, scale, y, x) -> exact tie resolution ->
// ordered compaction.  Leaves ctx->cand_key / cand_val / n_cand.
// ---------------------------------------------------------------------------
// Nearest fp32 at or below (dir < 0) / at or above (dir > 0) a double.
static float round_toward(double v, int dir) {
  float f = (float)v;
  if (dir < 0 && (double)f > v) f = std::nextafter(f, -INFINITY);
  if (dir > 0 && (double)f < v) f = std::nextafter(f, INFINITY);
  return f;
}

// Counter slots (ctx->counters): [0] ambiguous keys, [1] low-contrast
// extrema, [2] slots dropped by the exact pass, [3] uncertain refinements,
// [4] singular Hessians, [12] candidate slots, [13] keypoints, [16..] debug.
enum { kCntAmb = 0, kCntLow = 1, kCntDrop = 2, kCntUnc = 3, kCntSing = 4, kCntLowLate = 6, kCntLowSure = 7,
       kCntN = 12, kCntKp = 13 };
constexpr int kRetry = 1;  // internal: a capacity overflowed, grow and run again

// The extrema stage, launched without waiting, in three parts:
//   extrema_prepare  capacities, buffers, counter resets (on stream st);
//   extrema_scan     bitmap scan of octaves [o0, o1) (k_extrema) on st;
//   extrema_finish   row-count scan, ordered emission into cand_cap slots,
//                    exact tie resolution (context stream).
// Counts stay on the device.
static int extrema_prepare(sift_ctx* ctx, hipStream_t st, int nf) {
  Pyramid& P = ctx->P;
  const bool exact_planes = ctx->dog_source == kForeign;
  unsigned* cnt = ctx->counters.as<unsigned>();
  // Row / word geometry of the candidate bitmap: octaves < nf are decided in
  // the Gaussian pass (kFX-column words, bit 0 = column 1), the rest by the
  // scan (kXW-column words, bit 0 = column 0).
  ctx->x_nf = nf;
  ctx->x_word_off.assign(P.O, 0);
  ctx->x_row_off.assign(P.O, 0);
  ctx->x_nw.assign(P.O, 0);
  ctx->x_ww.assign(P.O, 0);
  ctx->x_woff.assign(P.O, 0);
  long long words = 0, rows = 0;
  for (int o = 0; o < P.O; ++o) {
    const bool f = o < nf;
    const int nw = f ? fused_words_per_row(P.oct[o].w) : extrema_words_per_row(P.oct[o].w);
    ctx->x_nw[o] = nw;
    ctx->x_ww[o] = f ? kFX : kXW;
    ctx->x_woff[o] = f ? 1 : 0;
    ctx->x_word_off[o] = words;
    ctx->x_row_off[o] = rows;
    words += (long long)P.S * P.oct[o].h * nw;
    rows += (long long)P.S * P.oct[o].h;
  }
  // A batch (P.nimg images) repeats the per-image words and rows image-major.
  const int ni = std::max(1, P.nimg);
  ctx->xl.words_per_img = words;
  ctx->xl.rows_per_img = (int)rows;
  words *= ni;
  rows *= ni;
  ctx->x_rows = rows;
  {  // capacities: an estimate for this geometry, grown on overflow (settle_extrema)
    const long long est = std::min<long long>(
        std::max<long long>((long long)P.S * total_plane_px(ctx) * ni / 192, 65536), 0x7fffffffLL);
    ctx->cand_cap = std::max(ctx->cand_cap, (unsigned)est);
    ctx->amb_cap = std::max(ctx->amb_cap, 4096 + (unsigned)est / 16);
  }
  HIPCHK(ctx->bitmap.ensure((size_t)words * sizeof(unsigned long long)));
  HIPCHK(ctx->rowcount.ensure((size_t)(rows + 1) * sizeof(unsigned)));
  HIPCHK(ctx->rowoff.ensure((size_t)(rows + 1) * sizeof(unsigned)));
  HIPCHK(ctx->amb_keys.ensure((size_t)ctx->amb_cap * sizeof(unsigned)));
  HIPCHK(ctx->cand_key.ensure((size_t)ctx->cand_cap * sizeof(unsigned)));
  HIPCHK(ctx->cand_val.ensure((size_t)ctx->cand_cap * sizeof(double)));
  HIPCHK(ctx->cand_keep.ensure((size_t)ctx->cand_cap * sizeof(unsigned)));
  ctx->want_low = (ctx->p.flags & SIFT_F_LOW_CONTRAST_LIST) != 0;
  ctx->have_low = false;
  if (ctx->want_low) {
    ctx->low_cap = std::max(ctx->low_cap, std::max(65536u, ctx->cand_cap / 4));
    HIPCHK(ctx->lowbitmap.ensure((size_t)words * sizeof(unsigned long long)));
    HIPCHK(ctx->lowrowcount.ensure((size_t)(rows + 1) * sizeof(unsigned)));
    HIPCHK(ctx->lowrowoff.ensure((size_t)(rows + 1) * sizeof(unsigned)));
    HIPCHK(ctx->low_key.ensure((size_t)ctx->low_cap * sizeof(unsigned)));
    HIPCHK(ctx->low_val.ensure((size_t)ctx->low_cap * sizeof(double)));
    HIPCHK(ctx->late_key.ensure((size_t)ctx->amb_cap * sizeof(unsigned)));
    HIPCHK(ctx->late_val.ensure((size_t)ctx->amb_cap * sizeof(double)));
  }
  // fp32 contrast thresholds: rounding is monotone, so |v32| < c_lo proves
  // |v64| < pix_thr and |v32| >= c_hi proves |v64| >= pix_thr.
  const float t_dn = round_toward(P.pix_thr, -1), t_up = round_toward(P.pix_thr, +1);
  // extrema and refinement counters and the refinement's per-block counts: one fill
  // (+ the row counts, and the low-contrast row counts when listed): one launch
  HIPCHK(launch_zero_words(cnt, kCntAll, ctx->rowcount.as<unsigned>(), rows + 1,
                           ctx->want_low ? ctx->lowrowcount.as<unsigned>() : nullptr, rows + 1, st));
  ctx->counters_zeroed = true;
  ExtremaLaunch& L = ctx->xl;
  const long long wpi = L.words_per_img;
  const int rpi = L.rows_per_img;
  L = ExtremaLaunch{};
  L.words_per_img = wpi;
  L.rows_per_img = rpi;
  L.exact_planes = exact_planes;
  L.c_lo = exact_planes ? t_up : t_dn;
  L.c_hi = exact_planes ? t_up : std::nextafter(t_up, INFINITY);
  L.bitmap = ctx->bitmap.as<unsigned long long>();
  L.rowcount = ctx->rowcount.as<unsigned>();
  for (int o = 0; o < P.O; ++o) {
    L.word_off[o] = ctx->x_word_off[o];
    L.row_off[o] = (int)ctx->x_row_off[o];
  }
  L.amb_keys = ctx->amb_keys.as<unsigned>();
  L.counters = cnt;
  L.amb_cap = ctx->amb_cap;
  // Ambiguous pixels are re-decided a word (62 pixels) at a time
  // (k_exact_words; SIFT_XWORDS=0: one wave per pixel key, experiments) --
  // not with fused octave-0 decisions, which list keys.
  static const int xwords = exp_knob("SIFT_XWORDS", 1);
  ctx->x_words = xwords && nf == 0 && !exact_planes;
  if (ctx->x_words) {
    HIPCHK(ctx->ambbitmap.ensure((size_t)words * sizeof(unsigned long long)));
    L.ambbitmap = ctx->ambbitmap.as<unsigned long long>();
  }
  L.lowbitmap = ctx->want_low ? ctx->lowbitmap.as<unsigned long long>() : nullptr;
  L.lowrowcount = ctx->want_low ? ctx->lowrowcount.as<unsigned>() : nullptr;
  // Patch capture (SIFT_PATCH=0: the refinement gathers every step, experiments).
  static const int capture = exp_knob("SIFT_PATCH", 1);
  const size_t slots = (size_t)ni * extrema_units(P) * kPatchUnitSlots;
  // the scan's patch stores take 32-bit byte offsets (a larger batch gathers);
  // the in-scan first step (SIFT_XREFINE) runs the fast pass's fp32 bounds,
  // so not on caller-supplied (exact) planes
  ctx->x_patch = kXCapture && capture != 0 &&
                 (SIFT_XREFINE == 1 ? !exact_planes : slots * kPatchFloats * sizeof(float) < ((size_t)1 << 31));
  ctx->has_patch = false;
  if (ctx->x_patch) {
    if (SIFT_XREFINE == 1) {
      HIPCHK(ctx->pre.ensure(std::max<size_t>(slots, 1) * sizeof(Keypoint)));
      L.pre = ctx->pre.as<Keypoint>();
      L.min_blur = ctx->p.min_blur;
      L.min_interpixel_distance = ctx->p.min_interpixel_distance;
    } else {
      HIPCHK(ctx->patch.ensure(std::max<size_t>(slots, 1) * kPatchFloats * sizeof(float)));
      L.patch = ctx->patch.as<float>();
    }
    HIPCHK(ctx->wslot.ensure((size_t)words * sizeof(unsigned)));
    HIPCHK(ctx->cand_patch.ensure((size_t)ctx->cand_cap * sizeof(unsigned)));
    L.wslot = ctx->wslot.as<unsigned>();
  }
  return SIFT_OK;
}

static int extrema_scan(sift_ctx* ctx, int o0, int o1, hipStream_t st) {
  HIPCHK(launch_extrema(ctx->P, ctx->xl, st, o0, o1));
  return SIFT_OK;
}

static int extrema_finish(sift_ctx* ctx) {
  Pyramid& P = ctx->P;
  unsigned* cnt = ctx->counters.as<unsigned>();
  const long long rows = ctx->x_rows;
  size_t tb = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ctx->rowcount.as<unsigned>(), ctx->rowoff.as<unsigned>(),
                                          (int)(rows + 1), ctx->stream));
  HIPCHK(ctx->temp.ensure(tb));
  tb = ctx->temp.bytes;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->temp.p, tb, ctx->rowcount.as<unsigned>(), ctx->rowoff.as<unsigned>(),
                                          (int)(rows + 1), ctx->stream));
  {
    EmitLaunch E{};
    E.n_out = cnt + kCntN;  // the list's length, written by k_emit (no 4-byte copy launch)
    E.n_index = rows;
    E.n_oct = P.O;
    E.o_first = std::min(std::max(ctx->o_first, ctx->scan_first), P.O - 1);  // rows of earlier octaves hold no decisions
    for (int o = 0; o < P.O; ++o) {
      E.row_off[o] = (int)ctx->x_row_off[o];
      E.word_off[o] = ctx->x_word_off[o];
      E.nw[o] = ctx->x_nw[o];
      E.ww[o] = ctx->x_ww[o];
      E.woff[o] = ctx->x_woff[o];
    }
    E.row_off[P.O] = ctx->xl.rows_per_img;
    E.words_per_img = ctx->xl.words_per_img;
    E.bitmap = ctx->bitmap.as<unsigned long long>();
    E.rowcount = ctx->rowcount.as<unsigned>();
    E.rowoff = ctx->rowoff.as<unsigned>();
    E.keys = ctx->cand_key.as<unsigned>();
    E.value = ctx->cand_val.as<double>();
    E.keep = ctx->cand_keep.as<unsigned>();
    E.cap = ctx->cand_cap;
    // Deferred values (SIFT_DEFER_VALUES=0: gathered here, experiments): the
    // refinement reads each candidate's plane value from its own patch.
    static const int defer = exp_knob("SIFT_DEFER_VALUES", 1);
    E.deferred = defer != 0;
    if (ctx->x_patch) {  // the scanned octaves carry captured patches, the fused ones gather
      E.wslot = ctx->wslot.as<unsigned>();
      E.cand_patch = ctx->cand_patch.as<unsigned>();
      for (int o = ctx->x_nf; o < P.O; ++o) E.patch_oct |= 1u << o;
    }
    HIPCHK(launch_emit(P, E, ctx->stream));
  }
  if (ctx->want_low) {  // the certain low-contrast extrema, in order (same scan + emission as the candidates)
    size_t lb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, lb, ctx->lowrowcount.as<unsigned>(),
                                            ctx->lowrowoff.as<unsigned>(), (int)(rows + 1), ctx->stream));
    HIPCHK(ctx->temp.ensure(lb));
    lb = ctx->temp.bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->temp.p, lb, ctx->lowrowcount.as<unsigned>(),
                                            ctx->lowrowoff.as<unsigned>(), (int)(rows + 1), ctx->stream));
    EmitLaunch E{};
    E.n_out = cnt + kCntLowSure;
    E.n_index = rows;
    E.n_oct = P.O;
    E.o_first = std::min(std::max(ctx->o_first, ctx->scan_first), P.O - 1);  // rows of earlier octaves hold no decisions
    for (int o = 0; o < P.O; ++o) {
      E.row_off[o] = (int)ctx->x_row_off[o];
      E.word_off[o] = ctx->x_word_off[o];
      E.nw[o] = ctx->x_nw[o];
      E.ww[o] = ctx->x_ww[o];
      E.woff[o] = ctx->x_woff[o];
    }
    E.row_off[P.O] = ctx->xl.rows_per_img;
    E.words_per_img = ctx->xl.words_per_img;
    E.bitmap = ctx->lowbitmap.as<unsigned long long>();
    E.rowcount = ctx->lowrowcount.as<unsigned>();
    E.rowoff = ctx->lowrowoff.as<unsigned>();
    E.keys = ctx->low_key.as<unsigned>();
    E.value = ctx->low_val.as<double>();
    E.keep = nullptr;
    E.cap = ctx->low_cap;
    HIPCHK(launch_emit(P, E, ctx->stream));
  }
  ExactLaunch X{};
  X.late_keys = ctx->want_low ? ctx->late_key.as<unsigned>() : nullptr;
  X.late_vals = ctx->want_low ? ctx->late_val.as<double>() : nullptr;
  X.amb_keys = ctx->amb_keys.as<unsigned>();
  X.amb_cap = ctx->amb_cap;
  X.keys = ctx->cand_key.as<unsigned>();
  X.n = cnt + kCntN;
  X.cap = ctx->cand_cap;
  X.keep = ctx->cand_keep.as<unsigned>();
  X.value = ctx->cand_val.as<double>();
  X.counters = cnt;
  static const int xpos = exp_knob("SIFT_XPOS", 1);
  if (xpos) {  // list positions from the emission geometry instead of a binary search
    X.bitmap = ctx->bitmap.as<unsigned long long>();
    X.rowoff = ctx->rowoff.as<unsigned>();
    X.words_per_img = ctx->xl.words_per_img;
    X.rows_per_img = ctx->xl.rows_per_img;
    for (int o = 0; o < P.O; ++o) {
      X.row_off[o] = (int)ctx->x_row_off[o];
      X.word_off[o] = ctx->x_word_off[o];
      X.nw[o] = ctx->x_nw[o];
      X.ww[o] = ctx->x_ww[o];
      X.woff[o] = ctx->x_woff[o];
    }
  }
  if (ctx->x_words) {
    X.ambbitmap = ctx->ambbitmap.as<unsigned long long>();
    X.bitmap = ctx->bitmap.as<unsigned long long>();
    X.rowoff = ctx->rowoff.as<unsigned>();
    X.words_per_img = ctx->xl.words_per_img;
    X.rows_per_img = ctx->xl.rows_per_img;
    for (int o = 0; o < P.O; ++o) {
      X.row_off[o] = (int)ctx->x_row_off[o];
      X.word_off[o] = ctx->x_word_off[o];
      X.nw[o] = ctx->x_nw[o];
      X.ww[o] = ctx->x_ww[o];
      X.woff[o] = ctx->x_woff[o];
    }
    HIPCHK(launch_exact_words(P, X, ctx->stream));
  } else {
    HIPCHK(launch_exact_extrema(P, X, ctx->stream));
  }
  HIPCHK(hipEventRecord(ctx->ev[4], ctx->stream));
  ctx->slot_cap = (int)ctx->cand_cap;
  ctx->has_keep = true;
  ctx->slots_rows = true;
  ctx->has_patch = ctx->x_patch;
  ctx->ext_pending = true;
  return SIFT_OK;
}

// The whole extrema stage on the context stream.
static int launch_extrema_stage(sift_ctx* ctx) {
  HIPCHK(hipEventRecord(ctx->ev[3], ctx->stream));
  int o0 = std::max(ctx->o_first, ctx->scan_first);
  if (ctx->x_prepared) {  // octaves < x_nf were decided in the Gaussian pass
    ctx->x_prepared = false;
    o0 = std::max(o0, ctx->x_nf);
  } else {
    const int rc = extrema_prepare(ctx, ctx->stream, 0);
    if (rc) return rc;
  }
  int rc = extrema_scan(ctx, o0, ctx->P.O, ctx->stream);
  if (rc) return rc;
  return extrema_finish(ctx);
}

// Reads the extrema counts (ctx->h_counters must hold the device counters):
// kRetry after growing the capacities when one overflowed.
static int settle_extrema(sift_ctx* ctx) {
  const unsigned* h = ctx->h_counters;
  ctx->ext_pending = false;
  const unsigned n = h[kCntN], n_amb = h[kCntAmb];
  const unsigned n_ls = ctx->want_low ? h[kCntLowSure] : 0u;
  if (n > ctx->cand_cap || n_amb > ctx->amb_cap || n_ls > ctx->low_cap || h[kAmbWords] > ctx->amb_cap) {
    if (n > ctx->cand_cap) ctx->cand_cap = n + n / 4 + 1024;
    if (n_amb > ctx->amb_cap) ctx->amb_cap = n_amb + n_amb / 4 + 1024;
    if (n_ls > ctx->low_cap) ctx->low_cap = n_ls + n_ls / 4 + 1024;
    return kRetry;
  }
  ctx->have_low = ctx->want_low;
  ctx->n_low_sure = n_ls;
  ctx->n_low_late = ctx->want_low ? h[kCntLowLate] : 0u;
  ctx->n_exact = n_amb;
  ctx->n_low = h[kCntLow];
  ctx->n_slots = n;
  ctx->n_cand = n - h[kCntDrop];
  ctx->have_cand = true;
  return SIFT_OK;
}

static int run_extrema(sift_ctx* ctx) {
  for (;;) {
    int rc = launch_extrema_stage(ctx);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(ctx->h_counters, ctx->counters.p, 16 * sizeof(unsigned), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    rc = settle_extrema(ctx);
    if (rc != kRetry) return rc;
  }
}

// Refinement over ctx->slot_cap slots, *counters[12] of them live, without
// a host round trip; refine_settle's one synchronisation reads every count
// back and returns kRetry when the extrema stage it follows overflowed.
static int refine_enqueue(sift_ctx* ctx) {
  Pyramid& P = ctx->P;
  const int cap = ctx->slot_cap;
  unsigned* cnt = ctx->counters.as<unsigned>();
  HIPCHK(hipEventRecord(ctx->ev[5], ctx->stream));
  HIPCHK(ctx->status.ensure((size_t)std::max(cap, 1) * sizeof(int)));
  HIPCHK(ctx->kp_tmp.ensure((size_t)std::max(cap, 1) * sizeof(Keypoint)));
  HIPCHK(ctx->kp.ensure((size_t)std::max(cap, 1) * sizeof(Keypoint)));
  HIPCHK(ctx->uncertain.ensure((size_t)std::max(cap, 1) * sizeof(unsigned)));
  HIPCHK(ctx->keep.ensure((size_t)std::max(cap, 1) * sizeof(unsigned)));
  HIPCHK(ctx->pos.ensure((size_t)std::max(cap, 1) * sizeof(unsigned)));
  if (!ctx->counters_zeroed) {  // refinement without a fresh extrema stage (caller candidates / re-run)
    HIPCHK(hipMemsetAsync(cnt + kCntUnc, 0, 2 * sizeof(unsigned), ctx->stream));
    HIPCHK(hipMemsetAsync(cnt + kCntKp, 0, sizeof(unsigned), ctx->stream));
    HIPCHK(hipMemsetAsync(cnt + 16, 0, 16 * sizeof(unsigned), ctx->stream));
    HIPCHK(hipMemsetAsync(cnt + kBlk, 0, (kCntAll - kBlk) * sizeof(unsigned), ctx->stream));
  }
  ctx->counters_zeroed = false;
  ctx->n_kp = 0;
  ctx->n_sing = 0;
  if (cap > 0) {
    RefineLaunch R{};
    R.cand_key = ctx->cand_key.as<unsigned>();
    R.cand_val = ctx->cand_val.as<double>();
    R.keep = ctx->has_keep ? ctx->cand_keep.as<unsigned>() : nullptr;
    R.n = cnt + kCntN;
    R.cap = cap;
    R.exact_planes = ctx->dog_source == kForeign;
    R.min_blur = ctx->p.min_blur;
    R.min_interpixel_distance = ctx->p.min_interpixel_distance;
    R.status = ctx->status.as<int>();
    R.kp = ctx->kp_tmp.as<Keypoint>();
    R.uncertain = ctx->uncertain.as<unsigned>();
    R.counters = cnt;
    R.perm = nullptr;
    if (ctx->has_patch && ctx->slots_rows) {
      R.cand_patch = ctx->cand_patch.as<unsigned>();
      if (SIFT_XREFINE == 1) R.pre = ctx->pre.as<Keypoint>();
      else R.patch = ctx->patch.as<float>();
    }
    static const int band_order = exp_knob("SIFT_BAND_ORDER", 1);
    if (band_order && ctx->slots_rows) {
      BandOrder B{};
      B.n_oct = P.O;
      B.S = P.S;
      int items = 0;
      for (int o = 0; o < P.O; ++o) {
        B.item_off[o] = items;
        B.row_off[o] = (int)ctx->x_row_off[o];
        items += P.S * ((P.oct[o].h + kBandRows - 1) / kBandRows);
      }
      B.item_off[P.O] = items;
      B.rows_per_img = ctx->xl.rows_per_img;
      items *= std::max(1, P.nimg);  // image-major
      B.n_items = items;
      HIPCHK(ctx->band_cnt.ensure((size_t)items * sizeof(unsigned)));
      HIPCHK(ctx->band_first.ensure((size_t)items * sizeof(unsigned)));
      HIPCHK(ctx->band_start.ensure((size_t)items * sizeof(unsigned)));
      HIPCHK(ctx->perm.ensure((size_t)cap * sizeof(unsigned)));
      B.rowoff = ctx->rowoff.as<unsigned>();
      B.count = ctx->band_cnt.as<unsigned>();
      B.first = ctx->band_first.as<unsigned>();
      B.start = ctx->band_start.as<unsigned>();
      B.perm = ctx->perm.as<unsigned>();
      B.cap = cap;
      HIPCHK(launch_band_items(P, B, ctx->stream));
      size_t tb = 0;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, B.count, ctx->band_start.as<unsigned>(), items,
                                              ctx->stream));
      HIPCHK(ctx->temp.ensure(tb));
      tb = ctx->temp.bytes;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->temp.p, tb, B.count, ctx->band_start.as<unsigned>(), items,
                                              ctx->stream));
      HIPCHK(launch_band_fill(P, B, ctx->stream));
      R.perm = B.perm;
    }
    HIPCHK(launch_refine_fast(P, R, ctx->stream));
    HIPCHK(hipEventRecord(ctx->ev_heavy, ctx->stream));  // the rest is latency-bound tail work
    // Uncertain decisions exist only with fp32-rounded native planes.
#ifndef SIFT_WIDE_EXACT
#define SIFT_WIDE_EXACT 0  // 1: 256-thread exact refinement for whole images too (A/B builds)
#endif
    R.wide_exact = SIFT_WIDE_EXACT || ctx->o_first > 0;  // a tail piece (sift_detect_from_seed*): latency over throughput
    if (ctx->dog_source == kNative) HIPCHK(launch_refine_exact(P, R, ctx->stream));
#if SIFT_KEEP_SCAN
    HIPCHK(ctx->keep_tile.ensure(keep_tiles(cap) * sizeof(unsigned)));
    HIPCHK(launch_keep_compact(P, R.status, R.cand_key, ctx->keep.as<unsigned>(), ctx->pos.as<unsigned>(),
                               ctx->keep_tile.as<unsigned>(), R.n, cap, ctx->own_lo, ctx->own_hi, cnt + kBlk, R.kp,
                               ctx->kp.as<Keypoint>(), ctx->stream));
#else
    HIPCHK(launch_status_to_keep(P, R.status, R.cand_key, ctx->keep.as<unsigned>(), R.n, cap, ctx->own_lo,
                                 ctx->own_hi, cnt + kBlk, ctx->stream));
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ctx->keep.as<unsigned>(), ctx->pos.as<unsigned>(), cap,
                                            ctx->stream));
    HIPCHK(ctx->temp.ensure(tb));
    tb = ctx->temp.bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->temp.p, tb, ctx->keep.as<unsigned>(), ctx->pos.as<unsigned>(), cap,
                                            ctx->stream));
    HIPCHK(launch_scatter_keypoints(ctx->keep.as<unsigned>(), ctx->pos.as<unsigned>(), R.kp, R.n, cap,
                                    ctx->kp.as<Keypoint>(), ctx->stream));
#endif
    HIPCHK(launch_count_keypoints(P, ctx->pos.as<unsigned>(), ctx->keep.as<unsigned>(), R.cand_key, R.n, cap,
                                  cnt + kCntKp, cnt + kBlk, ctx->stream));
    if (ctx->p.flags & SIFT_F_KEYPOINT_ORIGINS) {
      HIPCHK(ctx->kp_key.ensure((size_t)cap * sizeof(unsigned)));
      HIPCHK(launch_scatter_keys(ctx->keep.as<unsigned>(), ctx->pos.as<unsigned>(), R.cand_key, R.n, cap,
                                 ctx->kp_key.as<unsigned>(), ctx->stream));
    }
  }
  ctx->has_origins = (ctx->p.flags & SIFT_F_KEYPOINT_ORIGINS) != 0;
  // the counts and the kept keypoints per block (the block starts stay on the device)
  const int nblk = std::max(1, P.nimg) * P.O * P.S;
  HIPCHK(hipMemcpyAsync(ctx->h_counters, cnt, (kBlk + nblk) * sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev[6], ctx->stream));
  return SIFT_OK;
}

// Waits for the refinement enqueued by refine_enqueue and reads its counts
// (and the extrema counts when those are still pending).
static int refine_settle(sift_ctx* ctx) {
  const int cap = ctx->slot_cap;
  HIPCHK(hipEventSynchronize(ctx->ev[6]));
  if (ctx->ext_pending) {
    const int rc = settle_extrema(ctx);
    if (rc) return rc;
  }
  const unsigned* h = ctx->h_counters;
  if (h[kCntUnc] > (unsigned)cap) return set_err(ctx, SIFT_E_STATE, "uncertain list overflow");
  if (h[kCntUnc] && ctx->dog_source != kNative)
    return set_err(ctx, SIFT_E_STATE, "uncertain refinement without a native pyramid");
  ctx->n_exact += h[kCntUnc];
  ctx->n_kp = cap > 0 ? h[kCntKp] : 0;
  ctx->n_sing = h[kCntSing];
  ctx->blk_counts.assign((size_t)std::max(1, ctx->P.nimg) * ctx->P.O * ctx->P.S, 0);
  if (cap > 0)
    for (size_t b = 0; b < ctx->blk_counts.size(); ++b) ctx->blk_counts[b] = h[kBlk + b];
  if (exp_knob("SIFT_DEBUG_REFINE", 0))
    std::fprintf(stderr,
                 "refine uncertain %u: det %u alpha %u omega %u edge_dt %u edge_int %u round %u | iter %u %u %u %u %u"
                 " | output precision %u\n",
                 h[kCntUnc], h[16], h[17], h[18], h[19], h[20], h[21], h[22], h[23], h[24], h[25], h[26], h[27]);
  return SIFT_OK;
}

static int run_refine(sift_ctx* ctx) {
  const int rc = refine_enqueue(ctx);
  return rc ? rc : refine_settle(ctx);
}

static void read_stage_times(sift_ctx* ctx, bool extrema, bool refine) {
  float t = 0;
  (void)hipEventSynchronize(ctx->ev[6]);
  if (extrema && hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[4]) == hipSuccess) ctx->tm.extrema_ms = t;
  if (refine && hipEventElapsedTime(&t, ctx->ev[5], ctx->ev[6]) == hipSuccess) ctx->tm.refine_ms = t;
}

extern "C" {

int sift_copy_candidates(sift_ctx* ctx, sift_extremum* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (ctx->P.nimg > 1) return set_err(ctx, SIFT_E_UNSUPPORTED, "a batch detection returns keypoints only");
  if (!ctx->have_cand) return set_err(ctx, SIFT_E_STATE, "no candidates");
  if (n_out) *n_out = ctx->n_cand;
  if (!out) return SIFT_OK;
  if (cap < ctx->n_cand) return set_err(ctx, SIFT_E_CAPACITY, "candidate buffer too small");
  const size_t n = ctx->n_slots;
  std::vector<unsigned> keys(n), keep(n, 1u);
  std::vector<double> vals(n);
  if (n) {
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->slots_rows)  // deferred candidate values (EmitLaunch.deferred) from the DoG planes
      HIPCHK(launch_fill_values(ctx->P, ctx->cand_key.as<unsigned>(), ctx->cand_val.as<double>(),
                                ctx->counters.as<unsigned>() + kCntN, (int)n, ctx->stream));
    HIPCHK(hipMemcpyAsync(keys.data(), ctx->cand_key.p, n * sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(vals.data(), ctx->cand_val.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->has_keep)
      HIPCHK(hipMemcpyAsync(keep.data(), ctx->cand_keep.p, n * sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  const Pyramid& P = ctx->P;
  size_t j = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!keep[i]) continue;
    unsigned k = keys[i];
    int o = 0;
    while (o + 1 < P.O && k >= P.oct[o + 1].key_off) ++o;
    unsigned r = k - P.oct[o].key_off;
    const unsigned plane = (unsigned)P.oct[o].h * (unsigned)P.oct[o].w;
    const int s = (int)(r / plane) + 1;
    r -= (unsigned)(s - 1) * plane;
    out[j].octave = o;
    out[j].scale = s;
    out[j].y = (int)(r / (unsigned)P.oct[o].w);
    out[j].x = (int)(r % (unsigned)P.oct[o].w);
    out[j].value = vals[i];
    ++j;
  }
  if (n_out) *n_out = j;
  return SIFT_OK;
}

int sift_copy_low_contrast(sift_ctx* ctx, sift_extremum* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->have_low) return set_err(ctx, SIFT_E_STATE, "no low-contrast list (SIFT_F_LOW_CONTRAST_LIST)");
  const size_t ns = ctx->n_low_sure, nl = ctx->n_low_late, n = ns + nl;
  if (n_out) *n_out = n;
  if (!out) return SIFT_OK;
  if (cap < n) return set_err(ctx, SIFT_E_CAPACITY, "low-contrast buffer too small");
  std::vector<unsigned> k(n);
  std::vector<double> v(n);
  if (n) {
    HIPCHK(hipSetDevice(ctx->device));
    if (ns) {
      HIPCHK(hipMemcpyAsync(k.data(), ctx->low_key.p, ns * sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipMemcpyAsync(v.data(), ctx->low_val.p, ns * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    }
    if (nl) {
      HIPCHK(hipMemcpyAsync(k.data() + ns, ctx->late_key.p, nl * sizeof(unsigned), hipMemcpyDeviceToHost,
                            ctx->stream));
      HIPCHK(hipMemcpyAsync(v.data() + ns, ctx->late_val.p, nl * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  // The late entries (exact-pass decisions, unordered) merge into the ordered list by key.
  std::vector<size_t> idx(n);
  for (size_t i = 0; i < n; ++i) idx[i] = i;
  std::sort(idx.begin() + ns, idx.end(), [&](size_t a, size_t b) { return k[a] < k[b]; });
  std::inplace_merge(idx.begin(), idx.begin() + ns, idx.end(), [&](size_t a, size_t b) { return k[a] < k[b]; });
  const Pyramid& P = ctx->P;
  for (size_t j = 0; j < n; ++j) {
    const unsigned key = k[idx[j]];
    int o = 0;
    while (o + 1 < P.O && key >= P.oct[o + 1].key_off) ++o;
    const unsigned plane = (unsigned)P.oct[o].h * (unsigned)P.oct[o].w, r = key - P.oct[o].key_off;
    out[j].octave = o;
    out[j].scale = (int)(r / plane) + 1;
    out[j].y = (int)((r % plane) / (unsigned)P.oct[o].w);
    out[j].x = (int)((r % plane) % (unsigned)P.oct[o].w);
    out[j].value = v[idx[j]];
  }
  return SIFT_OK;
}

int sift_find_extrema(sift_ctx* ctx, sift_extremum* out, size_t cap, size_t* n_out, size_t* n_low) {
  if (!ctx) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no DoG pyramid: build or load one first");
  HIPCHK(hipSetDevice(ctx->device));
  int rc = run_extrema(ctx);
  if (rc) return rc;
  HIPCHK(hipEventRecord(ctx->ev[6], ctx->stream));
  read_stage_times(ctx, true, false);
  if (n_low) *n_low = ctx->n_low;
  return sift_copy_candidates(ctx, out, cap, n_out);
}

int sift_refine_params(sift_ctx* ctx, double min_blur_level, double min_interpixel_distance) {
  if (!ctx) return SIFT_E_ARG;
  if (!(min_blur_level > 0) || !(min_interpixel_distance > 0)) return set_err(ctx, SIFT_E_ARG, "bad refine scalars");
  ctx->p.min_blur = min_blur_level;
  ctx->p.min_interpixel_distance = min_interpixel_distance;
  return SIFT_OK;
}

int sift_set_candidates(sift_ctx* ctx, const sift_extremum* cand, size_t n) {
  if (!ctx || (!cand && n)) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no DoG pyramid");
  const Pyramid& P = ctx->P;
  std::vector<unsigned> keys(n);
  std::vector<double> vals(n);
  for (size_t i = 0; i < n; ++i) {
    const sift_extremum& c = cand[i];
    if (c.octave < 0 || c.octave >= P.O) return set_err(ctx, SIFT_E_ARG, "candidate octave out of range");
    const Octave& oc = P.oct[c.octave];
    if (c.scale < 1 || c.scale > P.S || c.y < 1 || c.y > oc.h - 2 || c.x < 1 || c.x > oc.w - 2)
      return set_err(ctx, SIFT_E_ARG, "candidate outside the refinable interior");
    keys[i] = oc.key_off + (unsigned)(c.scale - 1) * (unsigned)oc.h * (unsigned)oc.w + (unsigned)c.y * oc.w + c.x;
    vals[i] = c.value;
  }
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(ctx->cand_key.ensure(std::max<size_t>(n, 1) * sizeof(unsigned)));
  HIPCHK(ctx->cand_val.ensure(std::max<size_t>(n, 1) * sizeof(double)));
  if (n) {
    HIPCHK(hipMemcpyAsync(ctx->cand_key.p, keys.data(), n * sizeof(unsigned), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->cand_val.p, vals.data(), n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  }
  const unsigned n32 = (unsigned)n;
  HIPCHK(hipMemcpyAsync(ctx->counters.as<unsigned>() + kCntN, &n32, sizeof(unsigned), hipMemcpyHostToDevice,
                        ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->n_cand = n;
  ctx->n_slots = n;
  ctx->slot_cap = (int)n;
  ctx->ext_pending = false;
  ctx->has_keep = false;
  ctx->slots_rows = false;
  ctx->has_patch = false;
  ctx->have_cand = true;
  return SIFT_OK;
}

int sift_copy_keypoints(sift_ctx* ctx, sift_keypoint* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (n_out) *n_out = ctx->n_kp;
  if (!out) return SIFT_OK;
  if (cap < ctx->n_kp) return set_err(ctx, SIFT_E_CAPACITY, "keypoint buffer too small");
  if (ctx->n_kp) {
    HIPCHK(hipMemcpyAsync(out, ctx->kp.p, ctx->n_kp * sizeof(sift_keypoint), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  return SIFT_OK;
}

// The records as two field arrays (one DMA into the context's pinned staging,
// one pass over it on the host threads).
int sift_copy_keypoints_soa(sift_ctx* ctx, int32_t* ints, double* reals, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (n_out) *n_out = ctx->n_kp;
  if (!ints || !reals) return ints || reals ? SIFT_E_ARG : SIFT_OK;
  if (cap < ctx->n_kp) return set_err(ctx, SIFT_E_CAPACITY, "keypoint buffer too small");
  const size_t n = ctx->n_kp;
  if (!n) return SIFT_OK;
  HIPCHK(hipSetDevice(ctx->device));
  // Page-locked destinations (sift_host_register; the N-API result pool's
  // recycled buffers): split on the device, one DMA into each array.
  if (host_registered(ints, n * 4 * sizeof(int32_t)) && host_registered(reals, n * 4 * sizeof(double))) {
    HIPCHK(ctx->kp_soa.ensure(n * sizeof(sift_keypoint)));
    int32_t* di = ctx->kp_soa.as<int32_t>();
    double* dr = reinterpret_cast<double*>(di + 4 * n);  // 16 n bytes in: 16-byte aligned
    HIPCHK(launch_kp_soa(ctx->kp.as<Keypoint>(), (int)n, di, dr, ctx->stream));
    HIPCHK(hipMemcpyAsync(ints, di, n * 4 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(reals, dr, n * 4 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SIFT_OK;
  }
  HIPCHK(ctx->hkp.ensure(n * sizeof(sift_keypoint)));
  HIPCHK(hipMemcpyAsync(ctx->hkp.p, ctx->kp.p, n * sizeof(sift_keypoint), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const sift_keypoint* k = (const sift_keypoint*)ctx->hkp.p;
  auto part = [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1; ++i) {
      ints[4 * i] = k[i].octave;
      ints[4 * i + 1] = k[i].scale_level;
      ints[4 * i + 2] = k[i].local_x;
      ints[4 * i + 3] = k[i].local_y;
      reals[4 * i] = k[i].abs_sigma;
      reals[4 * i + 1] = k[i].abs_x;
      reals[4 * i + 2] = k[i].abs_y;
      reals[4 * i + 3] = k[i].interp_value;
    }
  };
  const int nt = n >= 65536 ? host_threads() : 1;
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) {
    const size_t i0 = std::min(n, t * per), i1 = std::min(n, (t + 1) * per);
    if (i0 < i1) th.emplace_back(part, i0, i1);
  }
  part(0, std::min(n, per));
  for (auto& x : th) x.join();
  return SIFT_OK;
}

int sift_refine(sift_ctx* ctx, sift_keypoint* out, size_t cap, size_t* n_out, size_t* n_singular) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->have_cand) return set_err(ctx, SIFT_E_STATE, "no candidates: run sift_find_extrema first");
  HIPCHK(hipSetDevice(ctx->device));
  int rc = run_refine(ctx);
  if (rc) return rc == kRetry ? set_err(ctx, SIFT_E_STATE, "candidate capacity overflow") : rc;
  read_stage_times(ctx, false, true);
  if (n_singular) *n_singular = ctx->n_sing;
  rc = sift_copy_keypoints(ctx, out, cap, n_out);
  if (rc) return rc;
  if (ctx->n_sing) return set_err(ctx, SIFT_E_SINGULAR, "singular Hessian (the reference throws a TypeError here)");
  return SIFT_OK;
}

// Enqueues one whole detection (Gaussian+DoG, extrema, refinement) without
// waiting; detect_finish completes it.
// Two phases: the Gaussian+DoG pass, then extrema + refinement (the caller
// may order the second phase after other contexts' work in between).
static int detect_begin(sift_ctx* ctx, const float* img_host, const float* img_dev, int W, int H, size_t stride,
                        const sift_params* p, int nimg = 1, size_t img_bstride = 0) {
  if (!ctx) return SIFT_E_ARG;
  int rc = build_common(ctx, img_host, img_dev, W, H, stride, p, nullptr, 0, nullptr, nullptr, nimg == 1, nimg,
                        img_bstride);
  if (rc) return rc;
  ctx->begin_pending = true;
  ctx->detect_host_img = img_host != nullptr;
  return SIFT_OK;
}

static int detect_end(sift_ctx* ctx) {
  if (!ctx->begin_pending) return set_err(ctx, SIFT_E_STATE, "no detection begun (sift_detect_begin_async)");
  ctx->begin_pending = false;
  int rc = launch_extrema_stage(ctx);
  if (rc) return rc;
  rc = refine_enqueue(ctx);
  if (rc) return rc;
  ctx->detect_pending = true;
  return SIFT_OK;
}

static int detect_enqueue(sift_ctx* ctx, const float* img_host, const float* img_dev, int W, int H,
                          size_t stride, const sift_params* p, int nimg = 1, size_t img_bstride = 0) {
  const int rc = detect_begin(ctx, img_host, img_dev, W, H, stride, p, nimg, img_bstride);
  return rc ? rc : detect_end(ctx);
}

// One host synchronisation per image; a capacity overflow (first images)
// grows the buffers and reruns extrema + refinement.
static int detect_finish(sift_ctx* ctx, sift_keypoint* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->detect_pending) return set_err(ctx, SIFT_E_STATE, "no detection in flight");
  ctx->detect_pending = false;
  int rc = refine_settle(ctx);
  while (rc == kRetry) {
    rc = launch_extrema_stage(ctx);
    if (rc) return rc;
    rc = run_refine(ctx);
  }
  if (rc) return rc;
  float a = 0;
  (void)hipEventSynchronize(ctx->ev[6]);
  if (ctx->detect_host_img && hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]) == hipSuccess) ctx->tm.h2d_ms = a;
  if (!ctx->detect_host_img) ctx->tm.h2d_ms = 0;
  read_gauss_times(ctx);
  read_stage_times(ctx, true, true);
  rc = sift_copy_keypoints(ctx, out, cap, n_out);
  if (rc) return rc;
  if (ctx->n_sing) return set_err(ctx, SIFT_E_SINGULAR, "singular Hessian (the reference throws a TypeError here)");
  return SIFT_OK;
}

static int detect_common(sift_ctx* ctx, const float* img_host, const float* img_dev, int W, int H,
                         size_t stride, const sift_params* p, sift_keypoint* out, size_t cap,
                         size_t* n_out) {
  const int rc = detect_enqueue(ctx, img_host, img_dev, W, H, stride, p);
  return rc ? rc : detect_finish(ctx, out, cap, n_out);
}

int sift_detect_device_async(sift_ctx* ctx, const float* d_img, int width, int height, size_t stride_px,
                             const sift_params* p) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (ctx->detect_pending || ctx->begin_pending)
    return set_err(ctx, SIFT_E_STATE, "a detection is already in flight on this context");
  return detect_enqueue(ctx, nullptr, d_img, width, height, stride_px, p);
}

int sift_detect_batch_device_async(sift_ctx* ctx, const float* d_imgs, int n_images, size_t image_stride_px,
                                   int width, int height, size_t stride_px, const sift_params* p) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (n_images < 1 || (n_images > 1 && image_stride_px < (size_t)height * stride_px))
    return set_err(ctx, SIFT_E_ARG, "n_images < 1 or overlapping images");
  if (ctx->detect_pending || ctx->begin_pending)
    return set_err(ctx, SIFT_E_STATE, "a detection is already in flight on this context");
  return detect_enqueue(ctx, nullptr, d_imgs, width, height, stride_px, p, n_images, image_stride_px);
}

int sift_detect_batch(sift_ctx* ctx, const float* imgs, int n_images, size_t image_stride_px, int width, int height,
                      size_t stride_px, const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (n_images < 1 || (n_images > 1 && image_stride_px < (size_t)height * stride_px))
    return set_err(ctx, SIFT_E_ARG, "n_images < 1 or overlapping images");
  if (ctx->detect_pending || ctx->begin_pending)
    return set_err(ctx, SIFT_E_STATE, "a detection is already in flight on this context");
  const int rc = detect_enqueue(ctx, imgs, nullptr, width, height, stride_px, p, n_images, image_stride_px);
  return host_image_exit(ctx, rc ? rc : detect_finish(ctx, out, cap, n_out));
}

int sift_detect_batch_device(sift_ctx* ctx, const float* d_imgs, int n_images, size_t image_stride_px, int width,
                             int height, size_t stride_px, const sift_params* p, sift_keypoint* out, size_t cap,
                             size_t* n_out) {
  const int rc = sift_detect_batch_device_async(ctx, d_imgs, n_images, image_stride_px, width, height, stride_px, p);
  return rc ? rc : detect_finish(ctx, out, cap, n_out);
}

int sift_detect_begin_async(sift_ctx* ctx, const float* d_img, int width, int height, size_t stride_px,
                            const sift_params* p) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (ctx->detect_pending || ctx->begin_pending)
    return set_err(ctx, SIFT_E_STATE, "a detection is already in flight on this context");
  return detect_begin(ctx, nullptr, d_img, width, height, stride_px, p);
}

int sift_detect_end_async(sift_ctx* ctx) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  return detect_end(ctx);
}

int sift_detect_wait(sift_ctx* ctx, sift_keypoint* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  return detect_finish(ctx, out, cap, n_out);
}

int sift_detect(sift_ctx* ctx, const float* img, int width, int height, size_t stride_px, const sift_params* p,
                sift_keypoint* out, size_t cap, size_t* n_out) {
  if (ctx) (void)hipSetDevice(ctx->device);
  return host_image_exit(ctx, detect_common(ctx, img, nullptr, width, height, stride_px, p, out, cap, n_out));
}

int sift_detect_device(sift_ctx* ctx, const float* d_img, int width, int height, size_t stride_px,
                       const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out) {
  if (ctx) (void)hipSetDevice(ctx->device);
  return detect_common(ctx, nullptr, d_img, width, height, stride_px, p, out, cap, n_out);
}

int sift_last_counts(sift_ctx* ctx, size_t* nc, size_t* nl, size_t* nk, size_t* ns, size_t* ne) {
  if (!ctx) return SIFT_E_ARG;
  if (nc) *nc = ctx->n_cand;
  if (nl) *nl = ctx->n_low;
  if (nk) *nk = ctx->n_kp;
  if (ns) *ns = ctx->n_sing;
  if (ne) *ne = ctx->n_exact;
  return SIFT_OK;
}

int sift_last_timings(sift_ctx* ctx, sift_timings* t) {
  if (!ctx || !t) return SIFT_E_ARG;
  *t = ctx->tm;
  return SIFT_OK;
}

int sift_last_octave_timings(sift_ctx* ctx, double* ms, int cap, int* n_out) {
  if (!ctx) return SIFT_E_ARG;
  const int n = (int)ctx->oct_ms.size();
  if (n_out) *n_out = n;
  if (!ms) return SIFT_OK;
  if (cap < n) return set_err(ctx, SIFT_E_CAPACITY, "destination too small (one per octave)");
  for (int o = 0; o < n; ++o) ms[o] = ctx->oct_ms[o];
  return SIFT_OK;
}

int sift_last_pass_kernels(sift_ctx* ctx, char* buf, size_t cap, size_t* len) {
  if (!ctx) return SIFT_E_ARG;
  std::string t;
  for (size_t o = 0; o < ctx->pass_kn.size(); ++o) {
    if (ctx->pass_kn[o].empty()) continue;
    if (!t.empty()) t += "; ";
    t += "o" + std::to_string(o) + ": " + ctx->pass_kn[o];
  }
  if (len) *len = t.size();
  if (!buf) return SIFT_OK;
  if (cap < t.size() + 1) return set_err(ctx, SIFT_E_CAPACITY, "destination too small");
  std::memcpy(buf, t.c_str(), t.size() + 1);
  return SIFT_OK;
}

int sift_copy_keypoints_device(sift_ctx* ctx, void* d_dst, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (n_out) *n_out = ctx->n_kp;
  if (!d_dst) return SIFT_OK;
  if (cap < ctx->n_kp) return set_err(ctx, SIFT_E_CAPACITY, "keypoint buffer too small");
  if (ctx->n_kp) {
    HIPCHK(hipSetDevice(ctx->device));
    // The keypoints are final (the detection was waited for): copy off the
    // context stream, so a detection queued behind them is not waited for.
    HIPCHK(hipMemcpy(d_dst, ctx->kp.p, ctx->n_kp * sizeof(sift_keypoint), hipMemcpyDeviceToDevice));
  }
  return SIFT_OK;
}

int sift_device_keypoints(sift_ctx* ctx, const sift_keypoint** d_kp, size_t* n) {
  if (!ctx || !d_kp || !n) return SIFT_E_ARG;
  *d_kp = ctx->kp.as<const sift_keypoint>();
  *n = ctx->n_kp;
  return SIFT_OK;
}

int sift_device_next_seed(sift_ctx* ctx, const double** d_seed, int* rows, int* cols) {
  if (!ctx || !d_seed) return SIFT_E_ARG;
  if (!ctx->has_xseed) return set_err(ctx, SIFT_E_STATE, "no next-octave base (SIFT_F_EXPORT_NEXT_SEED)");
  *d_seed = ctx->xseed.as<const double>();
  if (rows) *rows = ctx->xseed_h;
  if (cols) *cols = ctx->xseed_w;
  return SIFT_OK;
}

int sift_next_seed(sift_ctx* ctx, double* dst, size_t cap, int* rows, int* cols) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->has_xseed) return set_err(ctx, SIFT_E_STATE, "no next-octave base (SIFT_F_EXPORT_NEXT_SEED)");
  if (rows) *rows = ctx->xseed_h;
  if (cols) *cols = ctx->xseed_w;
  if (!dst) return SIFT_OK;
  const size_t n = (size_t)ctx->xseed_h * ctx->xseed_w;
  if (cap < n) return set_err(ctx, SIFT_E_CAPACITY, "destination too small");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(dst, ctx->xseed.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

static int detect_from_seed(sift_ctx* ctx, int o_first, const double* seed_host, const double* seed_dev, int W,
                            int H, const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out,
                            int scan_first = 0) {
  if (!ctx || !p) return SIFT_E_ARG;
  (void)hipSetDevice(ctx->device);
  if (ctx->detect_pending) return set_err(ctx, SIFT_E_STATE, "a detection is in flight on this context");
  if (o_first < 1) return set_err(ctx, SIFT_E_ARG, "octave_first must be >= 1");
  if (scan_first && (scan_first < o_first || scan_first >= p->num_octaves))
    return set_err(ctx, SIFT_E_ARG, "octave_scan_first outside [octave_first, num_octaves)");
  int rc = build_common(ctx, nullptr, nullptr, W, H, 0, p, nullptr, o_first, seed_host, seed_dev, false, 1, 0,
                        scan_first);
  if (rc) return rc;
  if (scan_first) ctx->scan_first = scan_first;
  rc = launch_extrema_stage(ctx);
  if (rc) return rc;
  rc = refine_enqueue(ctx);
  if (rc) return rc;
  ctx->detect_pending = true;
  ctx->detect_host_img = false;
  return detect_finish(ctx, out, cap, n_out);
}

int sift_detect_from_seed(sift_ctx* ctx, int octave_first, const double* seed, int width, int height,
                          const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out) {
  return detect_from_seed(ctx, octave_first, seed, nullptr, width, height, p, out, cap, n_out);
}

int sift_detect_from_seed_device(sift_ctx* ctx, int octave_first, const double* d_seed, int width, int height,
                                 const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out) {
  return detect_from_seed(ctx, octave_first, nullptr, d_seed, width, height, p, out, cap, n_out);
}

int sift_detect_from_seed_range_device(sift_ctx* ctx, int octave_first, int octave_scan_first, const double* d_seed,
                                       int width, int height, const sift_params* p, sift_keypoint* out, size_t cap,
                                       size_t* n_out) {
  return detect_from_seed(ctx, octave_first, nullptr, d_seed, width, height, p, out, cap, n_out,
                          std::max(octave_scan_first, octave_first));
}

int sift_merge_keypoint_blocks_device(sift_ctx* ctx, const sift_keypoint* d_in, const int64_t* counts, int n_parts,
                                      int n_blocks, sift_keypoint* d_out) {
  if (!ctx || !counts || n_parts < 1 || n_blocks < 1 || n_parts > 1024 || n_blocks > 4096) return SIFT_E_ARG;
  // Every (part, block) run is contiguous in d_in and in d_out: the merge is
  // one copy per non-empty run (seg = src, dst, bytes; cstart = first chunk).
  const int np = n_parts, nb = n_blocks;
  constexpr long long kRec = sizeof(sift_keypoint), kChunk = kMergeChunk;
  std::vector<long long> part_start((size_t)np + 1, 0);
  for (int q = 0; q < np; ++q) {
    long long a = 0;
    for (int b = 0; b < nb; ++b) {
      const long long c = counts[(size_t)q * nb + b];
      a += c < 0 ? -c : c;  // negative: skipped records (padding)
    }
    part_start[q + 1] = part_start[q] + a;
  }
  std::vector<long long> in_at(part_start.begin(), part_start.end() - 1);  // next record of each part
  std::vector<long long> seg, cstart;
  long long o = 0, chunks = 0;
  for (int b = 0; b < nb; ++b)
    for (int q = 0; q < np; ++q) {
      const long long c = counts[(size_t)q * nb + b];
      if (c <= 0) {
        in_at[q] -= c;
        continue;
      }
      seg.push_back(in_at[q] * kRec);
      seg.push_back(o * kRec);
      seg.push_back(c * kRec);
      cstart.push_back(chunks);
      chunks += (c * kRec + kChunk - 1) / kChunk;
      in_at[q] += c;
      o += c;
    }
  if (o == 0) return SIFT_OK;
  if (!d_in || !d_out) return SIFT_E_ARG;
  const int nseg = (int)cstart.size();
  std::vector<long long> tab(seg);
  tab.insert(tab.end(), cstart.begin(), cstart.end());
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(ctx->merge_tab.ensure(tab.size() * sizeof(long long)));
  // through the context's pinned staging (an asynchronous DMA; a pageable
  // source is copied through the runtime's own staging first)
  HIPCHK(ctx->hpl.ensure(tab.size() * sizeof(long long)));
  std::memcpy(ctx->hpl.p, tab.data(), tab.size() * sizeof(long long));
  HIPCHK(hipMemcpyAsync(ctx->merge_tab.p, ctx->hpl.p, tab.size() * sizeof(long long), hipMemcpyHostToDevice,
                        ctx->stream));
  HIPCHK(launch_merge_blocks(reinterpret_cast<const Keypoint*>(d_in), ctx->merge_tab.as<long long>(),
                             ctx->merge_tab.as<long long>() + 3 * (size_t)nseg, nseg, chunks,
                             reinterpret_cast<Keypoint*>(d_out), ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_order_after(sift_ctx* ctx, const sift_ctx* prev, int after) {
  if (!ctx || !prev) return SIFT_E_ARG;
  if (after < SIFT_AFTER_OCTAVE0 || after > SIFT_AFTER_REFINEMENT) return SIFT_E_ARG;
  if (ctx == prev || ctx->stream == prev->stream) return SIFT_OK;  // already ordered
  HIPCHK(hipSetDevice(ctx->device));
  // ev[7]: octave 0's Gaussian+DoG done; ev[2]: all octaves; ev_heavy: the
  // fast refinement (the rest is the latency-bound tail).
  const hipEvent_t e = after == SIFT_AFTER_OCTAVE0 ? prev->ev[7] : after == SIFT_AFTER_GAUSSIAN ? prev->ev[2]
                                                                                                 : prev->ev_heavy;
  HIPCHK(hipStreamWaitEvent(ctx->stream, e, 0));
  return SIFT_OK;
}

// ---- Image products either side of the path (sift_image.hip) -------------

static int check_rgba(sift_ctx* ctx, const void* rgba, int W, int H, size_t stride_bytes) {
  if (!ctx) return SIFT_E_ARG;
  if (!rgba || W <= 0 || H <= 0) return set_err(ctx, SIFT_E_ARG, "null or empty RGBA image");
  if (stride_bytes < (size_t)W * 4 || stride_bytes % 4) return set_err(ctx, SIFT_E_ARG, "bad RGBA row stride");
  return SIFT_OK;
}

// Upload the RGBA rows (dense) and convert them into ctx->img on ctx's stream.
static int rgba_to_ctx_img(sift_ctx* ctx, const uint8_t* rgba, int W, int H, size_t stride_bytes,
                           bool alpha = false) {
  int rc = check_rgba(ctx, rgba, W, H, stride_bytes);
  if (rc) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(ctx->rgba.ensure((size_t)W * H * 4));
  HIPCHK(ctx->img.ensure((size_t)W * H * sizeof(float)));
  if (stride_bytes == (size_t)W * 4 && host_registered(rgba, (size_t)W * H * 4))  // page-locked: one DMA
    HIPCHK(hipMemcpyAsync(ctx->rgba.p, rgba, (size_t)W * H * 4, hipMemcpyHostToDevice, ctx->stream));
  else
    HIPCHK(hipMemcpy2DAsync(ctx->rgba.p, (size_t)W * 4, rgba, stride_bytes, (size_t)W * 4, H, hipMemcpyHostToDevice,
                            ctx->stream));
  if (alpha) HIPCHK(ctx->alpha.ensure((size_t)W * H * sizeof(float)));
  HIPCHK(launch_rgba_to_gray(ctx->rgba.as<unsigned char>(), (size_t)W * 4, W, H, ctx->img.as<float>(),
                             alpha ? ctx->alpha.as<float>() : nullptr, ctx->stream));
  return SIFT_OK;
}

int sift_rgba_to_gray_device(sift_ctx* ctx, const uint8_t* d_rgba, int width, int height, size_t stride_bytes,
                             float* d_gray, float* d_alpha) {
  int rc = check_rgba(ctx, d_rgba, width, height, stride_bytes);
  if (rc) return rc;
  if (!d_gray) return set_err(ctx, SIFT_E_ARG, "null gray destination");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(launch_rgba_to_gray(d_rgba, stride_bytes, width, height, d_gray, d_alpha, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_rgba_to_gray(sift_ctx* ctx, const uint8_t* rgba, int width, int height, size_t stride_bytes, float* gray,
                      float* alpha) {
  if (ctx && !gray) return set_err(ctx, SIFT_E_ARG, "null gray destination");
  int rc = rgba_to_ctx_img(ctx, rgba, width, height, stride_bytes, alpha != nullptr);
  if (rc) return rc;
  const size_t n = (size_t)width * height;
  if (alpha) HIPCHK(hipMemcpyAsync(alpha, ctx->alpha.p, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(gray, ctx->img.p, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_build_scale_space_rgba(sift_ctx* ctx, const uint8_t* rgba, int width, int height, size_t stride_bytes,
                                const sift_params* p, const double* sig) {
  int rc = rgba_to_ctx_img(ctx, rgba, width, height, stride_bytes);
  if (rc) return rc;
  return sift_build_scale_space_device(ctx, ctx->img.as<float>(), width, height, (size_t)width, p, sig);
}

int sift_detect_rgba(sift_ctx* ctx, const uint8_t* rgba, int width, int height, size_t stride_bytes,
                     const sift_params* p, sift_keypoint* out, size_t cap, size_t* n_out) {
  int rc = rgba_to_ctx_img(ctx, rgba, width, height, stride_bytes);
  if (rc) return rc;
  return detect_common(ctx, nullptr, ctx->img.as<float>(), width, height, (size_t)width, p, out, cap, n_out);
}

static int plane_image_common(sift_ctx* ctx, int kind, int o, int s, int mode, double coef, uint8_t* dst,
                              size_t cap_bytes, bool host) {
  if (!ctx || !dst) return SIFT_E_ARG;
  if (ctx->dog_source == kNone) return set_err(ctx, SIFT_E_STATE, "no pyramid");
  if (mode < SIFT_DISPLAY_PLAIN || mode > SIFT_DISPLAY_SAMPLED) return set_err(ctx, SIFT_E_ARG, "bad display mode");
  const Pyramid& P = ctx->P;
  if (o < 0 || o >= P.O) return set_err(ctx, SIFT_E_ARG, "octave out of range");
  if (o < ctx->planes_first) return set_err(ctx, SIFT_E_STATE, "octave not built (sift_detect_from_seed[_range])");
  const Octave& oc = P.oct[o];
  const size_t plane = (size_t)oc.h * oc.w;
  if (cap_bytes < plane * 4) return set_err(ctx, SIFT_E_CAPACITY, "destination too small (4 bytes per pixel)");
  const float* src = nullptr;
  if (kind == SIFT_PLANE_GAUSS) {
    if (!ctx->have_gauss) return set_err(ctx, SIFT_E_STATE, "Gaussian planes not materialised");
    if (s < 0 || s >= P.NS) return set_err(ctx, SIFT_E_ARG, "scale out of range");
    src = ctx->gauss.as<float>() + oc.gauss_off + (size_t)s * plane;
  } else if (kind == SIFT_PLANE_DOG) {
    if (s < 0 || s >= P.ND) return set_err(ctx, SIFT_E_ARG, "scale out of range");
    src = ctx->dog.as<float>() + oc.dog_off + (size_t)s * plane;
  } else {
    return set_err(ctx, SIFT_E_ARG, "bad plane kind");
  }
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(ctx->mm_parts.ensure((size_t)plane_image_parts((long long)plane) * sizeof(float2)));
  unsigned* out = reinterpret_cast<unsigned*>(dst);
  if (host) {
    HIPCHK(ctx->display.ensure(plane * 4));
    out = ctx->display.as<unsigned>();
  }
  HIPCHK(launch_plane_image(src, (long long)plane, mode, coef, ctx->mm_parts.as<float2>(), out, ctx->stream));
  if (host) HIPCHK(hipMemcpyAsync(dst, out, plane * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_plane_image(sift_ctx* ctx, int kind, int octave, int scale, int mode, double coefficient, uint8_t* rgba,
                     size_t cap_bytes) {
  return plane_image_common(ctx, kind, octave, scale, mode, coefficient, rgba, cap_bytes, true);
}

int sift_plane_image_device(sift_ctx* ctx, int kind, int octave, int scale, int mode, double coefficient,
                            uint8_t* d_rgba, size_t cap_bytes) {
  return plane_image_common(ctx, kind, octave, scale, mode, coefficient, d_rgba, cap_bytes, false);
}

int sift_set_flags(sift_ctx* ctx, int flags) {
  if (!ctx) return SIFT_E_ARG;
  ctx->p.flags = flags;
  return SIFT_OK;
}

int sift_set_owned_rows(sift_ctx* ctx, int row_begin, int row_end) {
  if (!ctx) return SIFT_E_ARG;
  if (row_begin < 0) {
    ctx->own_lo = ctx->own_hi = -1;
    return SIFT_OK;
  }
  if (row_end >= 0 && row_end < row_begin) return set_err(ctx, SIFT_E_ARG, "row_end < row_begin");
  ctx->own_lo = row_begin;
  ctx->own_hi = row_end;
  return SIFT_OK;
}

int sift_last_block_counts(sift_ctx* ctx, int64_t* counts, int cap, int* n_blocks) {
  if (!ctx) return SIFT_E_ARG;
  const int n = (int)ctx->blk_counts.size();
  if (n_blocks) *n_blocks = n;
  if (!counts) return SIFT_OK;
  if (cap < n) return set_err(ctx, SIFT_E_CAPACITY, "destination too small (num_octaves * scales_per_octave)");
  for (int b = 0; b < n; ++b) counts[b] = ctx->blk_counts[b];
  return SIFT_OK;
}

int sift_set_row_origin(sift_ctx* ctx, int input_row0) {
  if (!ctx || input_row0 < 0) return SIFT_E_ARG;
  ctx->row0 = input_row0;
  return SIFT_OK;
}

int sift_copy_keypoint_origins_device(sift_ctx* ctx, int32_t* d_dst, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->has_origins) return set_err(ctx, SIFT_E_STATE, "no keypoint origins (SIFT_F_KEYPOINT_ORIGINS)");
  if (n_out) *n_out = ctx->n_kp;
  if (!d_dst || ctx->n_kp == 0) return SIFT_OK;
  if (cap < 4 * ctx->n_kp) return set_err(ctx, SIFT_E_CAPACITY, "destination too small (4 per keypoint)");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(launch_decode_origins(ctx->P, ctx->kp_key.as<unsigned>(), (int)ctx->n_kp, d_dst, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_copy_next_seed_device(sift_ctx* ctx, double* d_dst, size_t cap, int row_begin, int row_end) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->has_xseed) return set_err(ctx, SIFT_E_STATE, "no next-octave base (SIFT_F_EXPORT_NEXT_SEED)");
  if (row_begin < 0 || row_end > ctx->xseed_h || row_begin > row_end) return set_err(ctx, SIFT_E_ARG, "bad row range");
  const size_t n = (size_t)(row_end - row_begin) * ctx->xseed_w;
  if (!d_dst || n == 0) return SIFT_OK;
  if (cap < n) return set_err(ctx, SIFT_E_CAPACITY, "destination too small");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(d_dst, ctx->xseed.as<double>() + (size_t)row_begin * ctx->xseed_w, n * sizeof(double),
                        hipMemcpyDeviceToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return SIFT_OK;
}

int sift_keypoint_origins(sift_ctx* ctx, int32_t* out, size_t cap, size_t* n_out) {
  if (!ctx) return SIFT_E_ARG;
  if (!ctx->has_origins) return set_err(ctx, SIFT_E_STATE, "no keypoint origins (SIFT_F_KEYPOINT_ORIGINS)");
  if (n_out) *n_out = ctx->n_kp;
  if (!out || ctx->n_kp == 0) return SIFT_OK;
  if (cap < 4 * ctx->n_kp) return set_err(ctx, SIFT_E_CAPACITY, "destination too small (4 per keypoint)");
  HIPCHK(hipSetDevice(ctx->device));
  std::vector<unsigned> keys(ctx->n_kp);
  HIPCHK(hipMemcpyAsync(keys.data(), ctx->kp_key.p, keys.size() * sizeof(unsigned), hipMemcpyDeviceToHost,
                        ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const Pyramid& P = ctx->P;
  for (size_t i = 0; i < keys.size(); ++i) {  // key = key_off(o) + (s-1) h w + y w + x
    int o = P.O - 1;
    while (o > 0 && keys[i] < P.oct[o].key_off) --o;
    const Octave& oc = P.oct[o];
    const unsigned plane = (unsigned)oc.h * (unsigned)oc.w, r = keys[i] - oc.key_off;
    out[4 * i + 0] = o;
    out[4 * i + 1] = (int32_t)(r / plane) + 1;
    out[4 * i + 2] = (int32_t)((r % plane) / (unsigned)oc.w) + ((P.row0 * 2) >> o);
    out[4 * i + 3] = (int32_t)((r % plane) % (unsigned)oc.w);
  }
  return SIFT_OK;
}

}  // extern "C"
