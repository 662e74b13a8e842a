// Launch interfaces of the gfx950 SIFT kernels (internal to libsift_hip.so).
#pragma once
#include <algorithm>

#include "sift_common.h"

namespace sift {

// Device twin of sift_keypoint (include/sift_hip.h), same 48-byte layout.
struct Keypoint {
  int32_t octave, scale_level, local_x, local_y;
  double abs_x, abs_y, abs_sigma, interp_value;
};

struct GaussLaunch {
  int o;
  float* gauss;       // plane (o, 0) of the Gaussian pyramid, nullptr = do not store
  float* dog;         // plane (o, 0) of the DoG pyramid
  double* next_seed;  // base of octave o+1 (nullptr for the last octave)
  int next_w;
};

constexpr int kXStrip = 64;  // rows per wave in the extrema scan
constexpr int kXG = 4;       // rows fetched per group in the extrema scan

struct ExtremaLaunch {
  int o;
  int exact_planes;              // DoG planes are the data itself (caller-supplied): no fp32 ties
  unsigned long long* bitmap;    // this octave's candidate bitmap [S][h][nw]
  int nw;                        // 64-pixel words per row
  unsigned* rowcount;            // this octave's candidates per (scale, row) [S][h]
  unsigned* amb_keys;            // keys needing an exact fp64 decision (unordered)
  unsigned* counters;            // [0] ambiguous, [1] low-contrast, [2] dropped by exact pass
  unsigned amb_cap;
};

struct EmitLaunch {
  int o;
  const unsigned long long* bitmap;
  int nw;
  const unsigned* rowcount;      // this octave's [S][h]
  const unsigned* rowoff;        // exclusive scan over all octaves' row counts
  int row_base;                  // index of this octave's first row in rowoff
  unsigned* keys;                // ordered candidate keys
  double* value;
  unsigned* keep;
};

struct ExactLaunch {
  const unsigned* amb_keys;
  const unsigned* keys;          // ordered candidates
  unsigned n;
  unsigned* keep;
  double* value;
  unsigned* counters;
};

struct RefineLaunch {
  const unsigned* cand_key;
  const double* cand_val;
  const unsigned* keep;  // nullptr = every entry is a candidate
  int n;
  int exact_planes;
  double min_blur, min_interpixel_distance;
  int* status;        // per candidate kRef*
  Keypoint* kp;       // per candidate (valid where status == kRefKeep)
  unsigned* uncertain;// indices for the exact pass
  unsigned* counters; // [3] n uncertain, [4] n singular
};

size_t gauss_lds_bytes(const Pyramid& P, int o);
hipError_t launch_gauss_dog(const Pyramid& P, const GaussLaunch& L, hipStream_t st);
hipError_t launch_dog_from_gauss(const float* g, float* d, long long plane, int nd, hipStream_t st);

hipError_t launch_extrema(const Pyramid& P, const ExtremaLaunch& L, hipStream_t st);
hipError_t launch_emit(const Pyramid& P, const EmitLaunch& E, hipStream_t st);
// One wave per ambiguous candidate: fp64 pointwise recompute of the 3x3x3 DoG patch.
hipError_t launch_exact_extrema(const Pyramid& P, const ExactLaunch& X, unsigned n_amb, hipStream_t st);

hipError_t launch_refine_fast(const Pyramid& P, const RefineLaunch& R, hipStream_t st);
hipError_t launch_refine_exact(const Pyramid& P, const RefineLaunch& R, unsigned n_uncertain,
                               hipStream_t st);

// Order-preserving compaction helpers.
hipError_t launch_scatter_keypoints(const int* status, const unsigned* pos, const Keypoint* kp,
                                    int n, Keypoint* out, hipStream_t st);
hipError_t launch_status_to_keep(const int* status, unsigned* keep, int n, hipStream_t st);

size_t exact_lds_bytes(const Pyramid& P);

}  // namespace sift
