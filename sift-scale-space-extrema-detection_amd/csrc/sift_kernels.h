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
  int base_lds;       // stage the replicated-edge base region in LDS
};

struct ExtremaLaunch {
  int o;
  int exact_planes;            // DoG planes are the data itself (caller-supplied): no fp32 ties
  unsigned* keys;              // candidate sort keys (unordered)
  unsigned long long* payload; // float bits << 32 | flags
  unsigned* counters;          // [0] emitted, [1] certain low-contrast
  unsigned cap;
};

struct CandInit {
  const unsigned* keys;              // sorted
  const unsigned long long* payload; // sorted alongside
  int n;
  unsigned* keep;     // out: 1 = candidate
  double* value;      // out: DoG value (exact fp64 where re-decided)
  unsigned* flagged;  // out: indices needing an exact decision
  unsigned* counters; // [2] n flagged, [1] low-contrast (exact decisions add here)
};

struct RefineLaunch {
  const unsigned* cand_key;
  const double* cand_val;
  int n;
  int exact_planes;
  double min_blur, min_interpixel_distance;
  int* status;        // per candidate kRef*
  Keypoint* kp;       // per candidate (valid where status == kRefKeep)
  unsigned* uncertain;// indices for the exact pass
  unsigned* counters; // [3] n uncertain, [4] n singular
};

size_t gauss_lds_bytes(const Octave& oc, bool base_lds);
hipError_t launch_gauss_dog(const Pyramid& P, const GaussLaunch& L, hipStream_t st);
hipError_t launch_dog_from_gauss(const float* g, float* d, long long plane, int nd, hipStream_t st);

hipError_t launch_extrema(const Pyramid& P, const ExtremaLaunch& L, hipStream_t st);
hipError_t launch_cand_init(const CandInit& C, hipStream_t st);
// One wave per flagged candidate: fp64 pointwise recompute of the 3x3x3 DoG patch.
hipError_t launch_exact_extrema(const Pyramid& P, const CandInit& C, unsigned n_flagged,
                                hipStream_t st);

hipError_t launch_refine_fast(const Pyramid& P, const RefineLaunch& R, hipStream_t st);
hipError_t launch_refine_exact(const Pyramid& P, const RefineLaunch& R, unsigned n_uncertain,
                               hipStream_t st);

// Order-preserving compaction helpers.
hipError_t launch_scatter_candidates(const unsigned* keep, const unsigned* pos, const unsigned* keys,
                                     const double* val, int n, unsigned* out_key, double* out_val,
                                     hipStream_t st);
hipError_t launch_scatter_keypoints(const int* status, const unsigned* pos, const Keypoint* kp,
                                    int n, Keypoint* out, hipStream_t st);
hipError_t launch_status_to_keep(const int* status, unsigned* keep, int n, hipStream_t st);

// Exact fp64 DoG patch for host-side checks (tests): d[27] for (o, s, y, x).
size_t exact_lds_bytes(const Pyramid& P);

}  // namespace sift
