// Shared device/host definitions for the gfx950 SIFT path.
//
// HBM layout (one context, one image):
//   img      fp32  H x W                 input (octave 0 base = its 2x NN upsample,
//                                        never materialised: read as img[y>>1][x>>1])
//   seed[o]  fp64  h_o x w_o, o >= 1     octave base = L[o-1][S][2i][2j] (background.js:114-118)
//   gauss    fp32  sum_o (S+3) h_o w_o   octave-major, scale, row-major
//   dog      fp32  sum_o (S+2) h_o w_o   D[t] = L[t] - L[t+1] formed in fp64, rounded once
//   wts      fp64  per (o,s): [PAD zeros][2r+1 normalised taps][PAD zeros]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

namespace sift {

// Experiment knobs: with -DSIFT_EXPERIMENTS (tools/build_variant.sh A/B
// builds) the named environment variable overrides the default; the shipping
// library (`make lib`) reads no environment and always takes the default,
// the measured winner.
inline int exp_knob(const char* name, int dflt) {
#ifdef SIFT_EXPERIMENTS
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

constexpr int kMaxOctaves = 12;
constexpr int kMaxScales = 12;   // S+3 <= kMaxScales  (S <= 9)
constexpr int kWPad = 16;        // zero taps on both sides of every weight vector

// fp64 in the constant address space: uniform indices become scalar loads.
typedef __attribute__((address_space(4))) const double cdouble;

// Per-octave geometry, passed by value in kernel arguments.
struct Octave {
  int h, w;
  long long gauss_off;   // element offset of plane (o, 0) in gauss
  long long dog_off;     // element offset of plane (o, 0) in dog
  long long seed_off;    // element offset of this octave's base in seeds (o >= 1)
  unsigned key_off;      // sum_{o' < o} S * h_o' * w_o'  (candidate sort keys)
  int wofs[kMaxScales];  // offset of tap 0 of scale s in wts (PAD zeros precede it)
  int rad[kMaxScales];   // radius of scale s (0 = un-blurred copy)
  int rmax;
  long long l64_off;     // element offset of plane (o, 0) in l64 (fp64 Gaussian planes), -1 = not kept
};

struct Pyramid {
  int O, S, NS, ND;      // octaves, scales per octave, S+3, S+2
  int W, H, img_stride;  // input
  const float* img;
  const double* seeds;
  const double* wts;
  const float* dog;
  const double* l64;     // fp64 Gaussian planes of the octaves built by the wide-radius path (l64_off >= 0)
  double pix_thr;        // 0.8 * thr   (sift.js:285-294)
  double thr;            // thr         (background.js:572)
  int row0;              // input row of the input's first row (a row-band crop; 0 = whole image)
  // A batch of nimg independent images of the same geometry (sift_detect_batch_device):
  // image b's input, seeds, DoG and fp64 planes start b * *_bstride elements
  // after image 0's, and its candidate keys b * kpi after (keys per image).
  int nimg;
  unsigned kpi;
  long long img_bstride, seed_bstride, dog_bstride, l64_bstride;
  // The split vertical pass's fp64 scratch (k_gauss_vert) as the pass left
  // it: the vertical sums of every (scale, row, column) of octave vsum_oct
  // (the last split octave; -1 = none), image b at b * vsum_bstride.  The
  // exact passes read their patches' vertical sums from it.
  const double* vsum;
  long long vsum_bstride;
  int vsum_oct;
  Octave oct[kMaxOctaves];
};

// Base pixel of octave o of image b at (y, x), coordinates already clamped to the plane.
__device__ __forceinline__ double base_at(const Pyramid& P, int b, int o, int y, int x) {
  if (o == 0) return (double)P.img[b * P.img_bstride + (long long)(y >> 1) * P.img_stride + (x >> 1)];
  return P.seeds[b * P.seed_bstride + P.oct[o].seed_off + (long long)y * P.oct[o].w + x];
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Candidate sort key -> (image, octave, scale, y, x): key = b kpi + the
// image-local key of (o, s, y, x).
__device__ __forceinline__ void decode_key(const Pyramid& P, unsigned key, int& b, int& o, int& s, int& y,
                                           int& x) {
  b = 0;
  if (P.nimg > 1) {
    b = (int)(key / P.kpi);
    key -= (unsigned)b * P.kpi;
  }
  o = 0;
  while (o + 1 < P.O && key >= P.oct[o + 1].key_off) ++o;
  unsigned r = key - P.oct[o].key_off;
  const unsigned plane = (unsigned)P.oct[o].h * (unsigned)P.oct[o].w;
  s = (int)(r / plane) + 1;
  r -= (unsigned)(s - 1) * plane;
  y = (int)(r / (unsigned)P.oct[o].w);
  x = (int)(r - (unsigned)y * (unsigned)P.oct[o].w);
}

// Extremum record flags.
enum : unsigned {
  kFlagTie = 1u,       // an fp32 neighbour equals the centre: re-decide in fp64
  kFlagContrast = 2u,  // |v| within fp32 rounding of 0.8*thr: re-decide in fp64
};

// Refinement status.
enum : int {
  kRefDiscard = 0,
  kRefKeep = 1,
  kRefUncertain = 2,  // a decision fell within the fp32-plane error bound: redo exactly
  kRefSingular = 3,
};

}  // namespace sift
