// Sub-pixel quadratic refinement with contrast and edge rejection (gfx950).
//
// Replaces refineCandidateKeypoints (background.js:455-685) with its helpers
// SIFT_generateGradientVector / SIFT_generateHessianMatrix (sift.js:333-446)
// and the 3x3 adjugate inverse (matrix2d.js:197-546).  The arithmetic is
// written in the reference's exact operation order with FP contraction off,
// so on the same fp64 inputs it rounds exactly as the JS does.  Quirks kept:
// omega uses the ORIGINAL candidate value (:565); tr^2/det < 0 and NaN pass
// the edge test (:599); Math.round ties go to +inf (:638-640); duplicates
// are kept; |det| < DBL_EPSILON is reported as singular (the reference
// throws a TypeError there, matrix2d.js:482 -> :455).
//
// k_refine_fast: one thread per candidate, reading the fp32 DoG planes.  A
// first-order bound of the fp32 rounding error is carried through every
// decision; a decision inside its bound marks the candidate uncertain and
// k_refine_exact redoes it from an fp64 pointwise recompute (sift_exact.h).
// With caller-supplied planes (exact_planes) the fp32 values ARE the data,
// the bound is zero and the fast pass is exact.
#include "sift_exact.h"
#include "sift_kernels.h"

#pragma clang fp contract(off)

namespace sift {

__device__ __forceinline__ double js_round(double v) {
  const double f = floor(v);
  return (v - f >= 0.5) ? f + 1.0 : f;
}

// Distance of v from the nearest Math.round decision point (k + 0.5).
__device__ __forceinline__ double round_margin(double v) {
  const double f = v - floor(v);
  return fabs(f - 0.5);
}

struct StepOut {
  int state;         // 0 continue (moved), 1 keep, 2 discard, 3 singular
  bool uncertain;
  unsigned why;      // diagnostic: which decisions were uncertain (bits 0..6)
  double a[3];
  double omega;
  bool imprecise;    // kept, but its (x, y, sigma) or value may be off by more than kKeypointTol / kValueTol
  int s, m, n;       // position after the step (moved) or of the keypoint
};

// Largest error of a kept keypoint's absolute (x, y, sigma) that the fast
// pass may leave (the parity bar is 1e-4; the bounds below are first-order
// with a factor kSafe of slack).  The absolute coordinates scale the offset
// alpha by 2^(o-1) -- 16 at octave 5 of an 8K pyramid, where the DoG values
// are small and fp32 rounding of the planes moves alpha by ~1e-5 -- so a
// keypoint whose bound exceeds this is recomputed from exact fp64 patches.
#ifndef SIFT_KP_TOL
#define SIFT_KP_TOL 2e-5
#endif
constexpr double kKeypointTol = SIFT_KP_TOL;
constexpr double kValueTol = 1e-7;  // interpolatedValue (the tests hold it to 1e-6)
constexpr unsigned kPolish = 0x80000000u;  // uncertain-list entry: exact values at the final position only

// One iteration of background.js:480-664 on the patch d[k][a][c]
// (k: scale s-1+k, a: row m-1+a, c: col n-1+c).  `delta` bounds the error of
// every patch value (0 = exact), `dval` that of the candidate value.  With
// delta > 0 every decision carries an error bound: gradient entries are off
// by <= delta, Hessian entries by <= 4 delta (diagonal worst case); the
// inverse is bounded through ||H^-1 E|| <= kappa < 1/2 (perturbation lemma),
// and each bound gets a factor kSafe of slack.  A decision inside its bound
// sets `uncertain`.  On the last iteration (`last`) a move discards, so the
// new position's rounding does not matter.
// APPROX (fast pass on fp32 planes only): the inverse uses one reciprocal
// instead of nine divisions.  Its extra rounding (~1e-16 relative) is far
// inside the fp32-plane error bounds every decision already carries; the
// exact pass and caller-supplied planes (delta == 0) keep the reference's
// divisions.
// sig0 = min_blur / min_interpixel_distance (abs_sigma = 2^(o-1) sig0 2^((a0+s)/S)).
template <bool APPROX>
__device__ inline StepOut refine_step(const double* d, int o, int s, int m, int n, double value,
                                      double delta, double dval, int S, int ND, int h, int w,
                                      double thr, bool last, double sig0) {
  constexpr double kSafe = 2.0;
#define DP(k, a, c) d[(k) * 9 + (a) * 3 + (c)]
  StepOut R;
  R.uncertain = false;
  R.why = 0;
  R.imprecise = false;
  const double cc = DP(1, 1, 1);
  const double g0 = (DP(2, 1, 1) - DP(0, 1, 1)) / 2;
  const double g1 = (DP(1, 2, 1) - DP(1, 0, 1)) / 2;
  const double g2 = (DP(1, 1, 2) - DP(1, 1, 0)) / 2;
  const double h11 = DP(2, 1, 1) + DP(0, 1, 1) - (2 * cc);
  const double h22 = DP(1, 2, 1) + DP(1, 0, 1) - (2 * cc);
  const double h33 = DP(1, 1, 2) + DP(1, 1, 0) - (2 * cc);
  const double h12 = (DP(2, 2, 1) - DP(2, 0, 1) - DP(0, 2, 1) + DP(0, 0, 1)) / 4;
  const double h13 = (DP(2, 1, 2) - DP(2, 1, 0) - DP(0, 1, 2) + DP(0, 1, 0)) / 4;
  const double h23 = (DP(1, 2, 2) - DP(1, 2, 0) - DP(1, 0, 2) + DP(1, 0, 0)) / 4;
#undef DP
  const double M[3][3] = {{h11, h12, h13}, {h12, h22, h23}, {h13, h23, h33}};
  double mn[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int r0 = i == 0 ? 1 : 0, r1 = i == 2 ? 1 : 2;
      const int c0 = j == 0 ? 1 : 0, c1 = j == 2 ? 1 : 2;
      mn[i][j] = (M[r0][c0] * M[r1][c1]) - (M[r0][c1] * M[r1][c0]);
    }
  const double det = ((M[0][0] * mn[0][0]) - (M[0][1] * mn[0][1])) + (M[0][2] * mn[0][2]);
  const double dG = delta, dH = 4 * delta;
  if (delta > 0) {
    double cof1 = 0, hmax = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        cof1 += fabs(mn[i][j]);
        hmax = fmax(hmax, fabs(M[i][j]));
      }
    // d det <= sum |cofactor| dH + second order (3 (2 hmax + dH) dH^2 ... )
    const double Edet = kSafe * (cof1 * dH + 9 * (2 * hmax + dH) * dH * dH) + 1e-300;
    if (fabs(fabs(det) - 2.220446049250313e-16) <= Edet) R.uncertain = true, R.why |= 1;
  }
  if (fabs(det) < 2.220446049250313e-16) {
    R.state = 3;
    return R;
  }
  double ninv[3][3];
  double inv_norm = 0;
  const double rdet = APPROX ? 1.0 / det : 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double rs = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double cof = ((i + j) & 1) ? mn[j][i] * -1.0 : mn[j][i];
      ninv[i][j] = (APPROX ? cof * rdet : cof / det) * -1;
      rs += fabs(ninv[i][j]);
    }
    inv_norm = fmax(inv_norm, rs);
  }
  const double gv[3] = {g0, g1, g2};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double r = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) r += ninv[i][j] * gv[j];
    R.a[i] = r;
  }
  const double a1 = fabs(R.a[0]) + fabs(R.a[1]) + fabs(R.a[2]);
  // |d alpha| <= ||H^-1|| (dG + ||E|| |alpha|) / (1 - kappa),  ||E||_inf <= 3 dH.
  double Ea = 0.0;
  if (delta > 0) {
    const double kappa = inv_norm * 3 * dH;
    if (kappa >= 0.5) {
      R.uncertain = true, R.why |= 2;
      Ea = 1e300;
    } else {
      Ea = kSafe * inv_norm * (dG + 3 * dH * a1) / (1 - kappa) + 1e-300;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (fabs(fabs(R.a[i]) - 0.6) <= Ea) R.uncertain = true, R.why |= 2;
  }
  if (fabs(R.a[0]) < 0.6 && fabs(R.a[1]) < 0.6 && fabs(R.a[2]) < 0.6) {
    const double omega = value + (((0.5 * R.a[0]) * g0) + ((0.5 * R.a[1]) * g1) + ((0.5 * R.a[2]) * g2));
    R.omega = omega;
    R.s = s; R.m = m; R.n = n;
    if (delta > 0) {
      // Output precision, componentwise: d alpha = -H^-1 (dg + dH alpha) to
      // first order, with |dg_j| <= dG, |dH_jj| <= dH, |dH_jk| <= dG (k != j);
      // abs (x, y) move by 2^(o-1) d alpha, abs_sigma by abs_sigma (ln 2 / S)
      // d alpha_0, omega = value + 0.5 alpha . g by the rest.
      const double kappa = inv_norm * 3 * dH;
      double r[3], e[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) r[j] = dG + dH * fabs(R.a[j]) + dG * (a1 - fabs(R.a[j]));
#pragma unroll
      for (int i = 0; i < 3; ++i)
        e[i] = kSafe * (fabs(ninv[i][0]) * r[0] + fabs(ninv[i][1]) * r[1] + fabs(ninv[i][2]) * r[2]) / (1 - kappa);
      const double dlt = ldexp(1.0, o - 1);
      const double e_xy = dlt * fmax(e[1], e[2]);
      // 2^((a0 + s) / S) < 2^((S + 0.6) / S) <= 2^1.6 < 3.04
      const double e_sig = dlt * sig0 * 3.04 * (0.6931471805599453 / S) * e[0];
      const double e_val = kSafe * (dval + 0.5 * (e[0] * fabs(g0) + e[1] * fabs(g1) + e[2] * fabs(g2) +
                                                  (a1 + e[0] + e[1] + e[2]) * dG));
      R.imprecise = fmax(e_xy, e_sig) > kKeypointTol || e_val > kValueTol;
    }
    if (delta > 0 || dval > 0) {
      const double Eo = kSafe * (dval + 0.5 * (Ea * (fabs(g0) + fabs(g1) + fabs(g2)) + (a1 + 3 * Ea) * dG)) + 1e-300;
      if (fabs(fabs(omega) - thr) <= Eo) R.uncertain = true, R.why |= 4;
    }
    if (fabs(omega) < thr) { R.state = 2; return R; }
    const double tr = (0 + h22) + h33;
    const double dt = (h22 * h33) - (h23 * h23);
    const double edgeness = (tr * tr) / dt;
    if (delta > 0) {
      // Interval bound on tr^2/det2: |dtr| <= 2 dH, |ddet2| <= (|h22|+|h33|) dH + 2|h23| dG + dH^2 + dG^2.
      const double Etr = kSafe * 2 * dH;
      const double Edt = kSafe * ((fabs(h22) + fabs(h33)) * dH + 2 * fabs(h23) * dG + dH * dH + dG * dG) + 1e-300;
      if (fabs(dt) <= Edt) {
        R.uncertain = true;
        R.why |= 8;
      } else {
        const double t_hi = fabs(tr) + Etr, t_lo = fmax(0.0, fabs(tr) - Etr);
        const double d_lo = fabs(dt) - Edt, d_hi = fabs(dt) + Edt;
        double e_lo, e_hi;
        if (dt > 0) { e_lo = t_lo * t_lo / d_hi; e_hi = t_hi * t_hi / d_lo; }
        else { e_lo = -(t_hi * t_hi / d_lo); e_hi = -(t_lo * t_lo / d_hi); }
        if (e_lo <= 12.1 && 12.1 <= e_hi) R.uncertain = true, R.why |= 16;
      }
    }
    if (edgeness > ((10 + 1) * (10 + 1)) / 10.0) { R.state = 2; return R; }
    R.state = 1;
    return R;
  }
  if (last) {  // the reference gives up after 5 moves: discard wherever it lands
    R.state = 2;
    return R;
  }
  const double vs = s + R.a[0], vm = m + R.a[1], vn = n + R.a[2];
  if (delta > 0 && (round_margin(vs) <= Ea || round_margin(vm) <= Ea || round_margin(vn) <= Ea)) {
    // Rounding is monotone: if every position within the bound leaves the
    // refinable interior in some coordinate, the move discards either way.
    const bool out_s = js_round(vs + Ea) < 1 || js_round(vs - Ea) >= ND - 1;
    const bool out_m = js_round(vm + Ea) < 1 || js_round(vm - Ea) >= h - 1;
    const bool out_n = js_round(vn + Ea) < 1 || js_round(vn - Ea) >= w - 1;
    if (!(out_s || out_m || out_n)) R.uncertain = true, R.why |= 32;
  }
  R.s = (int)js_round(vs);
  R.m = (int)js_round(vm);
  R.n = (int)js_round(vn);
  if (R.s < 1 || R.s >= ND - 1 || R.m < 1 || R.m >= h - 1 || R.n < 1 || R.n >= w - 1) {
    R.state = 2;
    return R;
  }
  R.state = 0;
  return R;
}

// moff: octave-row offset of a row-band crop (P.row0 in octave-o rows), so
// local_y and abs_y are those of the whole image: delta (a1 + m) with the
// image row m, the reference's own rounding.
__device__ inline void make_keypoint(Keypoint& k, int o, const StepOut& R, int S, double min_blur,
                                     double mid, int moff) {
  const double delta = ldexp(1.0, o - 1);  // Math.pow(2, octave - 1), exact
  k.octave = o;
  k.scale_level = R.s;
  k.local_x = R.n;
  k.local_y = R.m + moff;
  k.abs_y = delta * (R.a[1] + (R.m + moff));
  k.abs_x = delta * (R.a[2] + R.n);
  k.abs_sigma = (delta / mid) * min_blur * pow(2.0, (R.a[0] + R.s) / S);
  k.interp_value = R.omega;
}

#ifndef SIFT_REFINE_XCD
#define SIFT_REFINE_XCD 1
#endif
// Candidates are in raster order per (octave, scale), so neighbouring slots
// gather overlapping DoG lines.  Blocks are dispatched round-robin over the
// 8 XCDs (separate L2s): block b runs the logical block of a contiguous range
// per XCD, so those shared lines hit in one L2 instead of being fetched by
// every XCD.  A bijection over the live blocks (the count is on the device).
__device__ __forceinline__ int xcd_block(int b, int nb) {
  constexpr int kXcd = 8;
  const int q = nb / kXcd, r = nb % kXcd, x = b % kXcd;
  return x * q + min(x, r) + b / kXcd;
}

// EXACT: caller-supplied planes (the fp32 values are the data, no error
// bound); one instantiation per mode keeps the register allocation of the
// common fp32-plane path to its own code.
template <bool EXACT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_refine_fast(const Pyramid P,
                                                                                           const RefineLaunch L) {
  const int n = (int)min(*L.n, (unsigned)L.cap);
  const int nb = (n + 255) / 256;
  if ((int)blockIdx.x >= nb) return;  // whole block past the live slots
  const int t = (SIFT_REFINE_XCD ? xcd_block(blockIdx.x, nb) : (int)blockIdx.x) * 256 + threadIdx.x;
  const int i = (L.perm && t < n) ? min((int)L.perm[t], n - 1) : t;
  bool unc = false, polish = false;
  if (i < n && L.keep && !L.keep[i]) {
    L.status[i] = kRefDiscard;
  } else if (i < n) {
    int im, o, s, m, n;
    decode_key(P, L.cand_key[i], im, o, s, m, n);
    const Octave& oc = P.oct[o];
    const int h = oc.h, w = oc.w;
    const long long plane = (long long)h * w;
    const float* __restrict__ D = P.dog + im * P.dog_bstride + oc.dog_off;
    // the first step's patch as captured by the scan (kPatchFloats layout), if any
    const unsigned pidx = L.cand_patch ? L.cand_patch[i] : ~0u;
    const float* __restrict__ pp = L.patch + (size_t)(pidx == ~0u ? 0u : pidx) * kPatchFloats;
    double value = L.cand_val[i];
    if (value != value)  // deferred: the fp32 plane value
      value = pidx != ~0u ? (double)pp[4] : (double)D[s * plane + (long long)m * w + n];
    const double dval = EXACT ? 0.0 : fabs(value) * 0x1p-24;
    int status = kRefDiscard;
    double d[27];
    for (int it = 0; it < 5; ++it) {
      double mx = 0;
      if (it == 0 && pidx != ~0u) {
        const float4 c0 = *reinterpret_cast<const float4*>(pp), c1 = *reinterpret_cast<const float4*>(pp + 4);
        const float4 lf = *reinterpret_cast<const float4*>(pp + 8), rt = *reinterpret_cast<const float4*>(pp + 12);
        const float4 ex = *reinterpret_cast<const float4*>(pp + 16);
        const float v19[19] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, ex.x,  // d(k, a, 1), 3k + a
                               lf.x, lf.y, lf.z, lf.w, ex.y, rt.x, rt.y, rt.z, rt.w, ex.z};
        constexpr int at[19] = {1, 4, 7, 10, 13, 16, 19, 22, 25, 9, 12, 15, 3, 21, 11, 14, 17, 5, 23};
#pragma unroll
        for (int j = 0; j < 27; ++j) d[j] = 0.0;
#pragma unroll
        for (int j = 0; j < 19; ++j) {
          d[at[j]] = (double)v19[j];
          mx = fmax(mx, fabs((double)v19[j]));
        }
      } else {
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            // The 8 corners (k, a, c all != 1) enter neither the gradient nor
            // the Hessian (sift.js:333-446): 19 loads, and the error bound is
            // taken over the values that are used.
            if (k != 1 && a != 1 && c != 1) {
              d[k * 9 + a * 3 + c] = 0.0;
              continue;
            }
            const double v = (double)D[(s - 1 + k) * plane + (long long)(m - 1 + a) * w + (n - 1 + c)];
            d[k * 9 + a * 3 + c] = v;
            mx = fmax(mx, fabs(v));
          }
      }
      // fp32 rounding of the fp64 value (<= |v| 2^-24) plus fp64 noise vs the reference.
      const double delta = EXACT ? 0.0 : mx * (0x1p-24 + 0x1p-40);
      const StepOut R = refine_step<!EXACT>(d, o, s, m, n, value, delta, dval, P.S, P.ND, h, w, P.thr, it == 4,
                                            L.min_blur / L.min_interpixel_distance);
      if (R.uncertain) {
        unc = true;
        for (int b = 0; b < 6; ++b)
          if ((R.why >> b) & 1u) atomicAdd(&L.counters[16 + b], 1u);
        atomicAdd(&L.counters[22 + min(it, 4)], 1u);
        break;
      }
      if (R.state == 3) { status = kRefSingular; break; }
      if (R.state == 2) { status = kRefDiscard; break; }
      if (R.state == 1) {
        if (R.imprecise) {  // decisions certain, output not precise enough: exact values at this position
          unc = polish = true;
          Keypoint& k = L.kp[i];  // the final position for the exact pass (it rewrites the record)
          k.scale_level = s;
          k.local_y = m;
          k.local_x = n;
          atomicAdd(&L.counters[27], 1u);
          break;
        }
        status = kRefKeep;
        make_keypoint(L.kp[i], o, R, P.S, L.min_blur, L.min_interpixel_distance, (P.row0 * 2) >> o);
        break;
      }
      s = R.s; m = R.m; n = R.n;
    }
    L.status[i] = unc ? kRefUncertain : status;
    if (!unc && status == kRefSingular) atomicAdd(&L.counters[4], 1u);
  }
  const unsigned long long mask = __ballot(unc);
  if (mask) {
    const int leader = __ffsll((long long)mask) - 1;
    unsigned base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&L.counters[3], (unsigned)__popcll(mask));
    base = __shfl(base, leader);
    const unsigned pre = __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    if (unc) L.uncertain[base + pre] = (unsigned)i | (polish ? kPolish : 0u);
  }
}

// One block of NT threads per uncertain candidate (persistent over the
// device-side count): exact fp64 patches (dog_patch, the block's threads
// share each patch's vertical chains), thread 0 decides.  NT = 64 (one wave)
// for whole-image detections, whose exact pass runs beside other images'
// kernels (4K pipelined: 7.18-7.27 vs 7.06-7.16 Gpix/s with 256); NT = 256
// where it is alone on the critical path (the tail pieces of a sharded image,
// RefineLaunch::wide_exact): at radius 47 one wave's lanes walk ~15 chains of
// 95 dependent loads in turn (4K isolated 117 vs 60 us).  Polish entries (kPolish: every
// decision of the fast pass was certain, only the kept keypoint's output was
// not precise enough) recompute just the candidate's exact value (omega uses
// it, background.js:565) and the final position's patch.
template <int NT>
__global__ __launch_bounds__(NT) void k_refine_exact(const Pyramid P, const RefineLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int pos[4];
  const unsigned nu = min(L.counters[3], (unsigned)L.cap);
  for (unsigned j = blockIdx.x; j < nu; j += gridDim.x) {
    const unsigned e = L.uncertain[j];
    const unsigned i = e & ~kPolish;
    int im, o, s, m, n;
    decode_key(P, L.cand_key[i], im, o, s, m, n);
    const Octave& oc = P.oct[o];
    double* d27 = smem;
    double* Lbuf = smem + 32;
    double* sh = smem + 32 + 40;
    double value = 0;
    int status = kRefDiscard;
    if (e & kPolish) {
      dog_patch<NT>(P, im, o, s, m, n, sh, Lbuf, d27);
      value = d27[13];  // all lanes: d27 is visible after the patch's barrier
      const Keypoint& k = L.kp[i];
      const int s1 = k.scale_level, m1 = k.local_y, n1 = k.local_x;
      if (s1 != s || m1 != m || n1 != n) dog_patch<NT>(P, im, o, s1, m1, n1, sh, Lbuf, d27);
      if (threadIdx.x == 0) {
        const StepOut R = refine_step<false>(d27, o, s1, m1, n1, value, 0.0, 0.0, P.S, P.ND, oc.h, oc.w, P.thr,
                                             false, 0.0);
        pos[3] = R.state == 1;
        if (R.state == 1) make_keypoint(L.kp[i], o, R, P.S, L.min_blur, L.min_interpixel_distance, (P.row0 * 2) >> o);
      }
      __syncthreads();
      const bool done = pos[3];
      __syncthreads();
      if (done) {
        if (threadIdx.x == 0) L.status[i] = kRefKeep;
        continue;
      }
      // not kept on exact values (cannot happen with certain decisions): the whole chain
    }
    for (int it = 0; it < 5; ++it) {
      dog_patch<NT>(P, im, o, s, m, n, sh, Lbuf, d27);
      if (threadIdx.x == 0) {
        if (it == 0) value = d27[13];  // exact fp64 candidate value (:565 uses it)
        const StepOut R = refine_step<false>(d27, o, s, m, n, value, 0.0, 0.0, P.S, P.ND, oc.h, oc.w, P.thr, it == 4,
                                             0.0);
        int cont = 0;
        if (R.state == 3) status = kRefSingular;
        else if (R.state == 2) status = kRefDiscard;
        else if (R.state == 1) {
          status = kRefKeep;
          make_keypoint(L.kp[i], o, R, P.S, L.min_blur, L.min_interpixel_distance, (P.row0 * 2) >> o);
        } else {
          cont = 1;
          pos[0] = R.s; pos[1] = R.m; pos[2] = R.n;
        }
        pos[3] = cont;
      }
      __syncthreads();
      const int cont = pos[3];
      s = pos[0]; m = pos[1]; n = pos[2];
      __syncthreads();
      if (!cont) break;
    }
    if (threadIdx.x == 0) {
      L.status[i] = status;
      if (status == kRefSingular) atomicAdd(&L.counters[4], 1u);
    }
  }
}

// Block of a key: (image, octave, scale), image-major.
__device__ __forceinline__ int key_block(const Pyramid& P, unsigned key) {
  int im, o, s, y, x;
  decode_key(P, key, im, o, s, y, x);
  return (im * P.O + o) * P.S + (s - 1);
}

__global__ __launch_bounds__(256) void k_status_to_keep(const Pyramid P, const int* __restrict__ status,
                                                        const unsigned* __restrict__ key,
                                                        unsigned* __restrict__ keep, const unsigned* __restrict__ n,
                                                        int cap, int own_lo, int own_hi,
                                                        unsigned* __restrict__ blk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cap) return;
  const int m = (int)min(*n, (unsigned)cap);
  bool k = false;
  if (i < m) {
    int im, o, s, y, x;
    decode_key(P, key[i], im, o, s, y, x);
    const int b = (im * P.O + o) * P.S + (s - 1), nb = P.nimg * P.O * P.S;
    k = status[i] == kRefKeep;
    if (k && own_lo >= 0) {  // row-band ownership by candidate row (octave o rows: 2 r at o = 0, r >> (o-1))
      const int yw = y + ((P.row0 * 2) >> o);
      const int lo = o == 0 ? 2 * own_lo : own_lo >> (o - 1);
      const int hi = own_hi < 0 ? 0x7fffffff : (o == 0 ? 2 * own_hi : own_hi >> (o - 1));
      k = yw >= lo && yw < hi;
    }
    // block starts: slot i opens blocks (block(i-1), block(i)]; no atomics (a
    // per-block counter would serialise ~10^4 same-address atomics)
    const int bp = i == 0 ? -1 : key_block(P, key[i - 1]);
    if (b < bp) blk[kBlkUnsorted] = 1u;
    for (int q = bp + 1; q <= b; ++q) blk[kBlkStart + q] = (unsigned)i;
    if (i == m - 1)
      for (int q = max(b, bp) + 1; q <= nb; ++q) blk[kBlkStart + q] = (unsigned)m;
  }
  keep[i] = k ? 1u : 0u;
}

// keep: k_status_to_keep's flags (kept keypoint, in the owned rows).
__global__ __launch_bounds__(256) void k_scatter_kp(const unsigned* __restrict__ keep,
                                                    const unsigned* __restrict__ pos,
                                                    const Keypoint* __restrict__ kp,
                                                    const unsigned* __restrict__ n, int cap,
                                                    Keypoint* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < cap && i < (int)min(*n, (unsigned)cap) && keep[i]) out[pos[i]] = kp[i];
}

// Candidate key of every kept keypoint, in keypoint order (the origin of a
// keypoint for callers that merge partial results, e.g. row-band shards).
__global__ __launch_bounds__(256) void k_scatter_key(const unsigned* __restrict__ keep,
                                                     const unsigned* __restrict__ pos,
                                                     const unsigned* __restrict__ key,
                                                     const unsigned* __restrict__ n, int cap,
                                                     unsigned* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < cap && i < (int)min(*n, (unsigned)cap) && keep[i]) out[pos[i]] = key[i];
}

__global__ __launch_bounds__(256) void k_count_kp(const Pyramid P, const unsigned* __restrict__ pos,
                                                  const unsigned* __restrict__ keep, const unsigned* __restrict__ key,
                                                  const unsigned* __restrict__ n, unsigned cap,
                                                  unsigned* __restrict__ out, unsigned* __restrict__ blk) {
  __shared__ unsigned hist[kBlkN];
  const unsigned m = min(*n, cap);
  const int nb = P.nimg * P.O * P.S;
  auto kept_before = [&](unsigned j) { return j < cap ? pos[j] : pos[cap - 1] + keep[cap - 1]; };
  if (threadIdx.x == 0) *out = m ? kept_before(m) : 0u;
  if (!m) return;  // blk[b] stays 0
  if (!blk[kBlkUnsorted]) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x)
      blk[b] = kept_before(blk[kBlkStart + b + 1]) - kept_before(blk[kBlkStart + b]);
    return;
  }
  for (int b = threadIdx.x; b < nb; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for (unsigned i = threadIdx.x; i < m; i += blockDim.x)
    if (keep[i]) atomicAdd(&hist[key_block(P, key[i])], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x) blk[b] = hist[b];
}

// Candidate key of each keypoint -> (octave, scale, whole-image row, x).
__global__ __launch_bounds__(256) void k_decode_origins(const Pyramid P, const unsigned* __restrict__ keys, int n,
                                                        int32_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int im, o, s, y, x;
  decode_key(P, keys[i], im, o, s, y, x);
  out[4 * i + 0] = o;
  out[4 * i + 1] = s;
  out[4 * i + 2] = y + ((P.row0 * 2) >> o);
  out[4 * i + 3] = x;
}

// Block-major merge as segment copies: every (part, block) run of keypoints
// is contiguous in the input and in the output, so one workgroup copies one
// 16-KiB chunk of one run with 16-byte loads and stores (records are 48 B).
// seg[3 i] = {source byte offset, destination byte offset, bytes} of run i;
// cstart[i] = its first chunk (the grid is cstart[nseg]).

__global__ __launch_bounds__(256) void k_merge_blocks(const unsigned char* __restrict__ in,
                                                      unsigned char* __restrict__ out,
                                                      const long long* __restrict__ seg,
                                                      const long long* __restrict__ cstart, int nseg) {
  const long long c = blockIdx.x;
  int lo = 0, hi = nseg - 1;  // the run of chunk c: the last with cstart <= c
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cstart[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const long long* sg = seg + 3 * (long long)lo;
  const long long off = (c - cstart[lo]) * kMergeChunk;
  const long long n16 = min(kMergeChunk, sg[2] - off) >> 4;
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(in + sg[0] + off);
  uint4* __restrict__ dst = reinterpret_cast<uint4*>(out + sg[1] + off);
  for (long long i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
}

hipError_t launch_merge_blocks(const Keypoint* in, const long long* seg, const long long* cstart, int nseg,
                               long long n_chunks, Keypoint* out, hipStream_t st) {
  if (nseg <= 0 || n_chunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_blocks, dim3((unsigned)n_chunks), dim3(256), 0, st,
                     reinterpret_cast<const unsigned char*>(in), reinterpret_cast<unsigned char*>(out), seg, cstart,
                     nseg);
  return hipGetLastError();
}

hipError_t launch_decode_origins(const Pyramid& P, const unsigned* keys, int n, int32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decode_origins, dim3((n + 255) / 256), dim3(256), 0, st, P, keys, n, out);
  return hipGetLastError();
}

// Deferred candidate values (EmitLaunch.deferred): the fp32 plane value of
// every slot still holding the NaN marker.
__global__ __launch_bounds__(256) void k_fill_values(const Pyramid P, const unsigned* __restrict__ keys,
                                                     double* __restrict__ value, const unsigned* n, int cap) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int)min(*n, (unsigned)cap)) return;
  const double v = value[i];
  if (v == v) return;
  int im, o, s, y, x;
  decode_key(P, keys[i], im, o, s, y, x);
  const Octave& oc = P.oct[o];
  value[i] = (double)P.dog[im * P.dog_bstride + oc.dog_off + (long long)s * oc.h * oc.w + (long long)y * oc.w + x];
}

hipError_t launch_fill_values(const Pyramid& P, const unsigned* keys, double* value, const unsigned* n, int cap,
                              hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_values, dim3((cap + 255) / 256), dim3(256), 0, st, P, keys, value, n, cap);
  return hipGetLastError();
}

// Band order items: one thread per (octave, band, scale) item, its slot
// range from the row offsets of the extrema stage.
__global__ __launch_bounds__(256) void k_band_items(const Pyramid P, const BandOrder B) {
  const int it = blockIdx.x * 256 + threadIdx.x;
  if (it >= B.n_items) return;
  const int ipi = B.item_off[B.n_oct];  // items per image (image-major)
  const int im = it / ipi, il = it - im * ipi;
  int o = 0;
  while (o + 1 < B.n_oct && il >= B.item_off[o + 1]) ++o;
  const int loc = il - B.item_off[o];
  const int b = loc / B.S, s = loc % B.S + 1;
  const int h = P.oct[o].h;
  const int y0 = b * kBandRows, y1 = min(h, y0 + kBandRows);
  const long long r0 = (long long)im * B.rows_per_img + B.row_off[o] + (s - 1) * h + y0;
  const unsigned f = B.rowoff[r0];
  B.first[it] = f;
  B.count[it] = B.rowoff[r0 + (y1 - y0)] - f;
}

// One wave per item: its slots in order at its position of the new order.
__global__ __launch_bounds__(256) void k_band_fill(const Pyramid P, const BandOrder B) {
  const int it = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (it >= B.n_items) return;
  const unsigned c = B.count[it], f = B.first[it], st = B.start[it];
  for (unsigned j = threadIdx.x & 63; j < c; j += 64)
    if (st + j < (unsigned)B.cap) B.perm[st + j] = f + j;
}

hipError_t launch_band_items(const Pyramid& P, const BandOrder& B, hipStream_t st) {
  if (B.n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_band_items, dim3((B.n_items + 255) / 256), dim3(256), 0, st, P, B);
  return hipGetLastError();
}

hipError_t launch_band_fill(const Pyramid& P, const BandOrder& B, hipStream_t st) {
  if (B.n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_band_fill, dim3((B.n_items + 3) / 4), dim3(256), 0, st, P, B);
  return hipGetLastError();
}

hipError_t launch_refine_fast(const Pyramid& P, const RefineLaunch& R, hipStream_t st) {
  if (R.cap <= 0) return hipSuccess;
  if (R.exact_planes) hipLaunchKernelGGL(k_refine_fast<true>, dim3((R.cap + 255) / 256), dim3(256), 0, st, P, R);
  else hipLaunchKernelGGL(k_refine_fast<false>, dim3((R.cap + 255) / 256), dim3(256), 0, st, P, R);
  return hipGetLastError();
}

hipError_t launch_refine_exact(const Pyramid& P, const RefineLaunch& R, hipStream_t st) {
  if (R.cap <= 0) return hipSuccess;
  const int grid = std::max(1, std::min(R.cap, 8192));
  const size_t lds = exact_lds_bytes(P);
  const void* fn = R.wide_exact ? (const void*)k_refine_exact<256> : (const void*)k_refine_exact<64>;
  if (lds > 64 * 1024) {  // scratch of radii above ~335
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (R.wide_exact) hipLaunchKernelGGL(k_refine_exact<256>, dim3(grid), dim3(256), lds, st, P, R);
  else hipLaunchKernelGGL(k_refine_exact<64>, dim3(grid), dim3(64), lds, st, P, R);
  return hipGetLastError();
}

hipError_t launch_status_to_keep(const Pyramid& P, const int* status, const unsigned* key, unsigned* keep,
                                 const unsigned* n, int cap, int own_lo, int own_hi, unsigned* blk, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_status_to_keep, dim3((cap + 255) / 256), dim3(256), 0, st, P, status, key, keep, n, cap,
                     own_lo, own_hi, blk);
  return hipGetLastError();
}

hipError_t launch_scatter_keypoints(const unsigned* keep, const unsigned* pos, const Keypoint* kp,
                                    const unsigned* n, int cap, Keypoint* out, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_kp, dim3((cap + 255) / 256), dim3(256), 0, st, keep, pos, kp, n, cap, out);
  return hipGetLastError();
}

hipError_t launch_scatter_keys(const unsigned* keep, const unsigned* pos, const unsigned* key, const unsigned* n,
                               int cap, unsigned* out, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_key, dim3((cap + 255) / 256), dim3(256), 0, st, keep, pos, key, n, cap, out);
  return hipGetLastError();
}

hipError_t launch_count_keypoints(const Pyramid& P, const unsigned* pos, const unsigned* keep, const unsigned* key,
                                  const unsigned* n, int cap, unsigned* out, unsigned* blk, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_count_kp, dim3(1), dim3(256), 0, st, P, pos, keep, key, n, (unsigned)cap, out, blk);
  return hipGetLastError();
}

}  // namespace sift
