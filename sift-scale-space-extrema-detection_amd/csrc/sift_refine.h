// Refinement step shared by the fast refinement (sift_refine.hip) and the
// first step taken inside the extrema scan (sift_extrema.hip, SIFT_XREFINE).
// FP contraction is off for every function below and for the code that
// follows this include: the step rounds exactly as the reference does.
#pragma once
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

}  // namespace sift
