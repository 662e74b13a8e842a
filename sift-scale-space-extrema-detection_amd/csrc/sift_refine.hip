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
  double a[3];
  double omega;
  int s, m, n;       // position after the step (moved) or of the keypoint
};

// One iteration of background.js:480-664 on the patch d[k][a][c]
// (k: scale s-1+k, a: row m-1+a, c: col n-1+c).  `delta` bounds the error of
// every patch value (0 = exact), `dval` that of the candidate value.
__device__ inline StepOut refine_step(const double* d, int o, int s, int m, int n, double value,
                                      double delta, double dval, int S, int ND, int h, int w,
                                      double thr) {
#define DP(k, a, c) d[(k) * 9 + (a) * 3 + (c)]
  StepOut R;
  R.uncertain = false;
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
  const double dH = 4 * delta;  // |error| of every Hessian entry (diagonal worst case)
  if (delta > 0) {
    double cof1 = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) cof1 += fabs(mn[i][j]);
    if (fabs(fabs(det) - 2.220446049250313e-16) <= 16 * (cof1 * dH + 1e-300)) R.uncertain = true;
  }
  if (fabs(det) < 2.220446049250313e-16) {
    R.state = 3;
    return R;
  }
  double ninv[3][3];
  double inv_norm = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double rs = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double cof = ((i + j) & 1) ? mn[j][i] * -1.0 : mn[j][i];
      ninv[i][j] = (cof / det) * -1;
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
  // First-order error of alpha = -H^-1 g under |dg| <= delta, |dH| <= 4 delta.
  const double Ea = delta > 0 ? 16 * inv_norm * (delta + dH * a1) + 1e-300 : 0.0;
  if (delta > 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (fabs(fabs(R.a[i]) - 0.6) <= Ea) R.uncertain = true;
  }
  if (fabs(R.a[0]) < 0.6 && fabs(R.a[1]) < 0.6 && fabs(R.a[2]) < 0.6) {
    const double omega = value + (((0.5 * R.a[0]) * g0) + ((0.5 * R.a[1]) * g1) + ((0.5 * R.a[2]) * g2));
    R.omega = omega;
    R.s = s; R.m = m; R.n = n;
    if (delta > 0 || dval > 0) {
      const double Eo = 16 * (dval + 0.5 * (Ea * (fabs(g0) + fabs(g1) + fabs(g2)) + a1 * delta)) + 1e-300;
      if (fabs(fabs(omega) - thr) <= Eo) R.uncertain = true;
    }
    if (fabs(omega) < thr) { R.state = 2; return R; }
    const double tr = (0 + h22) + h33;
    const double dt = (h22 * h33) - (h23 * h23);
    const double edgeness = (tr * tr) / dt;
    if (delta > 0) {
      // Interval bound on tr^2/det2 with |dtr| <= 8 delta, |ddet2| <= (|h22|+|h33|) 4 delta + 2|h23| delta.
      const double Etr = 16 * 8 * delta;
      const double Edt = 16 * ((fabs(h22) + fabs(h33)) * dH + 2 * fabs(h23) * delta) + 1e-300;
      if (fabs(dt) <= Edt) {
        R.uncertain = true;
      } else {
        const double t_hi = fabs(tr) + Etr, t_lo = fmax(0.0, fabs(tr) - Etr);
        const double d_lo = fabs(dt) - Edt, d_hi = fabs(dt) + Edt;
        double e_lo, e_hi;
        if (dt > 0) { e_lo = t_lo * t_lo / d_hi; e_hi = t_hi * t_hi / d_lo; }
        else { e_lo = -(t_hi * t_hi / d_lo); e_hi = -(t_lo * t_lo / d_hi); }
        if (e_lo <= 12.1 && 12.1 <= e_hi) R.uncertain = true;
      }
    }
    if (edgeness > ((10 + 1) * (10 + 1)) / 10.0) { R.state = 2; return R; }
    R.state = 1;
    return R;
  }
  const double vs = s + R.a[0], vm = m + R.a[1], vn = n + R.a[2];
  if (delta > 0 && (round_margin(vs) <= Ea || round_margin(vm) <= Ea || round_margin(vn) <= Ea))
    R.uncertain = true;
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

__device__ inline void make_keypoint(Keypoint& k, int o, const StepOut& R, int S, double min_blur,
                                     double mid) {
  const double delta = ldexp(1.0, o - 1);  // Math.pow(2, octave - 1), exact
  k.octave = o;
  k.scale_level = R.s;
  k.local_x = R.n;
  k.local_y = R.m;
  k.abs_y = delta * (R.a[1] + R.m);
  k.abs_x = delta * (R.a[2] + R.n);
  k.abs_sigma = (delta / mid) * min_blur * pow(2.0, (R.a[0] + R.s) / S);
  k.interp_value = R.omega;
}

__global__ __launch_bounds__(256) void k_refine_fast(const Pyramid P, const RefineLaunch L) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool unc = false;
  if (i < L.n && L.keep && !L.keep[i]) {
    L.status[i] = kRefDiscard;
  } else if (i < L.n) {
    int o, s, m, n;
    decode_key(P, L.cand_key[i], o, s, m, n);
    const Octave& oc = P.oct[o];
    const int h = oc.h, w = oc.w;
    const long long plane = (long long)h * w;
    const float* __restrict__ D = P.dog + oc.dog_off;
    const double value = L.cand_val[i];
    const double dval = L.exact_planes ? 0.0 : fabs(value) * 0x1p-24;
    int status = kRefDiscard;
    double d[27];
    for (int it = 0; it < 5; ++it) {
      double mx = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const double v = (double)D[(s - 1 + k) * plane + (long long)(m - 1 + a) * w + (n - 1 + c)];
            d[k * 9 + a * 3 + c] = v;
            mx = fmax(mx, fabs(v));
          }
      // fp32 rounding of the fp64 value (<= |v| 2^-24) plus fp64 noise vs the reference.
      const double delta = L.exact_planes ? 0.0 : mx * (0x1p-24 + 0x1p-40);
      const StepOut R = refine_step(d, o, s, m, n, value, delta, dval, P.S, P.ND, h, w, P.thr);
      if (R.uncertain) { unc = true; break; }
      if (R.state == 3) { status = kRefSingular; break; }
      if (R.state == 2) { status = kRefDiscard; break; }
      if (R.state == 1) {
        status = kRefKeep;
        make_keypoint(L.kp[i], o, R, P.S, L.min_blur, L.min_interpixel_distance);
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
    if (unc) L.uncertain[base + pre] = (unsigned)i;
  }
}

// One wave per uncertain candidate: exact fp64 patches, lane 0 decides.
__global__ __launch_bounds__(64) void k_refine_exact(const Pyramid P, const RefineLaunch L) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int pos[4];
  const unsigned i = L.uncertain[blockIdx.x];
  int o, s, m, n;
  decode_key(P, L.cand_key[i], o, s, m, n);
  const Octave& oc = P.oct[o];
  double* d27 = smem;
  double* Lbuf = smem + 32;
  double* sh = smem + 32 + 40;
  double value = 0;
  int status = kRefDiscard;
  for (int it = 0; it < 5; ++it) {
    wave_dog_patch(P, o, s, m, n, sh, Lbuf, d27);
    if (threadIdx.x == 0) {
      if (it == 0) value = d27[13];  // exact fp64 candidate value (:565 uses it)
      const StepOut R = refine_step(d27, o, s, m, n, value, 0.0, 0.0, P.S, P.ND, oc.h, oc.w, P.thr);
      int cont = 0;
      if (R.state == 3) status = kRefSingular;
      else if (R.state == 2) status = kRefDiscard;
      else if (R.state == 1) {
        status = kRefKeep;
        make_keypoint(L.kp[i], o, R, P.S, L.min_blur, L.min_interpixel_distance);
      } else {
        cont = 1;
        pos[0] = R.s; pos[1] = R.m; pos[2] = R.n;
      }
      pos[3] = cont;
    }
    __syncthreads();
    if (!pos[3]) break;
    s = pos[0]; m = pos[1]; n = pos[2];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    L.status[i] = status;
    if (status == kRefSingular) atomicAdd(&L.counters[4], 1u);
  }
}

__global__ __launch_bounds__(256) void k_status_to_keep(const int* __restrict__ status,
                                                        unsigned* __restrict__ keep, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) keep[i] = status[i] == kRefKeep ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_scatter_kp(const int* __restrict__ status,
                                                    const unsigned* __restrict__ pos,
                                                    const Keypoint* __restrict__ kp, int n,
                                                    Keypoint* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && status[i] == kRefKeep) out[pos[i]] = kp[i];
}

hipError_t launch_refine_fast(const Pyramid& P, const RefineLaunch& R, hipStream_t st) {
  if (R.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_refine_fast, dim3((R.n + 255) / 256), dim3(256), 0, st, P, R);
  return hipGetLastError();
}

hipError_t launch_refine_exact(const Pyramid& P, const RefineLaunch& R, unsigned n_uncertain,
                               hipStream_t st) {
  if (n_uncertain == 0) return hipSuccess;
  hipLaunchKernelGGL(k_refine_exact, dim3(n_uncertain), dim3(64), exact_lds_bytes(P), st, P, R);
  return hipGetLastError();
}

hipError_t launch_status_to_keep(const int* status, unsigned* keep, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_status_to_keep, dim3((n + 255) / 256), dim3(256), 0, st, status, keep, n);
  return hipGetLastError();
}

hipError_t launch_scatter_keypoints(const int* status, const unsigned* pos, const Keypoint* kp,
                                    int n, Keypoint* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_kp, dim3((n + 255) / 256), dim3(256), 0, st, status, pos, kp, n, out);
  return hipGetLastError();
}

}  // namespace sift
