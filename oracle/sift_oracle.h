/* CPU oracle for the SIFT scale-space extrema path -- TEST INFRASTRUCTURE.
 *
 * A plain-C fp64 restatement of the reference's algorithm (bingjetli/
 * sift-scale-space-extrema-detection, JS).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker or the
 * CPU baseline -- never as the product path.
 *
 * Layout: every pyramid is one fp64 buffer, octave-major, then scale, then
 * row-major (y, x).  Octave o has dims (h_o, w_o): h_0 = 2H, w_0 = 2W,
 * h_o = ceil(h_{o-1}/2) (matrix2d.js:112-138 with rate 0.5 / 2.0).
 */
#ifndef SIFT_ORACLE_H
#define SIFT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int num_octaves;
  int scales_per_octave;
  double min_blur;
  double assumed_blur;
  double min_interpixel_distance;
} oracle_params;

/* CONV_2D: the reference's 2D kernel and summation order (sift.js:96-144).
 * CONV_SEPARABLE: the same operator separably (rows, then columns).
 * CONV_SEPARABLE_FMA_VH: columns then rows, fma chains -- the HIP path's own
 * operation order (a bit-exact pin of its fp64 values, not of the reference). */
enum { ORACLE_CONV_2D = 0, ORACLE_CONV_SEPARABLE = 1, ORACLE_CONV_SEPARABLE_FMA_VH = 2 };

/* dims[2*o] = h_o, dims[2*o+1] = w_o; returns sum_o h_o*w_o. */
long oracle_octave_dims(int W, int H, int O, int *dims);

/* blur[o*(S+3)+s] = blurLevel, sigma[o*(S+3)+s] = offset sigma (0 = copy). */
void oracle_schedule(const oracle_params *p, double *blur, double *sigma);

/* Threads of the blur loops (default 1). */
void oracle_set_threads(int n);

/* Gaussian scale space, (S+3) planes per octave. mode: ORACLE_CONV_*. */
int oracle_scale_space(const float *img, int W, int H, const oracle_params *p,
                       int mode, double *gauss);

/* DoG: (S+2) planes per octave, D[s-1] = L[s-1] - L[s]. */
void oracle_dog(const oracle_params *p, int W, int H, const double *gauss, double *dog);

/* Strict 26-neighbour extrema for DoG scales 1..S in reference order.
 * rec[4*i] = {octave, scaleLevel, x, y}; val[i] = DoG value.  Returns the
 * number of candidates (|v| >= 0.8*thr); *n_low = low-contrast extrema.
 * Stops writing at cap but keeps counting. */
long oracle_find_extrema(const oracle_params *p, int W, int H, const double *dog,
                         int32_t *rec, double *val, long cap, long *n_low);

/* Same, also listing the low-contrast extrema (reference order, the
 * reference's lowContrastKeypoints, sift.js:293-306) into low_rec / low_val
 * (up to low_cap; NULL = count only).  With oracle_set_threads(n > 1) the rows
 * are scanned in parallel; the lists are identical. */
long oracle_find_extrema_ex(const oracle_params *p, int W, int H, const double *dog,
                            int32_t *rec, double *val, long cap, int32_t *low_rec,
                            double *low_val, long low_cap, long *n_low);

/* Quadratic refinement.  out[8*i] = {octave, scaleLevel, localX, localY,
 * absoluteSigma, absoluteX, absoluteY, interpolatedValue}.  Candidates must
 * be in reference order.  *n_singular counts candidates whose Hessian had
 * |det| < DBL_EPSILON (the reference throws there, matrix2d.js:482). */
long oracle_refine(const oracle_params *p, int W, int H, const double *dog,
                   const int32_t *rec, const double *val, long n, double *out,
                   long cap, long *n_singular);

/* Whole pipeline, counts only (CPU baseline timing). */
long oracle_detect_count(const float *img, int W, int H, const oracle_params *p,
                         int mode, long *n_candidates);

#ifdef __cplusplus
}
#endif
#endif
