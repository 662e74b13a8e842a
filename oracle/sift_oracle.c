/* CPU oracle -- TEST INFRASTRUCTURE ONLY (see sift_oracle.h).
 *
 * fp64 restatement of the reference (bingjetli/sift-scale-space-extrema-
 * detection).  Each function cites the reference lines it follows; the
 * 2D mode keeps the reference's own summation order so it reproduces the
 * reference's numbers up to libm exp() differences.  Pinned against the
 * golden vectors in tests/golden (made from the reference itself).
 */
#include "sift_oracle.h"

#include <float.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>
#include <string.h>

/* Math.round: nearest integer, ties toward +infinity (exact for |x|<2^52). */
/* Threads of the blur loops (oracle_set_threads; default 1 = the scalar
 * port the CPU baseline is quoted on).  Each output pixel is the same sum in
 * the same order whatever the thread count. */
static int g_threads = 1;

void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }

static double js_round(double x) {
  double f = floor(x);
  return (x - f >= 0.5) ? f + 1.0 : f;
}

long oracle_octave_dims(int W, int H, int O, int *dims) {
  /* background.js:84 upsample (rate 0.5), :118 subsample (rate 2.0);
   * matrix2d.js:112-138 loops i += rate, so sizes are 2H and ceil(h/2). */
  long total = 0;
  int h = 2 * H, w = 2 * W;
  for (int o = 0; o < O; o++) {
    if (o > 0) { h = (h + 1) / 2; w = (w + 1) / 2; }
    dims[2 * o] = h;
    dims[2 * o + 1] = w;
    total += (long)h * w;
  }
  return total;
}

void oracle_schedule(const oracle_params *p, double *blur, double *sigma) {
  /* background.js:89-177 */
  const int S = p->scales_per_octave, NS = S + 3;
  const double k = pow(2.0, 1.0 / S);
  double base_blur = p->min_blur;
  for (int o = 0; o < p->num_octaves; o++) {
    for (int s = 0; s < NS; s++) {
      if (o > 0 && s == 0) {
        base_blur = blur[(o - 1) * NS + S]; /* seed.blurLevel, :114-122 */
        blur[o * NS] = base_blur;
        sigma[o * NS] = 0.0;
      } else {
        double target = base_blur * pow(k, (double)s);
        double from = (o == 0) ? p->assumed_blur : base_blur;
        blur[o * NS + s] = target;
        sigma[o * NS + s] = sqrt((target * target) - (from * from));
      }
    }
  }
}

/* sift.js:31-67 buildGaussianKernel: (2r+1)^2 kernel, r = Math.round(3s),
 * g = exp(((i^2+j^2)/s^2)*-0.5)/(2*pi*s^2) built row-major, divided by its sum. */
static double *build_kernel_2d(double sig, int *size) {
  int off = (int)js_round(3.0 * sig);
  int ks = 2 * off + 1;
  double *K = (double *)malloc(sizeof(double) * ks * ks);
  double sum = 0.0;
  for (int i = 0; i < ks; i++)
    for (int j = 0; j < ks; j++) {
      double a = i - off, b = j - off;
      double g = exp((((a * a) + (b * b)) / (sig * sig)) * -0.5) / (2 * M_PI * (sig * sig));
      sum += g;
      K[i * ks + j] = g;
    }
  for (int i = 0; i < ks * ks; i++) K[i] = K[i] / sum;
  *size = ks;
  return K;
}

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* Rows [y0, y1) of fn's output; with g_threads > 1 the rows are split into
 * contiguous ranges, one per thread.  The hot loops live in the range
 * functions, so the 1-thread path runs exactly the scalar code. */
typedef void (*row_fn)(const void *ctx, int y0, int y1);

static void for_rows(row_fn fn, const void *ctx, int h) {
  if (g_threads <= 1 || h < 2) {
    fn(ctx, 0, h);
    return;
  }
#pragma omp parallel num_threads(g_threads)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num(), nt = omp_get_num_threads();
#else
    int t = 0, nt = 1;
#endif
    int y0 = (int)((long)h * t / nt), y1 = (int)((long)h * (t + 1) / nt);
    fn(ctx, y0, y1);
  }
}

typedef struct {
  const double *in;
  double *out;
  const double *K;
  int h, w, ks, shift;
} blur2d_ctx;

/* sift.js:72-149 SIFT_blurMatrix2DChunk over the whole plane: i (kernel row)
 * offsets x, j offsets y, clamped reads, x-offset outer / y-offset inner. */
static void blur_2d_rows(const void *vc, int y0, int y1) {
  const blur2d_ctx *c = (const blur2d_ctx *)vc;
  const double *in = c->in, *K = c->K;
  double *out = c->out;
  const int h = c->h, w = c->w, ks = c->ks, shift = c->shift;
  for (int y = y0; y < y1; y++)
    for (int x = 0; x < w; x++) {
      double acc = 0.0;
      for (int i = 0; i < ks; i++) {
        int xx = clampi(x + (i - shift), 0, w - 1);
        for (int j = 0; j < ks; j++) {
          int yy = clampi(y + (j - shift), 0, h - 1);
          acc += in[(long)yy * w + xx] * K[i * ks + j];
        }
      }
      out[(long)y * w + x] = acc;
    }
}

static void blur_2d(const double *in, double *out, int h, int w, double sig) {
  int ks;
  double *K = build_kernel_2d(sig, &ks);
  blur2d_ctx c = {in, out, K, h, w, ks, ks / 2};
  for_rows(blur_2d_rows, &c, h);
  free(K);
}

typedef struct {
  const double *in;
  double *out;
  const double *wt;
  int h, w, r, n;
} sep_ctx;

static void sep_rows_h(const void *vc, int y0, int y1) {
  const sep_ctx *c = (const sep_ctx *)vc;
  const int w = c->w, r = c->r, n = c->n;
  for (int y = y0; y < y1; y++)
    for (int x = 0; x < w; x++) {
      double acc = 0.0;
      for (int i = 0; i < n; i++) acc += c->wt[i] * c->in[(long)y * w + clampi(x + i - r, 0, w - 1)];
      c->out[(long)y * w + x] = acc;
    }
}

static void sep_rows_v(const void *vc, int y0, int y1) {
  const sep_ctx *c = (const sep_ctx *)vc;
  const int h = c->h, w = c->w, r = c->r, n = c->n;
  for (int y = y0; y < y1; y++)
    for (int x = 0; x < w; x++) {
      double acc = 0.0;
      for (int j = 0; j < n; j++) acc += c->wt[j] * c->in[(long)clampi(y + j - r, 0, h - 1) * w + x];
      c->out[(long)y * w + x] = acc;
    }
}

/* Same operator, separable: w(i) = g1(i)/sum g1 with g1 = exp((i^2/s^2)*-0.5),
 * exactly the 2D kernel's factorisation; rows then columns, fp64 throughout. */
static void blur_sep(const double *in, double *out, int h, int w, double sig) {
  int r = (int)js_round(3.0 * sig);
  int n = 2 * r + 1;
  double *wt = (double *)malloc(sizeof(double) * n);
  double sum = 0.0;
  for (int i = 0; i < n; i++) {
    double a = i - r;
    wt[i] = exp(((a * a) / (sig * sig)) * -0.5);
    sum += wt[i];
  }
  for (int i = 0; i < n; i++) wt[i] /= sum;
  double *tmp = (double *)malloc(sizeof(double) * (size_t)h * w);
  sep_ctx ch = {in, tmp, wt, h, w, r, n};
  for_rows(sep_rows_h, &ch, h);
  sep_ctx cv = {tmp, out, wt, h, w, r, n};
  for_rows(sep_rows_v, &cv, h);
  free(tmp);
  free(wt);
}

/* The GPU's operation order (k_gauss_dog, sift_exact.h): vertical pass then
 * horizontal, each output an fma chain over the taps in increasing order,
 * starting from 0.0.  Not the reference's order (that is CONV_2D); it pins
 * the HIP path bit for bit: its fp64 values, hence its fp32 planes, extrema
 * ties and low-contrast decisions, are these. */
static void sep_rows_v_fma(const void *vc, int y0, int y1) {
  const sep_ctx *c = (const sep_ctx *)vc;
  const int h = c->h, w = c->w, r = c->r, n = c->n;
  for (int y = y0; y < y1; y++)
    for (int x = 0; x < w; x++) {
      double acc = 0.0;
      for (int j = 0; j < n; j++) acc = fma(c->wt[j], c->in[(long)clampi(y + j - r, 0, h - 1) * w + x], acc);
      c->out[(long)y * w + x] = acc;
    }
}

static void sep_rows_h_fma(const void *vc, int y0, int y1) {
  const sep_ctx *c = (const sep_ctx *)vc;
  const int w = c->w, r = c->r, n = c->n;
  for (int y = y0; y < y1; y++)
    for (int x = 0; x < w; x++) {
      double acc = 0.0;
      for (int i = 0; i < n; i++) acc = fma(c->wt[i], c->in[(long)y * w + clampi(x + i - r, 0, w - 1)], acc);
      c->out[(long)y * w + x] = acc;
    }
}

static void blur_sep_fma_vh(const double *in, double *out, int h, int w, double sig) {
  int r = (int)js_round(3.0 * sig);
  int n = 2 * r + 1;
  double *wt = (double *)malloc(sizeof(double) * n);
  double sum = 0.0;
  for (int i = 0; i < n; i++) {
    double a = i - r;
    wt[i] = exp(((a * a) / (sig * sig)) * -0.5);
    sum += wt[i];
  }
  for (int i = 0; i < n; i++) wt[i] /= sum;
  double *tmp = (double *)malloc(sizeof(double) * (size_t)h * w);
  sep_ctx cv = {in, tmp, wt, h, w, r, n};
  for_rows(sep_rows_v_fma, &cv, h);
  sep_ctx ch = {tmp, out, wt, h, w, r, n};
  for_rows(sep_rows_h_fma, &ch, h);
  free(tmp);
  free(wt);
}

int oracle_scale_space(const float *img, int W, int H, const oracle_params *p, int mode,
                       double *gauss) {
  /* background.js:71-237 */
  const int O = p->num_octaves, S = p->scales_per_octave, NS = S + 3;
  int *dims = (int *)malloc(sizeof(int) * 2 * O);
  double *blur = (double *)malloc(sizeof(double) * O * NS);
  double *sigma = (double *)malloc(sizeof(double) * O * NS);
  oracle_octave_dims(W, H, O, dims);
  oracle_schedule(p, blur, sigma);
  /* :84 base = 2x nearest-neighbour upsample of the input */
  int h = dims[0], w = dims[1];
  double *base = (double *)malloc(sizeof(double) * (size_t)h * w);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) base[(long)y * w + x] = (double)img[(long)(y / 2) * W + (x / 2)];
  double *plane = gauss;
  double *prev_oct = NULL;
  int ph = 0, pw = 0;
  for (int o = 0; o < O; o++) {
    h = dims[2 * o];
    w = dims[2 * o + 1];
    if (o > 0) {
      /* :114-118 seed = L[o-1][S], subsampled by taking [2i][2j] */
      const double *seed = prev_oct + (size_t)S * ph * pw;
      free(base);
      base = (double *)malloc(sizeof(double) * (size_t)h * w);
      for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) base[(long)y * w + x] = seed[(long)(2 * y) * pw + 2 * x];
    }
    prev_oct = plane;
    for (int s = 0; s < NS; s++) {
      if (o > 0 && s == 0) {
        memcpy(plane, base, sizeof(double) * (size_t)h * w);
      } else if (mode == ORACLE_CONV_2D) {
        blur_2d(base, plane, h, w, sigma[o * NS + s]);
      } else if (mode == ORACLE_CONV_SEPARABLE_FMA_VH) {
        blur_sep_fma_vh(base, plane, h, w, sigma[o * NS + s]);
      } else {
        blur_sep(base, plane, h, w, sigma[o * NS + s]);
      }
      plane += (size_t)h * w;
    }
    ph = h;
    pw = w;
  }
  free(base);
  free(dims);
  free(blur);
  free(sigma);
  return 0;
}

void oracle_dog(const oracle_params *p, int W, int H, const double *gauss, double *dog) {
  /* background.js:258-354 with sift.js:154-188: D[s-1] = L[s-1] - L[s] */
  const int O = p->num_octaves, S = p->scales_per_octave;
  int *dims = (int *)malloc(sizeof(int) * 2 * O);
  oracle_octave_dims(W, H, O, dims);
  const double *g = gauss;
  double *d = dog;
  for (int o = 0; o < O; o++) {
    size_t P = (size_t)dims[2 * o] * dims[2 * o + 1];
    for (int s = 1; s < S + 3; s++) {
      const double *a = g + (size_t)(s - 1) * P, *b = g + (size_t)s * P;
      for (size_t i = 0; i < P; i++) d[i] = a[i] - b[i];
      d += P;
    }
    g += (size_t)(S + 3) * P;
  }
  free(dims);
}

static double contrast_threshold(int S) {
  /* sift.js:285 and background.js:572 */
  return ((pow(2.0, 1.0 / S) - 1) / (pow(2.0, 1.0 / 3) - 1)) * 0.015;
}

/* One extremum list being filled: records past cap are counted, not written. */
typedef struct {
  int32_t *rec;
  double *val;
  long cap;
} xlist;

static inline void xlist_put(const xlist *L, long i, int o, int s, int x, int y, double v) {
  if (!L->rec || i >= L->cap) return;
  L->rec[4 * i] = o; L->rec[4 * i + 1] = s; L->rec[4 * i + 2] = x; L->rec[4 * i + 3] = y;
  L->val[i] = v;
}

/* sift.js:212-316 on one row y of the DoG trio A, B, C: strict 26-neighbour
 * min/max, |v| >= 0.8*thr -> candidate list, else low-contrast list (:293-306),
 * x ascending.  nc / nl: running indices of the two lists. */
static void scan_row(const double *A, const double *B, const double *C, int w, int y, double pix_thr, int o,
                     int s, const xlist *cand, const xlist *lowl, long *nc, long *nl) {
  for (int x = 1; x < w - 1; x++) {
    const double c = B[(long)y * w + x];
    int is_min = 1, is_max = 1;
    for (int pl = 0; pl < 3; pl++) {
      const double *Q = pl == 0 ? A : (pl == 1 ? B : C);
      for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          if (pl == 1 && dy == 0 && dx == 0) continue;
          const double v = Q[(long)(y + dy) * w + x + dx];
          if (!(v > c)) is_min = 0;
          if (!(v < c)) is_max = 0;
        }
    }
    if (is_min || is_max) {
      if (fabs(c) >= pix_thr) xlist_put(cand, (*nc)++, o, s, x, y, c);
      else xlist_put(lowl, (*nl)++, o, s, x, y, c);
    }
  }
}

typedef struct {
  const double *A, *B, *C;
  int w, o, s;
  double pix_thr;
  long *row_nc, *row_nl;      /* per row (index y-1): counts (pass 1) / first index (pass 2) */
  const xlist *cand, *lowl;
  int write;
} xscan_ctx;

/* Rows 1 + [r0, r1) of one trio: pass 1 counts per row, pass 2 writes every
 * row at its precomputed offset -- the list order is the sequential one. */
static void xscan_rows(const void *vc, int r0, int r1) {
  const xscan_ctx *c = (const xscan_ctx *)vc;
  static const xlist none = {NULL, NULL, 0};
  for (int r = r0; r < r1; r++) {
    long nc = c->write ? c->row_nc[r] : 0, nl = c->write ? c->row_nl[r] : 0;
    scan_row(c->A, c->B, c->C, c->w, r + 1, c->pix_thr, c->o, c->s, c->write ? c->cand : &none,
             c->write ? c->lowl : &none, &nc, &nl);
    if (!c->write) {
      c->row_nc[r] = nc;
      c->row_nl[r] = nl;
    }
  }
}

long oracle_find_extrema_ex(const oracle_params *p, int W, int H, const double *dog, int32_t *rec,
                            double *val, long cap, int32_t *low_rec, double *low_val, long low_cap,
                            long *n_low) {
  /* background.js:359-450 (scales 1..S), sift.js:212-316 */
  const int O = p->num_octaves, S = p->scales_per_octave;
  int *dims = (int *)malloc(sizeof(int) * 2 * O);
  oracle_octave_dims(W, H, O, dims);
  const double pix_thr = contrast_threshold(S) * 0.8;
  long n = 0, low = 0;
  const double *d = dog;
  for (int o = 0; o < O; o++) {
    const int h = dims[2 * o], w = dims[2 * o + 1];
    const size_t P = (size_t)h * w;
    for (int s = 1; s < S + 1; s++) {
      const double *A = d + (size_t)(s - 1) * P, *B = d + (size_t)s * P, *C = d + (size_t)(s + 1) * P;
      const xlist cand = {rec, val, cap}, lowl = {low_rec, low_val, low_cap};
      if (g_threads <= 1 || h < 4) {
        for (int y = 1; y < h - 1; y++) scan_row(A, B, C, w, y, pix_thr, o, s, &cand, &lowl, &n, &low);
        continue;
      }
      const int nr = h - 2;
      long *rnc = (long *)calloc((size_t)nr, sizeof(long)), *rnl = (long *)calloc((size_t)nr, sizeof(long));
      xscan_ctx c = {A, B, C, w, o, s, pix_thr, rnc, rnl, &cand, &lowl, 0};
      for_rows(xscan_rows, &c, nr);
      for (int r = 0; r < nr; r++) {  /* counts -> first index of every row */
        const long a = rnc[r], b = rnl[r];
        rnc[r] = n;
        rnl[r] = low;
        n += a;
        low += b;
      }
      c.write = 1;
      for_rows(xscan_rows, &c, nr);
      free(rnc);
      free(rnl);
    }
    d += (size_t)(S + 2) * P;
  }
  free(dims);
  if (n_low) *n_low = low;
  return n;
}

long oracle_find_extrema(const oracle_params *p, int W, int H, const double *dog, int32_t *rec,
                         double *val, long cap, long *n_low) {
  return oracle_find_extrema_ex(p, W, H, dog, rec, val, cap, NULL, NULL, 0, n_low);
}

long oracle_refine(const oracle_params *p, int W, int H, const double *dog, const int32_t *rec,
                   const double *val, long n_cand, double *out, long cap, long *n_singular) {
  /* background.js:455-685; sift.js:333-446; matrix2d.js:197-546 */
  const int O = p->num_octaves, S = p->scales_per_octave, ND = S + 2;
  int *dims = (int *)malloc(sizeof(int) * 2 * O);
  size_t *ooff = (size_t *)malloc(sizeof(size_t) * O);
  oracle_octave_dims(W, H, O, dims);
  size_t acc = 0;
  for (int o = 0; o < O; o++) {
    ooff[o] = acc;
    acc += (size_t)ND * dims[2 * o] * dims[2 * o + 1];
  }
  const double thr = contrast_threshold(S);
  const double edge_thr = ((10 + 1) * (10 + 1)) / 10.0;
  long nout = 0, nsing = 0;
  for (long c = 0; c < n_cand; c++) {
    const int o = rec[4 * c];
    const int h = dims[2 * o], w = dims[2 * o + 1];
    const size_t P = (size_t)h * w;
    const double *Do = dog + ooff[o];
#define DV(ss, mm, nn) Do[(size_t)(ss) * P + (size_t)(mm) * w + (nn)]
    int s = rec[4 * c + 1], m = rec[4 * c + 3], nn = rec[4 * c + 2];
    for (int it = 0; it < 5; it++) {
      const double g0 = (DV(s + 1, m, nn) - DV(s - 1, m, nn)) / 2;
      const double g1 = (DV(s, m + 1, nn) - DV(s, m - 1, nn)) / 2;
      const double g2 = (DV(s, m, nn + 1) - DV(s, m, nn - 1)) / 2;
      const double cc = DV(s, m, nn);
      const double h11 = DV(s + 1, m, nn) + DV(s - 1, m, nn) - (2 * cc);
      const double h22 = DV(s, m + 1, nn) + DV(s, m - 1, nn) - (2 * cc);
      const double h33 = DV(s, m, nn + 1) + DV(s, m, nn - 1) - (2 * cc);
      const double h12 = (DV(s + 1, m + 1, nn) - DV(s + 1, m - 1, nn) - DV(s - 1, m + 1, nn) +
                          DV(s - 1, m - 1, nn)) / 4;
      const double h13 = (DV(s + 1, m, nn + 1) - DV(s + 1, m, nn - 1) - DV(s - 1, m, nn + 1) +
                          DV(s - 1, m, nn - 1)) / 4;
      const double h23 = (DV(s, m + 1, nn + 1) - DV(s, m + 1, nn - 1) - DV(s, m - 1, nn + 1) +
                          DV(s, m - 1, nn - 1)) / 4;
      const double M[3][3] = {{h11, h12, h13}, {h12, h22, h23}, {h13, h23, h33}};
      /* get3x3Determinant (:236) with top-row minors; get3x3Minors (:303)
       * fills the rest; cofactors (:395), transpose (:412), divide (:444). */
      double mn[3][3];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          double q[4];
          int k = 0;
          for (int ii = 0; ii < 3; ii++) {
            if (ii == i) continue;
            for (int jj = 0; jj < 3; jj++) {
              if (jj == j) continue;
              q[k++] = M[ii][jj];
            }
          }
          mn[i][j] = (q[0] * q[3]) - (q[1] * q[2]);
        }
      const double det = ((M[0][0] * mn[0][0]) - (M[0][1] * mn[0][1])) + (M[0][2] * mn[0][2]);
      if (fabs(det) < DBL_EPSILON) { /* matrix2d.js:482 -> null -> TypeError */
        nsing++;
        break;
      }
      double ninv[3][3];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          const double cof = mn[j][i] * (((i + j) & 1) ? -1.0 : 1.0); /* adj[i][j] = cof[j][i] */
          ninv[i][j] = (cof / det) * -1;
        }
      const double gv[3] = {g0, g1, g2};
      double a[3];
      for (int i = 0; i < 3; i++) {
        double r = 0;
        for (int j = 0; j < 3; j++) r += ninv[i][j] * gv[j];
        a[i] = r;
      }
      if (fabs(a[0]) < 0.6 && fabs(a[1]) < 0.6 && fabs(a[2]) < 0.6) {
        /* :565 uses the ORIGINAL candidate value */
        const double omega = val[c] + (((0.5 * a[0]) * g0) + ((0.5 * a[1]) * g1) + ((0.5 * a[2]) * g2));
        if (fabs(omega) < thr) break;
        const double tr = (0 + h22) + h33;
        const double dt = (h22 * h33) - (h23 * h23);
        const double edgeness = (tr * tr) / dt;
        if (edgeness > edge_thr) break; /* NaN and negative pass (quirks 2, 3) */
        const double delta = pow(2.0, o - 1);
        const double Y = delta * (a[1] + m);
        const double X = delta * (a[2] + nn);
        const double sig = (delta / p->min_interpixel_distance) * p->min_blur *
                           pow(2.0, (a[0] + s) / S);
        if (nout < cap) {
          double *r = out + 8 * nout;
          r[0] = o; r[1] = s; r[2] = nn; r[3] = m;
          r[4] = sig; r[5] = X; r[6] = Y; r[7] = omega;
        }
        nout++;
        break;
      }
      s = (int)js_round(s + a[0]);
      m = (int)js_round(m + a[1]);
      nn = (int)js_round(nn + a[2]);
      if (s < 1 || s >= ND - 1) break;
      if (m < 1 || m >= h - 1) break;
      if (nn < 1 || nn >= w - 1) break;
    }
#undef DV
  }
  free(dims);
  free(ooff);
  if (n_singular) *n_singular = nsing;
  return nout;
}

long oracle_detect_count(const float *img, int W, int H, const oracle_params *p, int mode,
                         long *n_candidates) {
  const int O = p->num_octaves, S = p->scales_per_octave;
  int *dims = (int *)malloc(sizeof(int) * 2 * O);
  long P = oracle_octave_dims(W, H, O, dims);
  double *g = (double *)malloc(sizeof(double) * P * (S + 3));
  double *d = (double *)malloc(sizeof(double) * P * (S + 2));
  oracle_scale_space(img, W, H, p, mode, g);
  oracle_dog(p, W, H, g, d);
  long low = 0;
  long nc = oracle_find_extrema(p, W, H, d, NULL, NULL, 0, &low);
  int32_t *rec = (int32_t *)malloc(sizeof(int32_t) * 4 * (nc + 1));
  double *val = (double *)malloc(sizeof(double) * (nc + 1));
  oracle_find_extrema(p, W, H, d, rec, val, nc, &low);
  double *out = (double *)malloc(sizeof(double) * 8 * (nc + 1));
  long sing = 0;
  long nk = oracle_refine(p, W, H, d, rec, val, nc, out, nc, &sing);
  free(out); free(val); free(rec); free(d); free(g); free(dims);
  if (n_candidates) *n_candidates = nc;
  return nk;
}
