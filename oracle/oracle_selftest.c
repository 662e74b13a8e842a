/* Sanitizer driver for the CPU oracle -- TEST INFRASTRUCTURE.
 *
 * Built with -fsanitize=address,undefined by `make asan` (oracle/Makefile) and
 * run by tests/test_oracle_sanitize.py.  It drives every oracle entry point
 * over the shapes the reference's own inputs take and the edges the tests
 * hold: odd and tiny images (down to 1x1, whose octaves shrink to a single
 * pixel), one to six octaves, every convolution order, threaded and serial
 * scans, capacity-limited and count-only calls (cap 0 / NULL), and the
 * refinement on its own candidate list.  It prints one line per case with a
 * checksum of the outputs so the instrumented build can be compared with the
 * plain one (`make selftest`): the numbers must agree exactly.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sift_oracle.h"

/* blob image in [0, 1]: a few Gaussian spots on a ramp plus hash noise */
static void synth(float *img, int W, int H, unsigned seed) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      double v = 0.25 + 0.2 * (double)x / (W > 1 ? W - 1 : 1);
      for (int k = 0; k < 14; ++k) {
        unsigned h = (seed + 977u * (unsigned)k) * 2654435761u;
        double cx = (double)(h % 1000u) / 1000.0 * W, cy = (double)((h >> 10) % 1000u) / 1000.0 * H;
        double r = 1.5 + (double)((h >> 20) % 7u);
        double d2 = ((x - cx) * (x - cx) + (y - cy) * (y - cy)) / (r * r);
        v += ((k & 1) ? -0.5 : 0.6) * exp(-0.5 * d2);
      }
      unsigned n = ((unsigned)x * 73856093u) ^ ((unsigned)y * 19349663u) ^ (seed * 83492791u);
      v += 0.15 * (double)(n % 1000u) / 1000.0;
      img[(size_t)y * W + x] = (float)(v < 0 ? 0 : v > 1 ? 1 : v);
    }
}

static double sum_d(const double *a, long n) {
  double s = 0;
  for (long i = 0; i < n; ++i) s += a[i] * (double)((i % 13) + 1);
  return s;
}

static long sum_i(const int32_t *a, long n) {
  long s = 0;
  for (long i = 0; i < n; ++i) s += (long)a[i] * ((i % 7) + 1);
  return s;
}

static int run_case(int W, int H, int O, int S, int mode, int threads) {
  oracle_params p = {O, S, 0.8, 0.5, 0.5};
  int *dims = malloc(sizeof(int) * 2 * (size_t)O);
  long P = oracle_octave_dims(W, H, O, dims);
  double *blur = malloc(sizeof(double) * (size_t)O * (S + 3)), *sig = malloc(sizeof(double) * (size_t)O * (S + 3));
  oracle_schedule(&p, blur, sig);
  float *img = malloc(sizeof(float) * (size_t)W * H);
  synth(img, W, H, (unsigned)(W * 31 + H * 7 + O + S));
  double *g = malloc(sizeof(double) * (size_t)P * (S + 3)), *d = malloc(sizeof(double) * (size_t)P * (S + 2));
  oracle_set_threads(threads);
  if (oracle_scale_space(img, W, H, &p, mode, g) != 0) {
    printf("case %dx%d O%d S%d mode %d: scale space refused\n", W, H, O, S, mode);
    return 1;
  }
  oracle_dog(&p, W, H, g, d);
  long n_low = 0, n_low2 = 0;
  long n = oracle_find_extrema(&p, W, H, d, NULL, NULL, 0, &n_low);
  /* capacity-limited call: writes at most one record, still counts all */
  int32_t one_rec[4] = {0, 0, 0, 0};
  double one_val = 0;
  long n1 = oracle_find_extrema_ex(&p, W, H, d, one_rec, &one_val, n ? 1 : 0, NULL, NULL, 0, &n_low2);
  int32_t *rec = malloc(sizeof(int32_t) * 4 * (size_t)(n + 1));
  double *val = malloc(sizeof(double) * (size_t)(n + 1));
  int32_t *lrec = malloc(sizeof(int32_t) * 4 * (size_t)(n_low + 1));
  double *lval = malloc(sizeof(double) * (size_t)(n_low + 1));
  long n2 = oracle_find_extrema_ex(&p, W, H, d, rec, val, n, lrec, lval, n_low, &n_low2);
  double *out = malloc(sizeof(double) * 8 * (size_t)(n + 1));
  long sing = 0;
  long k = oracle_refine(&p, W, H, d, rec, val, n, out, n, &sing);
  long nc = 0;
  long kc = oracle_detect_count(img, W, H, &p, mode, &nc);
  oracle_set_threads(1);
  int bad = (n1 != n) || (n2 != n) || (n_low2 != n_low) || (nc != n) || (kc != k) ||
            (n && (memcmp(one_rec, rec, sizeof one_rec) || one_val != val[0]));
  printf("case %dx%d O%d S%d mode %d threads %d: planes %ld cand %ld low %ld kp %ld sing %ld "
         "sum_g %.17g sum_d %.17g sum_rec %ld sum_low %ld sum_kp %.17g sum_sched %.17g%s\n",
         W, H, O, S, mode, threads, P, n, n_low, k, sing, sum_d(g, P * (S + 3)), sum_d(d, P * (S + 2)),
         sum_i(rec, 4 * n), sum_i(lrec, 4 * n_low), sum_d(out, 8 * k), sum_d(blur, O * (S + 3)) + sum_d(sig, O * (S + 3)),
         bad ? " MISMATCH" : "");
  free(dims); free(blur); free(sig); free(img); free(g); free(d);
  free(rec); free(val); free(lrec); free(lval); free(out);
  return bad;
}

int main(void) {
  static const int cases[][4] = {
      {1, 1, 1, 3},   {1, 1, 3, 3},  {2, 3, 2, 3},   {5, 4, 3, 2},    {17, 9, 4, 3},
      {64, 48, 3, 3}, {77, 51, 3, 4}, {40, 40, 6, 5}, {96, 24, 2, 1}, {33, 65, 4, 5},
  };
  int bad = 0;
  for (size_t c = 0; c < sizeof cases / sizeof cases[0]; ++c)
    for (int mode = 0; mode < 3; ++mode)
      bad |= run_case(cases[c][0], cases[c][1], cases[c][2], cases[c][3], mode, 1);
  bad |= run_case(77, 51, 3, 4, 1, 4);
  bad |= run_case(64, 48, 3, 3, 0, 3);
  printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
