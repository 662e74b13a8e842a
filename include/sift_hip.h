/*
 * sift_hip.h -- C ABI of the MI355X (gfx950) SIFT scale-space extrema path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (bingjetli/sift-scale-space-extrema-detection).  The reference exposes the
 * path as a Web-Worker message protocol (src/worker.js:5-98 helpers,
 * background.js:14-50 dispatcher); every entry point below names the
 * reference function whose behaviour it reproduces.  Plain C types only: no
 * C++ or torch types cross this boundary.  The Node N-API addon
 * (sift-scale-space-extrema-detection_amd/napi/sift_napi.c) and the Python
 * ctypes binding bind exactly these symbols.
 *
 * Threading: one sift_ctx per host thread; a ctx is not re-entrant; distinct
 * ctxs are independent.  Every call is synchronous with respect to the ctx's
 * HIP stream unless its name ends in _async.
 *
 * Numerics: Gaussian weights and every convolution accumulate in fp64 (the
 * reference computes in JS Number = fp64); Gaussian and DoG planes are
 * handed out as fp32 (the ImageData-shaped Float32 contract); octave seeds
 * stay fp64 on device; extrema decisions and refinement are fp64 and exact
 * with respect to the fp64 pyramid (fp32 ties are re-decided in fp64).
 */
#ifndef SIFT_HIP_H
#define SIFT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIFT_ABI_VERSION 9

/* Opaque context (one HIP stream + device-resident pyramids). */
struct sift_ctx;

/* Status codes.  Every function returns one of these. */
enum {
  SIFT_OK = 0,
  SIFT_E_ARG = -1,        /* invalid argument (null pointer, bad size, bad index)   */
  SIFT_E_HIP = -2,        /* HIP runtime error; see sift_last_error()               */
  SIFT_E_CAPACITY = -3,   /* output buffer too small; *n_out holds the needed count */
  SIFT_E_STATE = -4,      /* stage called before the stage it depends on            */
  SIFT_E_SINGULAR = -5,   /* refinement met a Hessian with |det| < DBL_EPSILON: the
                             reference throws a TypeError there (matrix2d.js:482 ->
                             :455); outputs for every other candidate are still
                             written and *n_singular counts the offenders           */
  SIFT_E_UNSUPPORTED = -6 /* configuration outside this build's limits              */
};

/* Plane kinds for sift_get_plane / sift_get_blur_level. */
enum { SIFT_PLANE_GAUSS = 0, SIFT_PLANE_DOG = 1 };

/* sift_params.flags */
enum {
  SIFT_F_SKIP_GAUSS_PLANES = 1 << 0, /* do not materialise Gaussian planes (seeds still kept) */
  SIFT_F_SKIP_DOG_PLANES = 1 << 1,   /* reserved: DoG planes are needed by refinement today   */
  SIFT_F_EXPORT_NEXT_SEED = 1 << 2,  /* also form the fp64 base of octave num_octaves (sift_next_seed) */
  SIFT_F_KEYPOINT_ORIGINS = 1 << 3,  /* record each keypoint's candidate (sift_keypoint_origins) */
  SIFT_F_FUSED_EXTREMA = 1 << 4,     /* detections: decide octave 0's extrema inside its Gaussian+DoG
                                        pass instead of re-reading its DoG planes (same results;
                                        measured slower on MI355X) */
  SIFT_F_LOW_CONTRAST_LIST = 1 << 5  /* also list the low-contrast extrema (sift_copy_low_contrast) */
};

/* Parameters of the pipeline.  Names and defaults follow
 * src/worker.js:29-98 (workerComputeGaussianScaleSpace / ...Refine...). */
typedef struct {
  int num_octaves;                /* number_of_octaves        default 5   (worker.js:33) */
  int scales_per_octave;          /* scales_per_octave        default 3   (worker.js:34) */
  double min_blur;                /* min_blur_level           default 0.8 (worker.js:35) */
  double assumed_blur;            /* assumed_blur             default 0.5 (worker.js:36) */
  double min_interpixel_distance; /* min_interpixel_distance  default 0.5 (worker.js:88) */
  int flags;                      /* SIFT_F_*                 default 0                  */
} sift_params;

/* One candidate extremum, reference order (octave, scale, y, x):
 * background.js:433-436 {scaleLevel, localExtremas:[{x, y, value}]}. */
typedef struct {
  int32_t octave;
  int32_t scale; /* scaleLevel: DoG index 1..S */
  int32_t x;
  int32_t y;
  double value; /* DoG value at (x, y) */
} sift_extremum;

/* One refined keypoint: background.js:619-628. */
typedef struct {
  int32_t octave;
  int32_t scale_level;
  int32_t local_x;
  int32_t local_y;
  double abs_x;
  double abs_y;
  double abs_sigma;
  double interp_value;
} sift_keypoint;

/* Per-stage device timings of the last call chain, milliseconds. */
typedef struct {
  double gauss_dog_ms; /* Gaussian + DoG kernels (all octaves)              */
  double extrema_ms;   /* extrema scan + ordering + exact tie resolution    */
  double refine_ms;    /* refinement + compaction                           */
  double h2d_ms;       /* input upload (0 for the device-pointer entry)     */
  double gauss_oct0_ms;/* octave 0's Gaussian + DoG launch alone (the        */
                       /* dominant, HBM-bound kernel; ABI version >= 2)     */
} sift_timings;

int sift_abi_version(void);
int sift_params_default(sift_params *p);

/* Context: owns one HIP stream and device-resident pyramids on `device`. */
int sift_ctx_create(int device, struct sift_ctx **out);
/* A context on the SAME stream as `share` (ABI version >= 2): its work is
 * ordered after everything already enqueued on `share`, so several
 * detections can be in flight (sift_detect_device_async) without their
 * kernels overlapping.  Destroy it before `share`. */
int sift_ctx_create_shared(struct sift_ctx *share, struct sift_ctx **out);
int sift_ctx_destroy(struct sift_ctx *ctx);
const char *sift_last_error(struct sift_ctx *ctx);

/* Offset sigma and blur level of every (octave, scale) for these params,
 * background.js:89-177.  Arrays are num_octaves*(scales_per_octave+3);
 * sigma 0 marks the un-blurred octave seed.  Pure host math. */
int sift_schedule(const sift_params *p, double *blur_levels, double *offset_sigmas);

/* Octave plane dims for a W x H input: dims[2o] = rows, dims[2o+1] = cols.
 * Pure host math (matrix2d.js:112-138 resize rules). */
int sift_octave_dims(int width, int height, int num_octaves, int *dims);

/* computeGaussianScaleSpace (background.js:71-237) fused with
 * computeDifferenceOfGaussians (background.js:258-354).  `img` is a gray
 * row-major Float32 host image (ImageData-shaped, stride in pixels).
 * `offset_sigmas` may be NULL (schedule computed here) or supply the
 * num_octaves*(S+3) offset sigmas computed by the caller (e.g. in JS with
 * Math.pow, so the schedule is bit-identical to the reference's). */
int sift_build_scale_space(struct sift_ctx *ctx, const float *img, int width, int height,
                           size_t stride_px, const sift_params *p, const double *offset_sigmas);

/* Same, with `d_img` already resident in device memory of ctx's device. */
int sift_build_scale_space_device(struct sift_ctx *ctx, const float *d_img, int width,
                                  int height, size_t stride_px, const sift_params *p,
                                  const double *offset_sigmas);

int sift_get_dims(struct sift_ctx *ctx, int octave, int *rows, int *cols);
int sift_get_blur_level(struct sift_ctx *ctx, int kind, int octave, int scale, double *blur);

/* Copy one plane to host memory owned by the caller (cap in pixels). */
int sift_get_plane(struct sift_ctx *ctx, int kind, int octave, int scale, float *dst,
                   size_t cap_px);

/* Replace the context's DoG pyramid with caller-supplied planes (for callers
 * that hand findCandidateKeypoints / refineCandidateKeypoints a pyramid this
 * context did not build).  `planes` is octave-major, (S+2) planes per
 * octave, each rows*cols fp32 in the dims sift_octave_dims gives. */
int sift_load_dog(struct sift_ctx *ctx, const float *planes, int width, int height,
                  const sift_params *p);

/* Replace the Gaussian pyramid with caller planes ((S+3) per octave) and
 * recompute the DoG from them: computeDifferenceOfGaussians on a foreign
 * scale space (background.js:258-354, sift.js:154-188). */
int sift_load_scale_space(struct sift_ctx *ctx, const float *planes, int width, int height,
                          const sift_params *p);

/* findCandidateKeypoints (background.js:359-450 + sift.js:212-316).
 * Strict 26-neighbour extrema of DoG scales 1..S with |v| >= 0.8*thr, in
 * reference order.  *n_low_contrast counts extrema failing 0.8*thr.
 * SIFT_E_CAPACITY: *n_out = required count, nothing written. */
int sift_find_extrema(struct sift_ctx *ctx, sift_extremum *out, size_t cap, size_t *n_out,
                      size_t *n_low_contrast);

/* The low-contrast extrema of the last extrema stage run with
 * SIFT_F_LOW_CONTRAST_LIST in its parameters (ABI version >= 5): strict
 * 26-neighbour extrema with |v| < 0.8*thr, the reference's
 * lowContrastKeypoints (sift.js:293-306), in its order (octave, scale, y, x)
 * with their DoG values.  SIFT_E_CAPACITY: *n_out = required count. */
int sift_copy_low_contrast(struct sift_ctx *ctx, sift_extremum *out, size_t cap, size_t *n_out);

/* Replace the sift_params.flags the context's current pyramid was built or
 * loaded with, for the stages that follow (ABI version >= 5): e.g.
 * SIFT_F_LOW_CONTRAST_LIST before sift_find_extrema on a built pyramid. */
int sift_set_flags(struct sift_ctx *ctx, int flags);

/* refineCandidateKeypoints (background.js:455-685) on the candidates of the
 * last sift_find_extrema (or sift_set_candidates).  Output keeps reference
 * order and duplicates. */
int sift_refine(struct sift_ctx *ctx, sift_keypoint *out, size_t cap, size_t *n_out,
                size_t *n_singular);

/* Copy the candidates / keypoints of the last find / refine / detect without
 * recomputing (cap in records; SIFT_E_CAPACITY if too small). */
int sift_copy_candidates(struct sift_ctx *ctx, sift_extremum *out, size_t cap, size_t *n_out);
int sift_copy_keypoints(struct sift_ctx *ctx, sift_keypoint *out, size_t cap, size_t *n_out);
/* The last keypoints as two field arrays (the JS typed result format):
 * ints[4i..4i+3] = octave, scale_level, local_x, local_y and reals[4i..4i+3]
 * = abs_sigma, abs_x, abs_y, interp_value of keypoint i, in the reference's
 * order (background.js:660-671).  Through the context's pinned staging. */
int sift_copy_keypoints_soa(struct sift_ctx *ctx, int32_t *ints, double *reals, size_t cap, size_t *n_out);

/* Page-lock a caller's host buffer for the device's DMA engines (ABI version
 * >= 8): plane and keypoint reads into a registered buffer are one
 * device -> host DMA instead of a staged copy through pinned memory.  For
 * buffers the caller recycles (the JS addon's result pool); unregister
 * before freeing.  Registration faults in and pins every page. */
int sift_host_register(void *p, size_t bytes);
int sift_host_unregister(void *p);

/* Override the two scalars refineCandidateKeypoints receives in its own
 * message (minBlurLevel, minInterpixelDistance: background.js:460-461,
 * :611-614) for the next sift_refine; build/load set them from sift_params. */
int sift_refine_params(struct sift_ctx *ctx, double min_blur_level, double min_interpixel_distance);

/* Use caller-supplied candidates (reference order) for the next sift_refine. */
int sift_set_candidates(struct sift_ctx *ctx, const sift_extremum *cand, size_t n);

/* Whole path in one call: build + extrema + refine.  Keypoints stay on
 * device when out == NULL (counts still returned). */
int sift_detect(struct sift_ctx *ctx, const float *img, int width, int height, size_t stride_px,
                const sift_params *p, sift_keypoint *out, size_t cap, size_t *n_out);
int sift_detect_device(struct sift_ctx *ctx, const float *d_img, int width, int height,
                       size_t stride_px, const sift_params *p, sift_keypoint *out, size_t cap,
                       size_t *n_out);

/* Counts of the last detect / find / refine: candidates, low-contrast
 * extrema, refined keypoints, singular Hessians, exact fp64 re-decisions. */
int sift_last_counts(struct sift_ctx *ctx, size_t *n_candidates, size_t *n_low_contrast,
                     size_t *n_keypoints, size_t *n_singular, size_t *n_exact);

/* Asynchronous one-call detection (ABI version >= 2): enqueue on the
 * context's stream and return; sift_detect_wait completes it (one host
 * synchronisation, capacity retries, counts) and copies the keypoints like
 * sift_detect.  One detection in flight per context: several contexts
 * (streams) keep the device busy while the host settles earlier images. */
int sift_detect_device_async(struct sift_ctx *ctx, const float *d_img, int width, int height,
                             size_t stride_px, const sift_params *p);
int sift_detect_wait(struct sift_ctx *ctx, sift_keypoint *out, size_t cap, size_t *n_out);

/* A batch of n_images independent device images of one geometry (ABI
 * version >= 6; BASELINE cfg 4's images per GPU): image b is width x height
 * at d_imgs + b * image_stride_px (row stride stride_px).  Each stage is ONE
 * launch over the whole batch -- a Gaussian+DoG launch per octave, one
 * extrema scan, one refinement -- with the planes image-major.  Per image the
 * results are exactly those of sift_detect_device on that image (the
 * reference's per-image path, background.js:71-685, run once per image); the
 * keypoints come out image-major, each image's in the reference's order, and
 * sift_last_block_counts gives n_images * num_octaves * scales_per_octave
 * block counts (image-major), so image b's count is the sum of its blocks.
 * Plain detection only: no low-contrast list, fused decisions, crops, owned
 * rows or exported seeds (SIFT_E_UNSUPPORTED); the candidate list of a batch
 * is not exposed.  _async enqueues it (sift_detect_wait completes it). */
int sift_detect_batch_device(struct sift_ctx *ctx, const float *d_imgs, int n_images, size_t image_stride_px,
                             int width, int height, size_t stride_px, const sift_params *p,
                             sift_keypoint *out, size_t cap, size_t *n_out);
/* The same batch from host images (image b at imgs + b * image_stride_px),
 * uploaded image by image into the context's device buffer. */
int sift_detect_batch(struct sift_ctx *ctx, const float *imgs, int n_images, size_t image_stride_px, int width,
                      int height, size_t stride_px, const sift_params *p, sift_keypoint *out, size_t cap,
                      size_t *n_out);
int sift_detect_batch_device_async(struct sift_ctx *ctx, const float *d_imgs, int n_images,
                                   size_t image_stride_px, int width, int height, size_t stride_px,
                                   const sift_params *p);

/* The same detection in two phases (ABI version >= 4): _begin enqueues the
 * Gaussian+DoG pass, _end the extrema scan and refinement; sift_detect_wait
 * completes it.  Between the two, sift_order_after can hold the second
 * phase back behind other contexts' work (bench.py --overlap phased: the
 * next image's octave 0 runs before this image's extrema scan, so the
 * HBM-bound phases of consecutive images alternate instead of contending). */
int sift_detect_begin_async(struct sift_ctx *ctx, const float *d_img, int width, int height, size_t stride_px,
                            const sift_params *p);
int sift_detect_end_async(struct sift_ctx *ctx);

/* Software pipelining of consecutive images on contexts with their own
 * streams (ABI version >= 3): the next work enqueued on ctx waits until
 * prev's last enqueued detection has passed `after`:
 *   SIFT_AFTER_OCTAVE0     its octave-0 Gaussian+DoG (HBM-write bound) -- the
 *                          next image's octave 0 then overlaps prev's small
 *                          octaves, extrema scan and refinement;
 *   SIFT_AFTER_GAUSSIAN    its whole Gaussian+DoG pass;
 *   SIFT_AFTER_REFINEMENT  its fast refinement (only the latency-bound tail
 *                          overlaps).
 * No-op for contexts sharing one stream (already in order). */
enum { SIFT_AFTER_OCTAVE0 = 0, SIFT_AFTER_GAUSSIAN = 1, SIFT_AFTER_REFINEMENT = 2 };
int sift_order_after(struct sift_ctx *ctx, const struct sift_ctx *prev, int after);

int sift_last_timings(struct sift_ctx *ctx, sift_timings *t);

/* Per-octave Gaussian+DoG launch times of the last build / detection, ms
 * (ABI version >= 5): ms[o] for o < *n_octaves (0 for octaves not built).
 * Launch o is timed from the end of launch o-1 on the same stream, so with
 * other streams' work overlapping it includes the wait for CUs. */
int sift_last_octave_timings(struct sift_ctx *ctx, double *ms, int cap, int *n_octaves);

/* The kernels the last build / detection launched for its Gaussian+DoG pass
 * (ABI version >= 9), one entry per octave: "o0: k_gauss_dog<octave0>; o1:
 * k_gauss_rw<12>; ..." -- what bench.py's roofline.kernel reports.  Writes
 * at most cap bytes including the terminating NUL; *len = the full length
 * (excluding the NUL); SIFT_E_CAPACITY when cap is too small. */
int sift_last_pass_kernels(struct sift_ctx *ctx, char *buf, size_t cap, size_t *len);

/* Device-to-device copy of the last keypoints into caller device memory
 * (e.g. an RCCL all-gather send buffer), ordered on ctx's stream and
 * completed before return. */
int sift_copy_keypoints_device(struct sift_ctx *ctx, void *d_dst, size_t cap, size_t *n_out);

/* Raw device pointers (for in-process consumers that stay on device, e.g.
 * the RCCL all-gather of keypoints).  Valid until the next build/detect. */
int sift_device_keypoints(struct sift_ctx *ctx, const sift_keypoint **d_kp, size_t *n);
void *sift_stream(struct sift_ctx *ctx);

/* Row-band sharding of one image over several devices (ABI version >= 3;
 * SURVEY.md §8e cfg 5, no reference counterpart: the reference is one Web
 * Worker).  A shard runs the leading octaves on a crop of whole input rows
 * (sift_detect with num_octaves = K + 1, SIFT_F_EXPORT_NEXT_SEED and
 * SIFT_F_KEYPOINT_ORIGINS), keeps the keypoints whose candidate row it owns
 * and contributes its owned rows of the octave-(K+1) base; the base rows of
 * all shards make the whole base, from which sift_detect_from_seed runs the
 * trailing octaves.  The pipeline is translation invariant in y, so rows far
 * enough from a crop edge are bit-identical to the whole-image run. */

/* Input row of the first row of the images given to the following builds /
 * detections (a crop of whole rows of a taller image; default 0): keypoint
 * local_y / abs_y and origins are reported in the whole image's rows.  The
 * crop's first row must be a multiple of 2^(num_octaves - 1) (octave rows
 * stay whole). */
int sift_set_row_origin(struct sift_ctx *ctx, int input_row0);

/* Keep only the keypoints whose candidate lies in input rows [row_begin,
 * row_end) of the whole image (row_end < 0: to the bottom; row_begin < 0:
 * every keypoint, the default) in the following refinements / detections
 * (ABI version >= 5): a row band's share of a sharded image, decided by the
 * candidate's octave row as the band plan cuts it (octave 0: 2 r, octave o:
 * r >> (o - 1)).  Applied in the keypoint compaction on the device. */
int sift_set_owned_rows(struct sift_ctx *ctx, int row_begin, int row_end);

/* Kept keypoints per (octave, scale) block of the last refinement /
 * detection (ABI version >= 5): counts[o * S + s - 1], *n_blocks =
 * num_octaves * scales_per_octave.  Host memory; the keypoint list is in
 * block order, so these are its block boundaries
 * (sift_merge_keypoint_blocks_device). */
int sift_last_block_counts(struct sift_ctx *ctx, int64_t *counts, int cap, int *n_blocks);

/* The fp64 base of octave num_octaves formed by the last build with
 * SIFT_F_EXPORT_NEXT_SEED: rows x cols, row-major (host copy / device
 * pointer valid until the next build). */
int sift_next_seed(struct sift_ctx *ctx, double *dst, size_t cap, int *rows, int *cols);
int sift_device_next_seed(struct sift_ctx *ctx, const double **d_seed, int *rows, int *cols);

/* Detection of octaves octave_first .. num_octaves-1 of a width x height
 * input from the fp64 base of octave octave_first (>= 1; rows x cols as
 * sift_octave_dims gives, row-major, host or device memory).  Octave
 * indices, scales and absolute coordinates are those of the whole-image run. */
int sift_detect_from_seed(struct sift_ctx *ctx, int octave_first, const double *seed, int width, int height,
                          const sift_params *p, sift_keypoint *out, size_t cap, size_t *n_out);
int sift_detect_from_seed_device(struct sift_ctx *ctx, int octave_first, const double *d_seed, int width,
                                 int height, const sift_params *p, sift_keypoint *out, size_t cap,
                                 size_t *n_out);

/* Detection of a tail of octaves split over several devices (ABI version >= 5):
 * like sift_detect_from_seed_device, building octaves octave_first ..
 * p->num_octaves - 1 from the fp64 base of octave_first, but scanning only
 * octaves octave_scan_first .. p->num_octaves - 1 for extrema.  The octaves
 * before it are evaluated for their successor's base only (L[S] at even rows
 * and columns, bit-identical to the full build): they have no Gaussian or
 * DoG planes (sift_get_plane returns SIFT_E_STATE for them).  Rank j of a
 * row-band run builds the tail up to its octave and detects that one
 * octave. */
int sift_detect_from_seed_range_device(struct sift_ctx *ctx, int octave_first, int octave_scan_first,
                                       const double *d_seed, int width, int height, const sift_params *p,
                                       sift_keypoint *out, size_t cap, size_t *n_out);

/* Block-major merge of keypoint lists in device memory (ABI version >= 5):
 * d_in holds n_parts lists back to back; list q holds, in block order,
 * counts[q * n_blocks + b] keypoints of block b.  d_out receives block 0 of
 * every list in list order, then block 1, ...  With blocks = (octave, scale)
 * and lists = row bands in row order, this is the reference's candidate order
 * (octave, scale, y, x) without a sort.  A negative count skips that many
 * records of list q in d_in (padding, e.g. of an all-gather padded to the
 * largest list); they are not copied.  counts is host memory; completes
 * before return. */
int sift_merge_keypoint_blocks_device(struct sift_ctx *ctx, const sift_keypoint *d_in, const int64_t *counts,
                                      int n_parts, int n_blocks, sift_keypoint *d_out);

/* The candidate (octave, scale, y, x) of each keypoint of the last
 * detection/refinement run with SIFT_F_KEYPOINT_ORIGINS: 4 int32 per
 * keypoint, keypoint order (the reference's candidate order). */
int sift_keypoint_origins(struct sift_ctx *ctx, int32_t *out, size_t cap, size_t *n_out);

/* ---- Image products either side of the path (ABI version >= 4) ---------- */

/* ImageUtils_convertImageDataToMatrix2D({convertToGrayscale: true,
 * usePerceptualGrayscale: true}) (image-utils.js:27-152, called by
 * main.js:98-103) on device: gray = ((R*0.299) + (G*0.587) + (B*0.114)) / 255,
 * alpha = A / 255, evaluated in fp64 in that order and rounded once to fp32
 * (bit-identical to Float32Array.from(<the reference's gray Matrix2D>)).
 * `rgba` is ImageData.data (Uint8 R,G,B,A per pixel, row stride in bytes, a
 * multiple of 4); `gray` (required) and `alpha` (NULL = discardAlphaChannel)
 * are dense width*height fp32.  Host buffers here, device buffers in the
 * _device form (ordered on ctx's stream, completed before return). */
int sift_rgba_to_gray(struct sift_ctx *ctx, const uint8_t *rgba, int width, int height, size_t stride_bytes,
                      float *gray, float *alpha);
int sift_rgba_to_gray_device(struct sift_ctx *ctx, const uint8_t *d_rgba, int width, int height,
                             size_t stride_bytes, float *d_gray, float *d_alpha);

/* sift_build_scale_space / sift_detect from an RGBA ImageData (host): the
 * RGBA bytes are uploaded and converted on device (no host gray pass). */
int sift_build_scale_space_rgba(struct sift_ctx *ctx, const uint8_t *rgba, int width, int height,
                                size_t stride_bytes, const sift_params *p, const double *offset_sigmas);
int sift_detect_rgba(struct sift_ctx *ctx, const uint8_t *rgba, int width, int height, size_t stride_bytes,
                     const sift_params *p, sift_keypoint *out, size_t cap, size_t *n_out);

/* Preview ImageData of one plane of the context's pyramid, as the reference
 * posts them to its UI: ImageUtils_convertMatrix2DToImageData with a gray
 * channel (image-utils.js:171-217): p = Math.round(g * 255) stored as
 * (p, p, p, 255) with Uint8ClampedArray clamping, where g is
 *   SIFT_DISPLAY_PLAIN    the plane value (Gaussian images, background.js:139, :218)
 *   SIFT_DISPLAY_SIGMOID  1/(1+exp(coefficient*(-1*v))) (Matrix2D_sigmoidNormalize,
 *                         matrix2d.js:151; DoG chunks use 5, background.js:303)
 *   SIFT_DISPLAY_SAMPLED  (v-min)/(max-min) over the plane (Matrix2D_sampledNormalize,
 *                         matrix2d.js:169; DoG images, background.js:336, :387)
 * computed in fp64 from the fp32 plane.  `rgba` holds rows*cols*4 bytes
 * (cap_bytes); host memory, or device memory in the _device form. */
enum { SIFT_DISPLAY_PLAIN = 0, SIFT_DISPLAY_SIGMOID = 1, SIFT_DISPLAY_SAMPLED = 2 };
int sift_plane_image(struct sift_ctx *ctx, int kind, int octave, int scale, int mode, double coefficient,
                     uint8_t *rgba, size_t cap_bytes);
int sift_plane_image_device(struct sift_ctx *ctx, int kind, int octave, int scale, int mode,
                            double coefficient, uint8_t *d_rgba, size_t cap_bytes);

/* Device-resident forms for a shard driver that keeps everything on the GPU
 * (ABI version >= 4): the origins of sift_keypoint_origins decoded on
 * device into caller device memory (4 int32 per keypoint), and rows
 * [row_begin, row_end) of the octave-(num_octaves) base into caller device
 * memory.  Both complete before return. */
int sift_copy_keypoint_origins_device(struct sift_ctx *ctx, int32_t *d_dst, size_t cap, size_t *n_out);
int sift_copy_next_seed_device(struct sift_ctx *ctx, double *d_dst, size_t cap, int row_begin, int row_end);

/* Wait for all work queued on ctx's stream. */
int sift_synchronize(struct sift_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* SIFT_HIP_H */
