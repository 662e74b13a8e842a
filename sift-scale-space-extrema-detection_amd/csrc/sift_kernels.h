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

#ifndef SIFT_FX
#define SIFT_FX 60
#endif
constexpr int kFX = SIFT_FX; // fused extrema: tile stride in x (64 computed columns, 60 owned, 60 decided)
constexpr int kFY = 30;      // ... in y (32 computed rows, 30 owned, 30 decided)

// Extrema decisions fused into the Gaussian+DoG pass of one octave (see
// k_gauss_dog): bitmap words of kFX columns, word bx of a row = tile column
// bx, bit b <-> x = kFX bx + 1 + b.
struct FusedExtrema {
  unsigned long long* bitmap;  // (scale 1, row 0, word 0) of the octave: [S][h][nw]
  unsigned* rowcount;          // (scale 1, row 0) of the octave: [S][h]
  int nw;                      // words per row (= tile columns of the launch)
  unsigned* amb_keys;          // keys needing an exact fp64 decision
  unsigned* counters;          // [0] ambiguous, [1] low-contrast
  unsigned amb_cap;
  float c_lo, c_hi;            // fp32 contrast thresholds (see ExtremaLaunch)
};

struct GaussLaunch {
  int o;
  int fuse;           // 1: extrema decisions of this octave in the same pass (X fields)
  FusedExtrema X;
  float* gauss;       // plane (o, 0) of the Gaussian pyramid, nullptr = do not store
  float* dog;         // plane (o, 0) of the DoG pyramid
  double* next_seed;  // base of octave o+1 (nullptr for the last octave)
  int next_w;
  const double* base; // fp64 octave base h x w (o >= 1: the seed; o == 0: only when materialised)
  double* l64;        // plane (o, 0) of the kept fp64 Gaussian planes, nullptr = not kept
  double* vsplit;     // large radii (gauss_vsplit): fp64 scratch of NS vertical-sum planes h x w, filled by a
                      // separate launch; the tile kernel copies its strip from it (nullptr = one pass)
  // filled by launch_gauss_dog
  int sw;             // strip row stride (doubles)
  int vec;            // float4 plane stores are aligned
  int zero;           // strips need zeroing (generic-radius path present)
  int dbg;            // timing experiments (SIFT_GAUSS_DBG): bit 0 = no plane stores
  int gb[kMaxScales + 1];  // scale groups: group g computes scales gb[g] .. gb[g+1]-1
  int gx, gy, G;      // tiles per row, tile rows, scale groups (1D grid of gx gy G blocks)
  int by0;            // first tile row of this launch (a band of tile rows by0 .. by0 + gy - 1)
  int xcd_band;       // 1: block -> tile so that each XCD runs a contiguous band of tile rows
  // batch: nimg images in one launch (blocks image-major); image im's
  // pointers are the fields above + im * these element strides
  int nimg;
  long long gauss_bs, dog_bs, seed_bs, base_bs, l64_bs, vsplit_bs;
};

constexpr int kXW = 62;      // output columns per extrema wave (lanes 1..62; lanes 0, 63 are halo)
#ifndef SIFT_XROWS
#define SIFT_XROWS 30
#endif
constexpr int kXRows = SIFT_XROWS;  // centre rows per extrema wave (multiple of 3)
#ifndef SIFT_XMAXGROUP
#define SIFT_XMAXGROUP 5
#endif
constexpr int kXMaxGroup = SIFT_XMAXGROUP;// scales per extrema wave (S > 5 splits the scales into groups)

// One launch scans every octave: unit u (one wave) = (octave, strip of kXRows
// rows, 62-column word, scale group).
struct ExtremaLaunch {
  int n_oct;
  int u_begin, u_end;            // units of this launch (a range of octaves)
  int exact_planes;              // DoG planes are the data itself (caller-supplied): no fp32 ties
  int ng;                        // scale groups per (strip, word)
  int xcd_band;                  // 1: block -> units so that each XCD scans a contiguous range of units
  float c_lo, c_hi;              // |v| < c_lo: certainly low contrast; |v| >= c_hi: certainly not
  int unit_off[kMaxOctaves + 1]; // first unit of each octave
  int nw[kMaxOctaves];           // words per row
  long long word_off[kMaxOctaves];  // first bitmap word of each octave ([S][h][nw])
  int row_off[kMaxOctaves];      // first row count of each octave ([S][h])
  unsigned long long* bitmap;
  unsigned* rowcount;
  unsigned* amb_keys;            // keys needing an exact fp64 decision (unordered)
  unsigned* counters;            // [0] ambiguous, [1] low-contrast, [2] dropped by exact pass
  unsigned amb_cap;
  unsigned long long* lowbitmap; // certain low-contrast extrema, same layout as bitmap (nullptr = not listed)
  unsigned* lowrowcount;
  long long words_per_img;       // batch (P.nimg images): image b's words / rows start b * these after image 0's
  int rows_per_img;
  // Ambiguous words (ambbitmap != nullptr): instead of one key per ambiguous
  // pixel, the scan writes the word's ambiguous bits to ambbitmap (same
  // layout as bitmap) and lists the word's index (into bitmap) in amb_keys
  // (counters[kAmbWords] of them); k_exact_words re-decides a whole word.
  unsigned long long* ambbitmap;
  // Patch capture (patch != nullptr): for every candidate bit the scan writes
  // the 19 fp32 DoG values of its first refinement step (kPatchFloats per
  // candidate) into its unit's kPatchUnitSlots slots -- unit (image b, u) owns
  // slots [(b * units_per_img + u) * kPatchUnitSlots, ...), taken in scan
  // order with a wave-uniform counter, no atomics -- and, for each non-zero
  // bitmap word, the slot of its first candidate to wslot (same index as
  // bitmap; ~0u: no patch, the unit's slots ran out: those candidates gather).
  float* patch;
  unsigned* wslot;
  int units_per_img;
  // First refinement step in the scan (pre != nullptr, SIFT_XREFINE builds):
  // the candidate's 19 values are captured into LDS instead of `patch`, and
  // after its strip the unit takes the first step of background.js:480-664
  // for each captured candidate (fp32 planes, the fast pass's error bounds),
  // writing its outcome to pre[slot] (kPre* in .octave; a kept keypoint's
  // record, or the position a move leads to with the candidate value in
  // interp_value).  The fast refinement continues from there.
  Keypoint* pre;
  double min_blur, min_interpixel_distance;
};
// pre[slot].octave: the first step's outcome (kPreDefer: uncertain or
// imprecise -- the fast refinement starts over from a gather).
constexpr int kPreMoved = 0, kPreKeep = 1, kPreDiscard = 2, kPreSingular = 3, kPreDefer = 4;
constexpr int kAmbWords = 8;     // counters slot: listed ambiguous words
#ifndef SIFT_PATCH_SLOTS
#define SIFT_PATCH_SLOTS 96
#endif
constexpr int kPatchUnitSlots = SIFT_PATCH_SLOTS;  // patch slots per scan unit (4K octave 0: ~40 candidates on average)
// Scan units per image (one wave each: octave, strip of kXRows rows, word, scale group).
int extrema_units(const Pyramid& P);
// Patch capture is built only into A/B libraries (-DSIFT_XPATCH=1): 4K
// extrema stage 0.40 -> 0.50 ms (148 instead of 111 VGPRs: 3 waves per SIMD;
// 19 dword stores per candidate) for a refinement stage 0.33 -> 0.27 ms,
// pipelined 7.10 -> 6.54 Gpix/s (profiles/r4p_patch_capture_ab.txt).
#ifndef SIFT_XPATCH
#define SIFT_XPATCH 0
#endif
#ifndef SIFT_XREFINE
#define SIFT_XREFINE 0
#endif
constexpr bool kXCapture = (SIFT_XPATCH != 0) || (SIFT_XREFINE != 0);  // the scan captures first-step patches (global / LDS)
// Captured patch of a candidate at (s, y, x), d(k, a, c) = D_{s-1+k}(y-1+a, x-1+c):
//   [0..8]   d(k, a, 1) at 3k + a (centre column, all three scales and rows) -- except d(2, 2, 1) at [16]
//   [8..11]  d(1, 0, 0), d(1, 1, 0), d(1, 2, 0), d(0, 1, 0)   (left column)
//   [12..15] d(1, 0, 2), d(1, 1, 2), d(1, 2, 2), d(0, 1, 2)   (right column)
//   [16..19] d(2, 2, 1), d(2, 1, 0), d(2, 1, 2), unused (LDS capture: the candidate's key - key of (s_first, 0, 0))
// Five 16-byte pieces: the centre lane writes 2 + 1, each side lane 1 + 1.
constexpr int kPatchFloats = 20;

// One launch over every octave: global row g (one wave each) = row_off[o] +
// (s-1) h_o + y.
struct EmitLaunch {
  int n_oct;
  int o_first;                   // first octave with decisions (earlier octaves' rows hold none: no waves)
  int row_off[kMaxOctaves + 1];  // first global row of each octave ([S][h] rows per octave)
  long long word_off[kMaxOctaves];  // first bitmap word of each octave
  int nw[kMaxOctaves];
  int ww[kMaxOctaves];           // columns per bitmap word: kXW (scan) or kFX (fused)
  int woff[kMaxOctaves];         // column of bit 0 of word 0: 0 (scan) or 1 (fused)
  const unsigned long long* bitmap;
  const unsigned* rowcount;      // [all rows]
  const unsigned* rowoff;        // exclusive scan of rowcount
  unsigned* keys;                // ordered candidate keys
  double* value;
  unsigned* keep;                // nullptr: not written
  unsigned cap;                  // slots in keys/value/keep (overflow is detected by the host)
  int deferred;                  // 1: value = NaN ("the fp32 plane value"): the refinement reads it from its
                                 // patch, launch_fill_values before the list is copied out; no plane gather here
  long long words_per_img;       // batch: bitmap words per image (rows per image = row_off[n_oct])
  // Patch indices (cand_patch != nullptr): cand_patch[pos] = wslot of the
  // word + the bit's rank in it for octaves in patch_oct (scanned with patch
  // capture), ~0u elsewhere.
  const unsigned* wslot;
  unsigned* cand_patch;
  unsigned patch_oct;
  unsigned* n_out;               // != nullptr: *n_out = rowoff[n_index] (the list's length), by thread 0
  long long n_index;
};

// Fills the deferred (NaN) candidate values of slots [0, *n) from the DoG planes.
hipError_t launch_fill_values(const Pyramid& P, const unsigned* keys, double* value, const unsigned* n, int cap,
                              hipStream_t st);

struct ExactLaunch {
  const unsigned* amb_keys;      // counters[0] of them (at most amb_cap stored)
  unsigned amb_cap;
  const unsigned* keys;          // ordered candidates
  const unsigned* n;             // device: number of candidates
  unsigned cap;
  unsigned* keep;
  double* value;
  unsigned* counters;            // [6]: late low-contrast extrema (ambiguous ones decided low)
  unsigned* late_keys;           // their keys / exact values (nullptr = not listed), amb_cap slots
  double* late_vals;
  // Emission geometry (EmitLaunch): a key's list position is its row's offset
  // plus the candidate bits before it in the row's bitmap words (bitmap ==
  // nullptr: binary search over keys).
  const unsigned long long* bitmap;
  const unsigned* rowoff;
  int row_off[kMaxOctaves];
  long long word_off[kMaxOctaves];
  int nw[kMaxOctaves], ww[kMaxOctaves], woff[kMaxOctaves];
  long long words_per_img;       // batch: bitmap words / rows per image
  int rows_per_img;
  const unsigned long long* ambbitmap;  // ambiguous words (k_exact_words; nullptr: amb_keys are pixel keys)
  int amb_lds_stride;            // k_exact_words: doubles per vertical-sum row (64 + 2 rmax)
  int amb_patch_stride;          // ... doubles per wave of the per-pixel patch scratch
};

struct RefineLaunch {
  const unsigned* cand_key;
  const double* cand_val;
  const unsigned* keep;  // nullptr = every entry is a candidate
  const unsigned* n;     // device: number of entries (<= cap)
  int cap;
  int exact_planes;
  double min_blur, min_interpixel_distance;
  int* status;        // per candidate kRef*
  Keypoint* kp;       // per candidate (valid where status == kRefKeep)
  unsigned* uncertain;// indices for the exact pass
  unsigned* counters; // [3] n uncertain, [4] n singular
  const unsigned* perm; // processing order: thread t refines slot perm[t] (nullptr = slot t)
  int wide_exact;       // k_refine_exact: 256 threads per patch (latency) instead of one wave (throughput)
  const unsigned* cand_patch;  // per slot: captured first-step patch (ExtremaLaunch.patch), ~0u = gather; nullptr = none
  const float* patch;
  const Keypoint* pre;  // != nullptr: cand_patch indexes the scan's first-step outcomes (ExtremaLaunch.pre) instead
};

// Processing order of the fast refinement (band_order): the slots of the
// extrema stage are ordered (octave, scale, row, column); the refinement
// takes them as (octave, band of kBandRows rows, scale, row, column) so the
// candidates whose 3x3x3 patches share DoG lines of adjacent scales run
// together (one XCD's L2) instead of a whole plane apart.
#ifndef SIFT_BAND_ROWS
#define SIFT_BAND_ROWS 16
#endif
constexpr int kBandRows = SIFT_BAND_ROWS;
struct BandOrder {
  int n_oct, S, n_items;
  int item_off[kMaxOctaves + 1];  // first item of each octave: items (band, scale) of octave o
  int row_off[kMaxOctaves + 1];   // first global row (o, s = 1, y = 0) of each octave in rowoff
  const unsigned* rowoff;         // exclusive scan of the extrema stage's row counts
  unsigned* count;                // per item: slots in it
  unsigned* first;                // per item: its first slot
  const unsigned* start;          // per item: exclusive scan of count (first position in the new order)
  unsigned* perm;                 // out: position -> slot
  int cap;
  int rows_per_img;               // batch: rowoff rows per image (items are image-major, item_off per image)
};
hipError_t launch_band_items(const Pyramid& P, const BandOrder& B, hipStream_t st);
hipError_t launch_band_fill(const Pyramid& P, const BandOrder& B, hipStream_t st);

size_t gauss_lds_bytes(const Pyramid& P, int o, bool fused = false);
// Octave o can run with its extrema decisions fused (GaussLaunch.fuse):
// octave 0 on the staged path, one scale group, a plane of at least 3 x 3.
bool gauss_can_fuse(const Pyramid& P, int o);
// Octave 0 radii above the unrolled range run on a materialised fp64 upsample
// of the input (4 H W doubles) instead of the staged input region.
bool gauss_needs_base0(const Pyramid& P);
hipError_t launch_upsample_base(const Pyramid& P, double* base0, hipStream_t st);
// The base of octave o+1 from octave o's base alone (no planes): L_o[S] at
// even rows / columns; vrow: seed_only_scratch(P, o) doubles.
size_t seed_only_scratch(const Pyramid& P, int o);
hipError_t launch_seed_only(const Pyramid& P, int o, const double* base, double* vrow, double* next, hipStream_t st);
// ty_end >= 0: only tile rows [ty_begin, ty_end) of the octave (a band;
// not for fused or split-pass octaves).
// kname (optional): the launches this call made, e.g. "k_gauss_rw<12>" or
// "k_gauss_vert + k_gauss_dog<64>" (a static string; sift_last_pass_kernels).
hipError_t launch_gauss_dog(const Pyramid& P, GaussLaunch L, hipStream_t st, int ty_begin = 0, int ty_end = -1,
                            const char** kname = nullptr);
int gauss_tile_rows(const Pyramid& P, int o);  // tile rows of octave o's Gaussian launch
constexpr int kGaussTileRows = 32;             // output rows per tile row
// Tile columns of a fused launch over a w-column octave (= bitmap words per row).
inline int fused_words_per_row(int w) { return w > 2 ? (w - 2 + kFX - 1) / kFX : 1; }
hipError_t launch_dog_from_gauss(const float* g, float* d, long long plane, int nd, hipStream_t st);

// Octave o stores its fp64 Gaussian planes too (GaussLaunch.l64): the exact
// passes then read the patch values instead of recomputing them.
bool gauss_keep_l64(const Pyramid& P, int o);

// Octave o runs the split vertical pass (GaussLaunch.vsplit scratch: NS x h x
// w doubles).
bool gauss_vsplit(const Pyramid& P, int o);
// Octave o (>= 1) runs k_gauss_rw (register-window tiles, 224 columns x 8 rows; no split pass).
bool gauss_wide(const Pyramid& P, int o);
// The octave-1 base straight from the input (bit-identical to the octave-0 launch's seeds).

// Fills the unit table of L (octave geometry) and launches the scan; returns
// the launch error.  L.bitmap words per octave: S * h * nw.
hipError_t launch_extrema(const Pyramid& P, ExtremaLaunch& L, hipStream_t st, int o_begin, int o_end);
inline int extrema_words_per_row(int w) { return (w + kXW - 1) / kXW; }
hipError_t launch_emit(const Pyramid& P, const EmitLaunch& E, hipStream_t st);
// Zeroes up to three word ranges in one launch (the extrema stage's counters
// and row counts: one kernel instead of hipMemsetAsync's body + tail fills each).
hipError_t launch_zero_words(unsigned* a, long long na, unsigned* b, long long nb, unsigned* c, long long nc,
                             hipStream_t st);
// One wave per ambiguous candidate: fp64 pointwise recompute of the 3x3x3 DoG patch.
// Persistent grid over the device-side count of ambiguous keys (no host sync).
hipError_t launch_exact_extrema(const Pyramid& P, const ExactLaunch& X, hipStream_t st);
// One wave per listed ambiguous word (ExtremaLaunch.ambbitmap mode).
hipError_t launch_exact_words(const Pyramid& P, ExactLaunch X, hipStream_t st);

hipError_t launch_refine_fast(const Pyramid& P, const RefineLaunch& R, hipStream_t st);
hipError_t launch_refine_exact(const Pyramid& P, const RefineLaunch& R, hipStream_t st);

// Order-preserving compaction helpers.
// Entries i >= *n (device count) of the cap-sized arrays are inactive.
hipError_t launch_scatter_keypoints(const unsigned* keep, const unsigned* pos, const Keypoint* kp,
                                    const unsigned* n, int cap, Keypoint* out, hipStream_t st);
// keep[i] = status[i] is a kept keypoint whose candidate row (whole-image
// octave rows, P.row0 applied) lies in the input rows [own_lo, own_hi) (own_lo
// < 0: every row; own_hi < 0: no upper bound).  blk (kBlkWords, zeroed by the
// caller) receives the first slot of every (octave, scale) block of the
// candidate list at blk[kBlkStart + b], b = o * S + s - 1 (candidates are in
// key order, so a block is a slot range), or sets blk[kBlkUnsorted] when the
// list is not in key order.
constexpr int kBlkN = 1024;  // blk[b]: kept keypoints of block b = (image, octave, scale) (launch_count_keypoints)
static_assert(kBlkN >= kMaxOctaves * kMaxScales, "one image's blocks");
constexpr int kBlkStart = kBlkN;                  // blk[kBlkStart + b], b <= O*S: first slot of block b
constexpr int kBlkUnsorted = kBlkStart + kBlkN + 1;
constexpr int kBlkWords = kBlkUnsorted + 1;
hipError_t launch_status_to_keep(const Pyramid& P, const int* status, const unsigned* key, unsigned* keep,
                                 const unsigned* n, int cap, int own_lo, int own_hi, unsigned* blk, hipStream_t st);
hipError_t launch_scatter_keys(const unsigned* keep, const unsigned* pos, const unsigned* key, const unsigned* n,
                               int cap, unsigned* out, hipStream_t st);
// launch_status_to_keep + an exclusive scan of keep into pos +
// launch_scatter_keypoints, with the work bounded by *n instead of cap: keep
// and pos are written for the slots of the tiles up to slot min(*n, cap)
// (what launch_count_keypoints and launch_scatter_keys read); tile holds
// keep_tiles(cap) words of scratch.
#ifndef SIFT_KEEP_SCAN
#define SIFT_KEEP_SCAN 1  // 0: capacity-sized device scan (the round-4 compaction; A/B builds)
#endif
constexpr int kKeepTile = 512;  // two slots per thread: 4K (714 K candidates) 1400 tiles
inline size_t keep_tiles(int cap) { return cap > 0 ? (size_t)(cap + kKeepTile - 1) / kKeepTile : 0; }
hipError_t launch_keep_compact(const Pyramid& P, const int* status, const unsigned* key, unsigned* keep,
                               unsigned* pos, unsigned* tile, const unsigned* n, int cap, int own_lo, int own_hi,
                               unsigned* blk, const Keypoint* kp, Keypoint* out, hipStream_t st);
// out = pos[n-1] + keep[n-1] (0 if n == 0): the number of keypoints; blk[b] =
// kept keypoints of block b, from the block starts and the exclusive scan pos
// (a histogram over the slots when the list was not in key order).
hipError_t launch_count_keypoints(const Pyramid& P, const unsigned* pos, const unsigned* keep, const unsigned* key,
                                  const unsigned* n, int cap, unsigned* out, unsigned* blk, hipStream_t st);

size_t exact_lds_bytes(const Pyramid& P);

// Block-major merge (sift_merge_keypoint_blocks_device) as copies of the
// nseg contiguous (part, block) runs: seg[3 i] = {source byte offset,
// destination byte offset, bytes}, cstart[i] = first 16-KiB chunk of run i,
// n_chunks = cstart[nseg] (device tables).
constexpr long long kMergeChunk = 16384;
hipError_t launch_merge_blocks(const Keypoint* in, const long long* seg, const long long* cstart, int nseg,
                               long long n_chunks, Keypoint* out, hipStream_t st);

// Keypoint records -> field arrays (4 int32 + 4 doubles per keypoint, sift_copy_keypoints_soa's layout).
hipError_t launch_kp_soa(const Keypoint* kp, int n, int32_t* ints, double* reals, hipStream_t st);

// keys -> 4 int32 per keypoint: octave, scale, whole-image octave row (row0 applied), x.
hipError_t launch_decode_origins(const Pyramid& P, const unsigned* keys, int n, int32_t* out, hipStream_t st);

// Image products either side of the path (sift_image.hip).
// gray/alpha rows are dense (w floats); alpha may be nullptr.
hipError_t launch_rgba_to_gray(const unsigned char* rgba, size_t stride_bytes, int w, int h, float* gray,
                               float* alpha, hipStream_t st);
// float2 partials needed by the sampled mode for an n-pixel plane.
int plane_image_parts(long long n);
hipError_t launch_plane_image(const float* plane, long long n, int mode, double coefficient, float2* parts,
                              unsigned* out, hipStream_t st);

}  // namespace sift
