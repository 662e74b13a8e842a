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

#include "sift_refine.h"

namespace sift {

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
    // (with SIFT_XREFINE=1 cand_patch indexes L.pre instead: no patch buffer)
    const bool patched = pidx != ~0u && (SIFT_XREFINE != 1 || L.patch);
    const float* __restrict__ pp = L.patch + (size_t)(patched ? pidx : 0u) * kPatchFloats;
    double value = L.cand_val[i];
    int status = kRefDiscard;
    int it0 = 0;
#if SIFT_XREFINE == 1
    // The scan's first step (L.pre): taken on the fp32 plane value, so only
    // for candidates whose value is still deferred (an exact re-decision
    // writes the fp64 value, and the chain starts over from it).
    if (!EXACT && L.pre && pidx != ~0u && value != value) {
      const Keypoint pr = L.pre[pidx];
      if (pr.octave == kPreKeep) {
        Keypoint k = pr;
        k.octave = o;
        L.kp[i] = k;
        status = kRefKeep;
        it0 = 5;
      } else if (pr.octave == kPreDiscard) {
        it0 = 5;
      } else if (pr.octave == kPreSingular) {
        status = kRefSingular;
        it0 = 5;
      } else if (pr.octave == kPreMoved) {
        s = pr.scale_level;
        m = pr.local_y;
        n = pr.local_x;
        value = pr.interp_value;
        it0 = 1;
      }
    }
#endif
    if (value != value)  // deferred: the fp32 plane value
      value = patched ? (double)pp[4] : (double)D[s * plane + (long long)m * w + n];
    const double dval = EXACT ? 0.0 : fabs(value) * 0x1p-24;
    double d[27];
    for (int it = it0; it < 5; ++it) {
      double mx = 0;
      if (it == 0 && patched) {
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

// Keep flag of slot i < cap of a list of m candidates (and the block starts it opens).
__device__ __forceinline__ bool keep_slot(const Pyramid& P, const int* __restrict__ status,
                                          const unsigned* __restrict__ key, int i, int m, int own_lo, int own_hi,
                                          unsigned* __restrict__ blk) {
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
  return k;
}

__global__ __launch_bounds__(256) void k_status_to_keep(const Pyramid P, const int* __restrict__ status,
                                                        const unsigned* __restrict__ key,
                                                        unsigned* __restrict__ keep, const unsigned* __restrict__ n,
                                                        int cap, int own_lo, int own_hi,
                                                        unsigned* __restrict__ blk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cap) return;
  const int m = (int)min(*n, (unsigned)cap);
  keep[i] = keep_slot(P, status, key, i, m, own_lo, own_hi, blk) ? 1u : 0u;
}

// ---------------------------------------------------------------------------
// Compaction bounded by the device count (launch_keep_compact): the slots are
// cut into tiles of kKeepTile; only the tiles up to the one holding slot m
// (= min(*n, cap)) do any work, where a capacity-sized device scan reads and
// writes every slot (4.6 M at 8K: 26 us for the scan alone, whatever m is).
// k_keep_flags: keep flags and block starts (keep_slot), one count per tile;
// k_keep_scan: exclusive scan of the tile counts (one workgroup);
// k_keep_scatter: pos[i] (in-tile prefix by wave ballots) and the kept
// keypoints' copies.  pos[i] is written for every slot of the tiles <= m's,
// so pos[m] (m < cap) is the total, as launch_count_keypoints reads it.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned block_sum256(unsigned c, unsigned* ws) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if (lane == 0) ws[w] = c;
  __syncthreads();
  return ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void k_keep_flags(const Pyramid P, const int* __restrict__ status,
                                                    const unsigned* __restrict__ key, unsigned* __restrict__ keep,
                                                    const unsigned* __restrict__ n, int cap, int own_lo, int own_hi,
                                                    unsigned* __restrict__ blk, unsigned* __restrict__ tile) {
  const int m = (int)min(*n, (unsigned)cap);
  const int t0 = blockIdx.x * kKeepTile;
  if (t0 > m) return;  // block-uniform: tiles past the count are never read
  __shared__ unsigned ws[4];
  unsigned c = 0;
#pragma unroll
  for (int k = 0; k < kKeepTile / 256; ++k) {
    const int i = t0 + k * 256 + (int)threadIdx.x;
    if (i < cap) {
      const bool f = keep_slot(P, status, key, i, m, own_lo, own_hi, blk);
      keep[i] = f ? 1u : 0u;
      c += f ? 1u : 0u;
    }
  }
  const unsigned tot = block_sum256(c, ws);
  if (threadIdx.x == 0) tile[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_keep_scan(unsigned* __restrict__ tile, const unsigned* __restrict__ n,
                                                    int cap) {
  __shared__ unsigned ws[16];
  const int m = (int)min(*n, (unsigned)cap);
  const int nt = min((cap + kKeepTile - 1) / kKeepTile, m / kKeepTile + 1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned carry = 0;
  for (int b0 = 0; b0 < nt; b0 += 1024) {
    const int b = b0 + (int)threadIdx.x;
    const unsigned v = b < nt ? tile[b] : 0u;
    unsigned x = v;  // inclusive scan within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned t = __shfl_up(x, d, 64);
      if (lane >= d) x += t;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    unsigned before = 0, all = 0;
    for (int q = 0; q < 16; ++q) {
      before += q < w ? ws[q] : 0u;
      all += ws[q];
    }
    if (b < nt) tile[b] = carry + before + x - v;
    carry += all;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_keep_scatter(const unsigned* __restrict__ keep, const unsigned* __restrict__ tile,
                                                      const Keypoint* __restrict__ kp, const unsigned* __restrict__ n,
                                                      int cap, unsigned* __restrict__ pos, Keypoint* __restrict__ out) {
  const int m = (int)min(*n, (unsigned)cap);
  const int t0 = blockIdx.x * kKeepTile;
  if (t0 > m) return;
  __shared__ unsigned ws[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned carry = tile[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kKeepTile / 256; ++k) {
    const int i = t0 + k * 256 + (int)threadIdx.x;
    const bool f = i < cap && keep[i] != 0u;
    const unsigned long long bal = __ballot(f);
    if (lane == 0) ws[k & 1][w] = (unsigned)__popcll(bal);
    __syncthreads();
    unsigned off = carry;
    for (int q = 0; q < w; ++q) off += ws[k & 1][q];
    const unsigned p = off + (unsigned)__popcll(bal & below);
    if (i < cap) pos[i] = p;
    if (f && i < m) out[p] = kp[i];
    carry += ws[k & 1][0] + ws[k & 1][1] + ws[k & 1][2] + ws[k & 1][3];
  }
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

// Keypoint records split into the field arrays callers take (ints: octave,
// scale_level, local_x, local_y; reals: abs_sigma, abs_x, abs_y,
// interp_value), so the host receives them by DMA with no reshuffle.
__global__ __launch_bounds__(256) void k_kp_soa(const Keypoint* __restrict__ kp, int n, int4* __restrict__ ints,
                                                double2* __restrict__ reals) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const Keypoint k = kp[i];
  ints[i] = make_int4(k.octave, k.scale_level, k.local_x, k.local_y);
  reals[2 * i] = make_double2(k.abs_sigma, k.abs_x);
  reals[2 * i + 1] = make_double2(k.abs_y, k.interp_value);
}

hipError_t launch_kp_soa(const Keypoint* kp, int n, int32_t* ints, double* reals, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_kp_soa, dim3((n + 255) / 256), dim3(256), 0, st, kp, n, reinterpret_cast<int4*>(ints),
                     reinterpret_cast<double2*>(reals));
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
  // SIFT_REFINE_LDS (experiments): dynamic LDS bytes per block, to cap the
  // blocks per CU (the candidates in flight, i.e. the DoG lines an XCD's L2
  // must hold at once).
  static const int lds = exp_knob("SIFT_REFINE_LDS", 0);
  if (R.exact_planes) hipLaunchKernelGGL(k_refine_fast<true>, dim3((R.cap + 255) / 256), dim3(256), lds, st, P, R);
  else hipLaunchKernelGGL(k_refine_fast<false>, dim3((R.cap + 255) / 256), dim3(256), lds, st, P, R);
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

hipError_t launch_keep_compact(const Pyramid& P, const int* status, const unsigned* key, unsigned* keep,
                               unsigned* pos, unsigned* tile, const unsigned* n, int cap, int own_lo, int own_hi,
                               unsigned* blk, const Keypoint* kp, Keypoint* out, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  const int nt = (int)keep_tiles(cap);
  hipLaunchKernelGGL(k_keep_flags, dim3(nt), dim3(256), 0, st, P, status, key, keep, n, cap, own_lo, own_hi, blk,
                     tile);
  hipLaunchKernelGGL(k_keep_scan, dim3(1), dim3(1024), 0, st, tile, n, cap);
  hipLaunchKernelGGL(k_keep_scatter, dim3(nt), dim3(256), 0, st, keep, tile, kp, n, cap, pos, out);
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
