// 26-neighbour extrema scan with ordered, sort-free emission (gfx950).
//
// Replaces findCandidateKeypoints (background.js:359-450) and its kernel
// SIFT_findExtremas (sift.js:212-316): for DoG scales s = 1..S a pixel
// strictly greater (or strictly smaller) than all 26 neighbours, border
// excluded, is an extremum; |v| >= 0.8*thr makes it a candidate, otherwise
// it is a low-contrast extremum.  Output order is the reference's: octave,
// scale, then raster (y, x).
//
// k_extrema: one wave per (62-column word, strip of kXRows rows, group of up
// to 5 scales), sliding a 3-row window down the strip over all the group's
// DoG planes.  Lanes 1..62 are output columns, lanes 0 and 63 their halo, so
// x-1 / x+1 come from DPP wave shifts without extra loads.  Each plane row is
// reduced once (3-wide max/min) and shared by the scales above and below it;
// the 26-neighbour decision is 6 compares per scale, the rest is lane-mask
// logic whose result is the bitmap word [s][y][word] directly, plus a per-row
// popcount.  k_emit
// expands the bitmap in order after an exclusive scan of the row counts --
// the candidate list comes out sorted without a sort.
//
// The planes are fp32 roundings of fp64 values.  Rounding is monotone, so an
// fp32 comparison decides the fp64 one unless two fp32 values tie; ties and
// |v| within rounding of 0.8*thr go to a short list that k_exact_extrema
// re-decides from an fp64 pointwise recompute (sift_exact.h).
#include <cstdlib>
#include <type_traits>

#include "sift_exact.h"
#include "sift_kernels.h"
#include "sift_xmask.h"
#include "sift_refine.h"

#ifndef SIFT_XLOAD_AUX
#define SIFT_XLOAD_AUX 0  // cache-policy bits of the scan's DoG loads (gfx950: 1 sc0, 2 nt, 16 sc1)
#endif

namespace sift {

template <int NP>
struct XUnit {
  const float* base;   // DoG plane of the group's first plane, row 0
  long long plane;
  __amdgpu_buffer_rsrc_t rsrc;  // the group's DoG planes
  unsigned plane_bytes;  // < 4 GiB per group (launch_extrema checks)
  int w, h, y1;
  unsigned xoff;       // lane byte offset of its (clamped) column
  unsigned long long colmask;  // lanes with an interior output column
  int lane, xw, nw, s_first, o;
  unsigned key_base;   // key of (s_first, 0, 0)
  unsigned long long* bitmap;  // (s_first, row 0, word 0) of this octave
  unsigned* rowcount;          // (s_first, row 0) of this octave
  unsigned long long* lowbitmap;  // the same for the certain low-contrast extrema (LOWL)
  unsigned* lowrowcount;
  unsigned low;
  unsigned pbase, pcount;  // patch capture: the unit's first slot, slots taken
  __amdgpu_buffer_rsrc_t prsrc;  // the patch buffer (< 4 GiB: extrema_prepare checks)
  float* cap;          // SIFT_XREFINE: this wave's capture slots in LDS
  unsigned capa;       // ... their LDS byte address
  bool capture;        // patches are captured (L.patch or L.pre)
  long long word0;     // index of (s_first, row 0, word 0) in L.bitmap (ambiguous word list)
  long long boff;      // lane l < NP-2: l h nw + xw (scale s_first + l, row 0, this word)
  long long roff;      // lane l < NP-2: l h (scale s_first + l, row 0)
};

// SIFT_XGLDS: the rows stream through a per-wave LDS ring of kXRing rows
// (buffer_load_dword ... lds: no VGPR holds a row in flight), kXRing rows
// ahead instead of the three the register window affords.
#ifndef SIFT_XGLDS
#define SIFT_XGLDS 0
#endif
#ifndef SIFT_XRING
#define SIFT_XRING 5
#endif
constexpr int kXRing = SIFT_XRING;
[[maybe_unused]] constexpr int kXRingFloats = kXRing * (kXMaxGroup + 2) * 64;  // one wave's ring

template <int NP>
struct XRing {
  unsigned lds;     // LDS byte address of the wave's ring (wave-uniform)
  unsigned vaddr;   // ... + lane * 4
  int islot, cslot; // next slot to fill / to read
  int next, last;   // next row to issue; rows past `last` re-read it
};

// Issues row ring.next (clamped) into slot islot: NP loads, one per plane.
template <int NP>
__device__ __forceinline__ void x_issue(const XUnit<NP>& U, XRing<NP>& R) {
  const unsigned rofs = (unsigned)min(R.next, R.last) * (unsigned)U.w * 4u;
  const unsigned base = R.lds + (unsigned)(R.islot * NP * 256);
#pragma unroll
  for (int q = 0; q < NP; ++q)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(U.rsrc, (__attribute__((address_space(3))) void*)(size_t)(base + q * 256), 4,
                                             (int)U.xoff, (int)(rofs + (unsigned)q * U.plane_bytes), 0,
                                             SIFT_XLOAD_AUX);
  R.islot = R.islot + 1 == kXRing ? 0 : R.islot + 1;
  ++R.next;
}

// The oldest row in flight (kXRing rows are: wait until kXRing - 1 remain),
// read from its slot; its slot then takes the next row.
template <int NP>
__device__ __forceinline__ void x_take(const XUnit<NP>& U, XRing<NP>& R, float (&dst)[NP]) {
  constexpr int N = NP * (kXRing - 1);  // loads younger than the row (stores in between only make this wait longer)
  static_assert(N <= 63, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  const unsigned a = R.vaddr + (unsigned)(R.cslot * NP * 256);
#pragma unroll
  for (int q = 0; q < NP; ++q) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(dst[q]) : "v"(a), "i"(q * 256));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  R.cslot = R.cslot + 1 == kXRing ? 0 : R.cslot + 1;
  x_issue(U, R);
}

template <int NP>
__device__ __forceinline__ void x_load(const XUnit<NP>& U, float (&dst)[NP], int row) {
  // buffer loads: lane byte offset in a VGPR, row + plane offset in an SGPR
  const unsigned rofs = (unsigned)row * (unsigned)U.w * 4u;
#if defined(SIFT_X_PROBE2COL)  // timing probe: 8-byte loads, two columns per lane (half the waves)
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(
        U.rsrc, (int)U.xoff, (int)(rofs + (unsigned)q * U.plane_bytes), SIFT_XLOAD_AUX);
    dst[q] = __builtin_bit_cast(float, v[0]) + __builtin_bit_cast(float, v[1]);
  }
  return;
#endif
#pragma unroll
  for (int q = 0; q < NP; ++q)
    dst[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           U.rsrc, (int)U.xoff, (int)(rofs + (unsigned)q * U.plane_bytes),
                                           SIFT_XLOAD_AUX));
}

// Patch capture of scale q at centre row y (ExtremaLaunch.patch): each
// candidate's 19 first-step values come from three lanes -- its own column (9
// values) and the columns left and right of it (5 each) -- all already in the
// window, so no DPP moves.  The word's candidates take the next slots of the
// unit (a wave-uniform count: no atomics -- one global counter serialised
// ~600 K atomics at the L2, 0.42 -> 6.8 ms).  Returns the slot of the first
// one (~0u: the unit is out of slots, these candidates gather in the refinement).
// SIFT_XREFINE: the same fields go to the wave's LDS slots (U.cap, local slot
// numbers), field 19 = the candidate's key relative to U.key_base.
template <int NP, int A, int B, int C>
__device__ __forceinline__ unsigned x_capture(const XWin<NP>& Wn, XUnit<NP>& U, const ExtremaLaunch& L,
                                              const int Q, unsigned long long b, unsigned rel_key) {
  const unsigned cnt = (unsigned)__popcll(b);
  if (U.pcount + cnt > (unsigned)kPatchUnitSlots) return ~0u;
  const unsigned base = U.pbase + U.pcount;
#if SIFT_XREFINE
  // ds_write_b32 one value at a time (inline asm): left to itself the compiler
  // merges the fields into b64 / b96 / b128 stores, whose consecutive source
  // registers cost copies and ~20 VGPRs across the scan (a wave per SIMD).
  const unsigned sa = U.capa + U.pcount * (unsigned)(kPatchFloats * 4);
  U.pcount += cnt;
  constexpr int kStride = kPatchFloats * 4;
#define X_ST(v, vo, field) \
  asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(sa + (unsigned)(vo)), "v"(v), "i"(4 * (field)))
#else
  U.pcount += cnt;
  // Buffer stores of the window registers themselves: the slot's byte offset
  // in one VGPR, the word's first slot in an SGPR, the field in the
  // instruction's offset (16-byte or flat stores would copy each quad into
  // consecutive registers / keep 64-bit addresses: a wave per SIMD less).
  const int sb = (int)(base * (unsigned)(kPatchFloats * 4));
  constexpr int kStride = kPatchFloats * 4;
#define X_ST(v, voff, field) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), U.prsrc, (voff) + 4 * (field), sb, 0)
#endif
  const int lane = U.lane;
  if ((b >> lane) & 1ull) {  // the candidate's own column: d(k, a, 1)
    const int vo = (int)lane_prefix(b) * kStride;
    X_ST(Wn.cv[A][Q - 1], vo, 0); X_ST(Wn.cv[B][Q - 1], vo, 1); X_ST(Wn.cv[C][Q - 1], vo, 2);
    X_ST(Wn.cv[A][Q], vo, 3); X_ST(Wn.cv[B][Q], vo, 4); X_ST(Wn.cv[C][Q], vo, 5);
    X_ST(Wn.cv[A][Q + 1], vo, 6); X_ST(Wn.cv[B][Q + 1], vo, 7); X_ST(Wn.cv[C][Q + 1], vo, 16);
#if SIFT_XREFINE
    X_ST(__uint_as_float(rel_key), vo, 19);
#endif
  }
  if (lane < 63 && ((b >> (lane + 1)) & 1ull)) {  // left of a candidate: d(1, a, 0), d(0, 1, 0), d(2, 1, 0)
    const int vo = (int)lane_prefix(b >> 1) * kStride;
    X_ST(Wn.cv[A][Q], vo, 8); X_ST(Wn.cv[B][Q], vo, 9); X_ST(Wn.cv[C][Q], vo, 10);
    X_ST(Wn.cv[B][Q - 1], vo, 11); X_ST(Wn.cv[B][Q + 1], vo, 17);
  }
  if (lane > 0 && ((b >> (lane - 1)) & 1ull)) {  // right of a candidate: d(1, a, 2), d(0, 1, 2), d(2, 1, 2)
    const int vo = (int)lane_prefix(b << 1) * kStride;
    X_ST(Wn.cv[A][Q], vo, 12); X_ST(Wn.cv[B][Q], vo, 13); X_ST(Wn.cv[C][Q], vo, 14);
    X_ST(Wn.cv[B][Q - 1], vo, 15); X_ST(Wn.cv[B][Q + 1], vo, 18);
  }
  return base;
#undef X_ST
}

// v_writelane_b32 (no clang builtin here): lane LANE of dst = the uniform v.
template <int LANE>
__device__ __forceinline__ void x_writelane(unsigned& dst, unsigned v) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(dst) : "s"(v), "i"(LANE));
}

// f(std::integral_constant<int, Q>) for Q = LO..HI in order (compile-time scale index).
template <int LO, int HI, class F>
__device__ __forceinline__ void x_for(F&& f) {
  if constexpr (LO <= HI) {
    f(std::integral_constant<int, LO>{});
    x_for<LO + 1, HI>(f);
  }
}

// Centre row y (slots A = y-1, B = y, C = y+1): decide every scale of the group.
template <int NP, int A, int B, int C, bool LOWL>
__device__ __forceinline__ void x_centre(const XWin<NP>& Wn, XUnit<NP>& U, const ExtremaLaunch& L, int y) {
#if defined(SIFT_X_PROBE)  // timing probe: no decisions
  {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < NP; ++q) acc += Wn.hx[B][q] + Wn.hn[A][q];
    if (acc == 1234.5f) U.low += 1;
    return;
  }
#endif
  float vx[NP], vn[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    vx[q] = max3f(Wn.hx[A][q], Wn.hx[B][q], Wn.hx[C][q]);
    vn[q] = min3f(Wn.hn[A][q], Wn.hn[B][q], Wn.hn[C][q]);
  }
  // The row's bitmap words are built lane by lane: scale q's word (wave-
  // uniform, in SGPRs) goes to lane q - 1 with v_writelane -- one VALU per
  // half-word and scale; selecting it into place with a lane compare cost a
  // v_mov + v_cndmask per half-word, count and scale (and the same again for
  // the ambiguous word) -- a third of the scan's VALU per row.  Every lane
  // 0..NP-3 is written each row; the other lanes' contents are never used.
  unsigned wlo = __builtin_nondeterministic_value(0u), whi = __builtin_nondeterministic_value(0u);
  unsigned llo = __builtin_nondeterministic_value(0u), lhi = __builtin_nondeterministic_value(0u);  // LOWL
  unsigned wsl = ~0u;                   // lane q-1: patch slot of scale q's first candidate
  x_for<1, NP - 2>([&](auto qc) {
    constexpr int q = decltype(qc)::value;
    const float v = Wn.cv[B][q];
    const float nmax = max3f(vx[q - 1], vx[q + 1], max3f(Wn.hx[A][q], Wn.hx[C][q], Wn.ex[B][q]));
    const float nmin = min3f(vn[q - 1], vn[q + 1], min3f(Wn.hn[A][q], Wn.hn[C][q], Wn.en[B][q]));
    const unsigned key = U.key_base + (unsigned)(q - 1) * (unsigned)U.plane + (unsigned)y * (unsigned)U.w +
                         (unsigned)(U.xw * kXW - 1 + U.lane);
    unsigned long long lowmask, ambmask;
    const unsigned long long bit =
        x_row_decide(v, nmax, nmin, U.colmask, L.c_lo, L.c_hi, L.exact_planes != 0, key, &L.counters[0],
                     L.ambbitmap ? nullptr : L.amb_keys, L.amb_cap, U.low, lowmask, ambmask);

    if (ambmask && L.ambbitmap && U.lane == 0) {  // an ambiguous word (rare): its bits and its index for k_exact_words
      const unsigned long long aw = ambmask >> 1;  // lanes 1..62 -> bits 0..61
      const long long gw = U.word0 + ((long long)(q - 1) * U.h + y) * U.nw + U.xw;
      L.ambbitmap[gw] = aw;
      atomicAdd(&L.counters[0], (unsigned)__popcll(aw));
      const unsigned slot = atomicAdd(&L.counters[kAmbWords], 1u);
      if (slot < L.amb_cap) L.amb_keys[slot] = (unsigned)gw;
    }
    const unsigned long long word = bit >> 1;  // lanes 1..62 -> bits 0..61
    x_writelane<q - 1>(wlo, (unsigned)word);
    x_writelane<q - 1>(whi, (unsigned)(word >> 32));
    if (kXCapture && U.capture && bit) {
      const unsigned ps = x_capture<NP, A, B, C>(Wn, U, L, q, bit, key - U.key_base);
      if (U.lane == q - 1) wsl = ps;
    }
    if (LOWL) {
      const unsigned long long lw = lowmask >> 1;
      x_writelane<q - 1>(llo, (unsigned)lw);
      x_writelane<q - 1>(lhi, (unsigned)(lw >> 32));
    }
  });
#if defined(SIFT_X_PROBE3)  // timing probe: decisions without bitmap stores
  if (wlo == 0x12345u && whi == 0x777u) U.low += 1;
  return;
#endif
  if (U.lane < NP - 2) {
    // lane l stores scale s_first + l's word of row y: a uniform row pointer
    // plus the lane's (scale, word) offset
    const unsigned long long* const brow = U.bitmap + (long long)y * U.nw;
    const_cast<unsigned long long*>(brow)[U.boff] = ((unsigned long long)whi << 32) | wlo;
    if (kXCapture && U.capture && (wlo | whi)) L.wslot[U.word0 + ((long long)U.lane * U.h + y) * U.nw + U.xw] = wsl;
    const unsigned wcnt = (unsigned)(__popc(wlo) + __popc(whi));
    if (wcnt) atomicAdd(&U.rowcount[U.roff + y], wcnt);
    if (LOWL) {
      const_cast<unsigned long long*>(U.lowbitmap + (long long)y * U.nw)[U.boff] = ((unsigned long long)lhi << 32) | llo;
      const unsigned lcnt = (unsigned)(__popc(llo) + __popc(lhi));
      if (lcnt) atomicAdd(&U.lowrowcount[U.roff + y], lcnt);
    }
  }
}

#if SIFT_XREFINE
// The first refinement step of every candidate the unit captured (lane j takes
// slots j, j + 64, ...): refine_step on the fp32 planes with the fast pass's
// error bounds, exactly as k_refine_fast's first iteration from a captured
// patch; the outcome goes to pre[slot] (kPre* codes).
template <int NP>
__device__ __forceinline__ void x_first_steps(const Pyramid& P, const ExtremaLaunch& L, const XUnit<NP>& U) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the capture's ds_write_b32s (inline asm) have landed
  const int o = U.o;
  const unsigned plane = (unsigned)U.plane, w = (unsigned)U.w;
  const int moff = (P.row0 * 2) >> o;
  for (unsigned j = (unsigned)U.lane; j < U.pcount; j += 64) {
    const float* pp = U.cap + j * kPatchFloats;
    const float4 c0 = *reinterpret_cast<const float4*>(pp), c1 = *reinterpret_cast<const float4*>(pp + 4);
    const float4 lf = *reinterpret_cast<const float4*>(pp + 8), rt = *reinterpret_cast<const float4*>(pp + 12);
    const float4 ex = *reinterpret_cast<const float4*>(pp + 16);
    const unsigned rel = __float_as_uint(ex.w);
    const unsigned sq = rel / plane, rem = rel - sq * plane, mr = rem / w;
    const int s = U.s_first + (int)sq, m = (int)mr, n = (int)(rem - mr * w);
    const float v19[19] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, ex.x,
                           lf.x, lf.y, lf.z, lf.w, ex.y, rt.x, rt.y, rt.z, rt.w, ex.z};
    constexpr int at[19] = {1, 4, 7, 10, 13, 16, 19, 22, 25, 9, 12, 15, 3, 21, 11, 14, 17, 5, 23};
    double d[27];
    double mx = 0;
#pragma unroll
    for (int k = 0; k < 27; ++k) d[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 19; ++k) {
      d[at[k]] = (double)v19[k];
      mx = fmax(mx, fabs((double)v19[k]));
    }
    const double value = (double)c1.x;  // d(1, 1, 1)
    const double dval = fabs(value) * 0x1p-24;
    const double delta = mx * (0x1p-24 + 0x1p-40);
    const StepOut R = refine_step<true>(d, o, s, m, n, value, delta, dval, P.S, P.ND, U.h, U.w, P.thr, false,
                                        L.min_blur / L.min_interpixel_distance);
    Keypoint k;
    k.octave = kPreDefer;
    if (!R.uncertain) {
      if (R.state == 3) k.octave = kPreSingular;
      else if (R.state == 2) k.octave = kPreDiscard;
      else if (R.state == 1) {
        if (!R.imprecise) {
          make_keypoint(k, o, R, P.S, L.min_blur, L.min_interpixel_distance, moff);
          k.octave = kPreKeep;
        }
      } else {
        k.octave = kPreMoved;
        k.scale_level = R.s;
        k.local_y = R.m;
        k.local_x = R.n;
        k.interp_value = value;
      }
    }
    L.pre[U.pbase + j] = k;
  }
}
#endif

template <int NP, bool LOWL>
__device__ __forceinline__ void x_scan(const Pyramid& P, const ExtremaLaunch& L, int b, int u, int o, int s_first,
                                       int xw, int y0, int y1, float* cap, float* ring) {
  const Octave& oc = P.oct[o];
  XUnit<NP> U;
  U.plane = (long long)oc.h * oc.w;
  U.w = oc.w;
  U.h = oc.h;
  U.y1 = y1;
  U.lane = threadIdx.x & 63;
  U.xw = xw;
  U.nw = L.nw[o];
  U.s_first = s_first;
  U.o = o;
  const int x = xw * kXW - 1 + U.lane;
  U.xoff = 4u * (unsigned)clampi(x, 0, oc.w - 1);
#if defined(SIFT_X_PROBE2COL)
  if (xw & 1) return;
  U.xoff = 4u * (unsigned)clampi(2 * kXW * (xw >> 1) - 2 + 2 * U.lane, 0, oc.w - 2);
#endif
  U.plane_bytes = (unsigned)(4 * U.plane);
  U.colmask = __ballot(U.lane >= 1 && U.lane <= kXW && x >= 1 && x <= oc.w - 2);
  U.base = P.dog + b * P.dog_bstride + oc.dog_off + (long long)(s_first - 1) * U.plane;
  U.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(U.base), 0, -1, 0x00020000);
  U.key_base = (unsigned)b * P.kpi + oc.key_off + (unsigned)(s_first - 1) * (unsigned)U.plane;
  const long long wb = b * L.words_per_img + L.word_off[o] + (long long)(s_first - 1) * oc.h * U.nw;
  const long long rb = (long long)b * L.rows_per_img + L.row_off[o] + (s_first - 1) * oc.h;
  U.bitmap = L.bitmap + wb;
  U.word0 = wb;
  U.boff = ((long long)U.lane * U.h) * U.nw + xw;
  U.roff = (long long)U.lane * U.h;
  U.rowcount = L.rowcount + rb;
  if (LOWL) {
    U.lowbitmap = L.lowbitmap + wb;
    U.lowrowcount = L.lowrowcount + rb;
  }
  U.low = 0;
  U.pbase = (unsigned)(b * L.units_per_img + u) * (unsigned)kPatchUnitSlots;
  U.pcount = 0;
  U.capture = L.pre != nullptr || L.patch != nullptr;
  if (SIFT_XPATCH && L.patch) U.prsrc = __builtin_amdgcn_make_buffer_rsrc(L.patch, 0, -1, 0x00020000);

  U.cap = cap;
  U.capa = (unsigned)(size_t)(__attribute__((address_space(3))) float*)cap;
  XWin<NP> Wn;
#if SIFT_XGLDS
  XRing<NP> R;
  R.lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) float*)ring);
  R.vaddr = R.lds + 4u * (unsigned)U.lane;
  R.islot = R.cslot = 0;
  R.next = y0 - 1;
  R.last = y1 + 1;
#pragma unroll
  for (int k = 0; k < kXRing; ++k) x_issue(U, R);
  {
    float t[NP];
    x_take(U, R, t);
    x_derive<NP, 2>(Wn, t);
    x_take(U, R, t);
    x_derive<NP, 0>(Wn, t);
  }
  for (int y = y0; y <= y1; y += 3) {
    float t[NP];
    x_take(U, R, t);
    x_derive<NP, 1>(Wn, t);
    x_centre<NP, 2, 0, 1, LOWL>(Wn, U, L, y);
    if (y + 1 > y1) break;
    x_take(U, R, t);
    x_derive<NP, 2>(Wn, t);
    x_centre<NP, 0, 1, 2, LOWL>(Wn, U, L, y + 1);
    if (y + 2 > y1) break;
    x_take(U, R, t);
    x_derive<NP, 0>(Wn, t);
    x_centre<NP, 1, 2, 0, LOWL>(Wn, U, L, y + 2);
  }
  // the ring's last loads land in LDS: drained before the wave's LDS can be reallocated
  __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
#else
  {
    float r_m1[NP], r_0[NP];
    x_load(U, r_m1, y0 - 1);
    x_load(U, r_0, y0);
    x_load(U, Wn.raw[1], y0 + 1);
    x_load(U, Wn.raw[2], min(y0 + 2, y1 + 1));
    x_load(U, Wn.raw[0], min(y0 + 3, y1 + 1));
    x_derive<NP, 2>(Wn, r_m1);
    x_derive<NP, 0>(Wn, r_0);
  }
  // Each row's loads are issued three rows before it is derived (rows past
  // the strip re-read row y1+1 from L2 instead of branching).
  for (int y = y0; y <= y1; y += 3) {
    x_derive<NP, 1>(Wn, Wn.raw[1]);
    x_load(U, Wn.raw[1], min(y + 4, y1 + 1));
    x_centre<NP, 2, 0, 1, LOWL>(Wn, U, L, y);
    if (y + 1 > y1) break;
    x_derive<NP, 2>(Wn, Wn.raw[2]);
    x_load(U, Wn.raw[2], min(y + 5, y1 + 1));
    x_centre<NP, 0, 1, 2, LOWL>(Wn, U, L, y + 1);
    if (y + 2 > y1) break;
    x_derive<NP, 0>(Wn, Wn.raw[0]);
    x_load(U, Wn.raw[0], min(y + 6, y1 + 1));
    x_centre<NP, 1, 2, 0, LOWL>(Wn, U, L, y + 2);
  }
#endif
#if SIFT_XREFINE
  if (U.capture && U.pcount) {
    if constexpr (SIFT_XREFINE == 1) {
      x_first_steps<NP>(P, L, U);
    } else {  // SIFT_XREFINE=2: the LDS slots copied out whole (16-byte stores, contiguous per unit)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const float4* src = reinterpret_cast<const float4*>(U.cap);
      float4* dst = reinterpret_cast<float4*>(L.patch + (size_t)U.pbase * kPatchFloats);
      for (unsigned t = (unsigned)U.lane; t < U.pcount * (kPatchFloats / 4); t += 64) dst[t] = src[t];
    }
  }
#endif
  if (U.lane == 0 && U.low) atomicAdd(&L.counters[1], U.low);
}

// One wave per unit (octave, strip of kXRows rows, 62-column word, scale
// group): all DoG planes of the group stream through once, each plane's row
// is reduced once (3-wide max/min with DPP shifts) and shared by the scales
// above and below it; the decisions are SALU lane-mask logic.
// LOWL: also the bitmap of the certain low-contrast extrema (their list).
#ifndef SIFT_XMINW
#define SIFT_XMINW 1  // minimum waves per SIMD of the scan (register budget; experiments)
#endif

template <bool LOWL>
__global__ __launch_bounds__(256, SIFT_XMINW) void k_extrema(const Pyramid P, const ExtremaLaunch L) {
  // Blocks are dealt round-robin over the 8 XCDs (separate L2s).  With
  // xcd_band, XCD k scans the k-th contiguous range of units, so the lines
  // shared by horizontally adjacent words (their halo columns) and by
  // vertically adjacent strips (their halo rows) are fetched into one L2.
  int lb = (int)blockIdx.x;
  if (L.xcd_band) {
    const int nb = (int)gridDim.x, q = nb >> 3, rm = nb & 7, xc = lb & 7;
    lb = xc * q + min(xc, rm) + (lb >> 3);
  }
  // units of image b: b * span + (u - u_begin), span = u_end - u_begin
  const int span = L.u_end - L.u_begin;
  const int ug = lb * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (ug >= span * P.nimg) return;
  const int b = ug / span;
  const int u = L.u_begin + ug - b * span;
  int o = 0;
  while (o + 1 < L.n_oct && u >= L.unit_off[o + 1]) ++o;
  int loc = u - L.unit_off[o];
  const int g = loc % L.ng;
  loc /= L.ng;
  const int nw = L.nw[o];
  const int xw = loc % nw, strip = loc / nw;
  const int y0 = 1 + strip * kXRows, y1 = min(P.oct[o].h - 2, y0 + kXRows - 1);
  const int per = P.S / L.ng, rem = P.S % L.ng;
  const int s_first = 1 + g * per + min(g, rem);
  const int cnt = per + (g < rem ? 1 : 0);
#if SIFT_XREFINE
  __shared__ __attribute__((aligned(16))) float xcap[4][kPatchUnitSlots * kPatchFloats];
  float* const cap = xcap[threadIdx.x >> 6];
#else
  float* const cap = nullptr;
#endif
#if SIFT_XGLDS
  __shared__ __attribute__((aligned(16))) float xring[4][kXRingFloats];
  float* const ring = xring[threadIdx.x >> 6];
#else
  float* const ring = nullptr;
#endif
  switch (cnt) {
    case 1: x_scan<3, LOWL>(P, L, b, u, o, s_first, xw, y0, y1, cap, ring); break;
    case 2: x_scan<4, LOWL>(P, L, b, u, o, s_first, xw, y0, y1, cap, ring); break;
    case 3: x_scan<5, LOWL>(P, L, b, u, o, s_first, xw, y0, y1, cap, ring); break;
    case 4: x_scan<6, LOWL>(P, L, b, u, o, s_first, xw, y0, y1, cap, ring); break;
    default: x_scan<7, LOWL>(P, L, b, u, o, s_first, xw, y0, y1, cap, ring); break;
  }
}

// One wave per (scale, row) of one octave: expand the row's bitmap words in
// order at the row's offset.  Candidate values are the fp32 plane values
// (ambiguous ones get their exact fp64 value from k_exact_extrema).
__global__ __launch_bounds__(256) void k_emit(const Pyramid P, const EmitLaunch E) {
  if (E.n_out && blockIdx.x == 0 && threadIdx.x == 0) *E.n_out = E.rowoff[E.n_index];
  const int lane = threadIdx.x & 63;
  const int rpi = E.row_off[E.n_oct];
  const int r0 = E.row_off[E.o_first], act = rpi - r0;  // rows per image with decisions
  const int ga = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ga >= act * P.nimg) return;
  const int im = ga / act, gl = r0 + (ga - im * act);
  const int g = im * rpi + gl;  // global row (image-major)
  int o = E.o_first;
  while (o + 1 < E.n_oct && gl >= E.row_off[o + 1]) ++o;
  const Octave& oc = P.oct[o];
  const int h = oc.h, w = oc.w;
  const int row = gl - E.row_off[o];  // (s-1)*h + y within the octave
  const int s = row / h + 1, y = row - (s - 1) * h;
  if (y < 1 || y > h - 2) return;
  const unsigned cnt = E.rowcount[g];
  if (cnt == 0) return;
  unsigned base = E.rowoff[g];
  const long long plane = (long long)h * w;
  const float* __restrict__ Dc = P.dog + im * P.dog_bstride + oc.dog_off + s * plane + (long long)y * w;
  const unsigned kbase = (unsigned)im * P.kpi + oc.key_off + (unsigned)(s - 1) * (unsigned)plane + (unsigned)y * (unsigned)w;
  const int nw = E.nw[o];
  const long long wrow = im * E.words_per_img + E.word_off[o] + (long long)row * nw;
  const unsigned long long* bm = E.bitmap + wrow;
  const bool patched = E.cand_patch && ((E.patch_oct >> o) & 1u);
  for (int xw0 = 0; xw0 < nw; xw0 += 64) {
    const int xw = xw0 + lane;
    unsigned long long word = xw < nw ? bm[xw] : 0ull;
    unsigned ps = (patched && word) ? E.wslot[wrow + xw] : ~0u;  // patch slot of the word's first candidate
    unsigned c = (unsigned)__popcll(word);
    // inclusive wave scan of c
    unsigned inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned t = __shfl_up(inc, off);
      if (lane >= off) inc += t;
    }
    unsigned pos = base + inc - c;
    const int xb = xw * E.ww[o] + E.woff[o];  // column of bit 0
    while (word) {
      const int b = __ffsll((long long)word) - 1;
      word &= word - 1;
      const int x = xb + b;
      if (pos < E.cap) {
        E.keys[pos] = kbase + (unsigned)x;
        E.value[pos] = E.deferred ? __builtin_bit_cast(double, 0x7ff8000000000000ull) : (double)Dc[x];
        if (E.keep) E.keep[pos] = 1u;
        if (E.cand_patch) E.cand_patch[pos] = ps;
      }
      if (ps != ~0u) ++ps;
      ++pos;
    }
    base += __shfl(inc, 63);
  }
}

// One 64-thread block (one wave) per ambiguous candidate, persistent over the
// device-side count: fp64 recompute of the 3x3x3 patch decides extremum and
// contrast exactly.
__global__ __launch_bounds__(64) void k_exact_extrema(const Pyramid P, const ExactLaunch X) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const unsigned n_amb = min(X.counters[0], X.amb_cap);
  const unsigned n = min(*X.n, X.cap);
  for (unsigned j = blockIdx.x; j < n_amb; j += gridDim.x) {
    const unsigned key = X.amb_keys[j];
    int im, o, s, y, x;
    decode_key(P, key, im, o, s, y, x);
    // position of key in the ordered candidate list
    unsigned idx;
    if (X.bitmap) {  // the row's offset + the candidate bits before x (parallel loads, one wave reduction)
      const int h = P.oct[o].h;
      const int rr = (s - 1) * h + y;
      const long long wbase = im * X.words_per_img + X.word_off[o] + (long long)rr * X.nw[o];
      const int xr = x - X.woff[o], xw = xr / X.ww[o], b = xr - xw * X.ww[o];
      unsigned c = 0;
      for (int w = (int)threadIdx.x; w <= xw; w += 64) {
        unsigned long long word = X.bitmap[wbase + w];
        if (w == xw) word &= (1ull << b) - 1ull;
        c += (unsigned)__popcll(word);
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
      idx = X.rowoff[(long long)im * X.rows_per_img + X.row_off[o] + rr] + c;
    } else {  // binary search
      unsigned lo = 0, hi = n;
      while (lo < hi) {
        const unsigned mid = (lo + hi) >> 1;
        if (X.keys[mid] < key) lo = mid + 1; else hi = mid;
      }
      idx = lo;
    }
    double* d27 = smem;
    double* Lbuf = smem + 32;
    double* sh = smem + 32 + 40;
    wave_dog_patch(P, im, o, s, y, x, sh, Lbuf, d27);
    if (threadIdx.x == 0 && idx < n && X.keys[idx] == key) {
      const double v = d27[13];
      bool gt = false, lt = false;
      for (int q = 0; q < 27; ++q) {
        if (q == 13) continue;
        gt |= d27[q] >= v;  // a neighbour >= v rules out a strict maximum
        lt |= d27[q] <= v;
      }
      const bool ext = !gt || !lt;
      const bool cand = ext && fabs(v) >= P.pix_thr;
      X.keep[idx] = cand ? 1u : 0u;
      X.value[idx] = v;
      if (ext && !cand) {
        atomicAdd(&X.counters[1], 1u);
        if (X.late_keys) {  // decided low contrast here: joins the low-contrast list
          const unsigned slot = atomicAdd(&X.counters[6], 1u);
          if (slot < X.amb_cap) {
            X.late_keys[slot] = key;
            X.late_vals[slot] = v;
          }
        }
      }
      if (!cand) atomicAdd(&X.counters[2], 1u);  // dropped entries
    }
    __syncthreads();  // smem is reused by the next key
  }
}

// One wave per listed ambiguous word (persistent over the device-side
// count): the fp64 DoG values of the word's 64 columns (62 pixels and their
// x-1 / x+1 halo), rows y-1..y+1, DoG scales s-1..s+1, recomputed from the
// octave base with the same sums as k_gauss_dog / wave_dog_patch (vertical
// sums V in LDS -- every (L-scale, row, column) chain once --, then the
// horizontal sums), or read from the kept fp64 planes (l64).  Every
// ambiguous pixel of the word is then decided exactly, as k_exact_extrema
// decides one key: a saturated (flat) region makes whole words ambiguous,
// and one wave then settles 62 pixels instead of one.
constexpr int kWordPixelMax = 4;  // up to this many ambiguous pixels a word is settled pixel by pixel, one per wave
constexpr int kWordThreads = 256;  // 4 waves per word: the block's chains spread 4x wider (latency)

__global__ __launch_bounds__(kWordThreads) void k_exact_words(const Pyramid P, const ExactLaunch X) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned nwd = min(X.counters[kAmbWords], X.amb_cap);
  const unsigned n = min(*X.n, X.cap);
  const int VS = X.amb_lds_stride;
  double* V = smem;              // [t * 3 + a][cc], t < 4 L-scales, a < 3 rows, cc < 64 + 2 r_t
  double* Lb = smem + 12 * VS;   // [t * 3 + a][c], c < 64
  for (unsigned j = blockIdx.x; j < nwd; j += gridDim.x) {
    const long long gw = X.amb_keys[j];
    const int im = (int)(gw / X.words_per_img);
    const long long lw = gw - im * X.words_per_img;
    int o = 0;
    while (o + 1 < P.O && lw >= X.word_off[o + 1]) ++o;
    const Octave& oc = P.oct[o];
    const int h = oc.h, w = oc.w, nw = X.nw[o];
    const long long rel = lw - X.word_off[o];
    const int rr = (int)(rel / nw), xw = (int)(rel - (long long)rr * nw);
    const int s = rr / h + 1, y = rr - (s - 1) * h;
    const unsigned long long amb = X.ambbitmap[gw], cand = X.bitmap[gw];
    // list slot of the row's first candidate in this word
    unsigned c = 0;
    for (int q = lane; q < xw; q += 64) c += (unsigned)__popcll(X.bitmap[gw - xw + q]);  // (each wave the same)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
    const unsigned base = X.rowoff[(long long)im * X.rows_per_img + X.row_off[o] + rr] + c;
    const int x0 = xw * kXW - 1;  // column of lane 0 (lanes 1..62 <-> bits 0..61)
    // Exact decision of the pixel at lane ln (bit ln - 1) from the fp64 DoG
    // value v and its 26 neighbours (nb(k, a, dc)), written at its slot.
    auto settle = [&](int ln, double v, auto nb) {
      bool gt = false, lt = false;
      for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a)
          for (int dc = -1; dc <= 1; ++dc) {
            if (k == 1 && a == 1 && dc == 0) continue;
            const double d = nb(k, a, dc);
            gt |= d >= v;  // a neighbour >= v rules out a strict maximum
            lt |= d <= v;
          }
      const bool ext = !gt || !lt;
      const bool cnd = ext && fabs(v) >= P.pix_thr;
      const unsigned idx = base + (unsigned)__popcll(cand & ((1ull << (ln - 1)) - 1ull));
      const unsigned key = (unsigned)im * P.kpi + oc.key_off + (unsigned)(s - 1) * (unsigned)h * (unsigned)w +
                           (unsigned)y * (unsigned)w + (unsigned)(x0 + ln);
      if (idx < n && X.keys[idx] == key) {
        X.keep[idx] = cnd ? 1u : 0u;
        X.value[idx] = v;
        if (ext && !cnd) {
          atomicAdd(&X.counters[1], 1u);
          if (X.late_keys) {  // decided low contrast here: joins the low-contrast list
            const unsigned slot = atomicAdd(&X.counters[6], 1u);
            if (slot < X.amb_cap) {
              X.late_keys[slot] = key;
              X.late_vals[slot] = v;
            }
          }
        }
        if (!cnd) atomicAdd(&X.counters[2], 1u);  // dropped entries
      }
    };
    if (__popcll(amb) <= kWordPixelMax) {
      // a few ambiguous pixels: their 3x3x3 patches alone (wave_dog_patch,
      // 12 (2r + 3) chains each) cost less than the word's block (12 (64 +
      // 2r)); wave w takes the w-th pixel, in its own LDS slice
      double* d27 = smem + wv * X.amb_patch_stride;
      double* Lp = d27 + 32;
      double* sh = d27 + 32 + 40;
      unsigned long long m = amb;
      for (int i = 0; i < wv && m; ++i) m &= m - 1;
      if (m) {
        const int ln = __ffsll((long long)m);  // bit ln - 1 <-> lane ln
        wave_dog_patch(P, im, o, s, y, x0 + ln, sh, Lp, d27);
        if (lane == 0) settle(ln, d27[13], [&](int k, int a, int dc) { return d27[k * 9 + a * 3 + 1 + dc]; });
      }
      __syncthreads();  // the slices are reused by the next word
      continue;
    }
    if (oc.l64_off >= 0) {
      const long long plane = (long long)h * w;
      const double* L0 = P.l64 + im * P.l64_bstride + oc.l64_off;
      for (int i = tid; i < 12 * 64; i += kWordThreads) {
        const int ta = i >> 6, cl = i & 63;
        const int t = s - 1 + ta / 3, a = ta % 3;
        Lb[i] = L0[t * plane + (long long)(y - 1 + a) * w + clampi(x0 + cl, 0, w - 1)];
      }
    } else {
      for (int t4 = 0; t4 < 4; ++t4) {
        const int t = s - 1 + t4, r = oc.rad[t], nc = 64 + 2 * r;
        const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
        for (int idx = tid; idx < 3 * nc; idx += kWordThreads) {
          const int a = idx / nc, cc = idx - a * nc;
          const int xx = clampi(x0 - r + cc, 0, w - 1);
          const int yb = y - 1 + a - r;
          double acc = 0.0;  // the chain of wave_dog_patch, term for term
          for (int jb = 0; jb <= 2 * r; jb += kExactBatch) {
            double v[kExactBatch];
#pragma unroll
            for (int k = 0; k < kExactBatch; ++k) v[k] = base_at(P, im, o, clampi(yb + jb + k, 0, h - 1), xx);
#pragma unroll
            for (int k = 0; k < kExactBatch; ++k) acc = fma(wp[jb + k], v[k], acc);
          }
          V[(t4 * 3 + a) * VS + cc] = acc;
        }
      }
      __syncthreads();
      for (int ta = wv; ta < 12; ta += kWordThreads / 64) {
        const int t = s - 1 + ta / 3, r = oc.rad[t];
        const cdouble* wp = (const cdouble*)(P.wts + oc.wofs[t]);
        const double* vr = V + ta * VS + lane;
        double acc = 0.0;
        for (int i = 0; i <= 2 * r; ++i) acc = fma(wp[i], vr[i], acc);
        Lb[ta * 64 + lane] = acc;
      }
    }
    __syncthreads();
    if (wv == 0 && lane >= 1 && lane <= kXW && ((amb >> (lane - 1)) & 1ull)) {
      auto D = [&](int k, int a, int cl) { return Lb[(k * 3 + a) * 64 + cl] - Lb[((k + 1) * 3 + a) * 64 + cl]; };
      settle(lane, D(1, 1, lane), [&](int k, int a, int dc) { return D(k, a, lane + dc); });
    }
    __syncthreads();  // smem is reused by the next word
  }
}

size_t exact_words_lds_bytes(const Pyramid& P, int* stride, int* patch_stride) {
  int rmax = 0;
  for (int o = 0; o < P.O; ++o)
    if (P.oct[o].l64_off < 0) rmax = std::max(rmax, P.oct[o].rmax);
  *stride = 64 + 2 * rmax;
  *patch_stride = (int)(exact_lds_bytes(P) / sizeof(double));  // one wave_dog_patch slice per wave
  return std::max(sizeof(double) * (size_t)(12 * (*stride) + 12 * 64),
                  (size_t)(kWordThreads / 64) * exact_lds_bytes(P));
}

hipError_t launch_exact_words(const Pyramid& P, ExactLaunch X, hipStream_t st) {
  const size_t lds = exact_words_lds_bytes(P, &X.amb_lds_stride, &X.amb_patch_stride);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_exact_words, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)std::min<size_t>(lds, 160 * 1024));
    if (e != hipSuccess) return e;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
  }
  const unsigned grid = std::max(1u, std::min(X.amb_cap, 4096u));
  hipLaunchKernelGGL(k_exact_words, dim3(grid), dim3(kWordThreads), lds, st, P, X);
  return hipGetLastError();
}

static int extrema_unit_table(const Pyramid& P, int* unit_off, int* nw) {
  const int ng = (P.S + kXMaxGroup - 1) / kXMaxGroup;
  int units = 0;
  for (int o = 0; o < P.O; ++o) {
    const Octave& oc = P.oct[o];
    unit_off[o] = units;
    nw[o] = extrema_words_per_row(oc.w);
    if (oc.h >= 3 && oc.w >= 3 && P.S >= 1) units += ng * nw[o] * ((oc.h - 2 + kXRows - 1) / kXRows);
  }
  unit_off[P.O] = units;
  return units;
}

int extrema_units(const Pyramid& P) {
  int uo[kMaxOctaves + 1], nw[kMaxOctaves];
  return extrema_unit_table(P, uo, nw);
}

hipError_t launch_extrema(const Pyramid& P, ExtremaLaunch& L, hipStream_t st, int o_begin, int o_end) {
  L.n_oct = P.O;
  L.ng = (P.S + kXMaxGroup - 1) / kXMaxGroup;
  L.units_per_img = extrema_unit_table(P, L.unit_off, L.nw);
  L.u_begin = L.unit_off[o_begin];
  L.u_end = L.unit_off[o_end];
  if (L.u_end <= L.u_begin) return hipSuccess;
  // 32-bit buffer offsets cover one scale group's planes
  const int np = std::min(P.S, kXMaxGroup) + 2;
  if (4.0 * np * (double)P.oct[0].h * P.oct[0].w >= 4294967296.0) return hipErrorInvalidValue;
  // SIFT_XLDS (bytes, experiments): unused dynamic LDS per block, capping the
  // scan's blocks per CU (160 KiB / SIFT_XLDS) to leave CUs to other images.
  // Values outside [0, 160 KiB] are ignored.
  static const int xlds = [] {
    const int v = exp_knob("SIFT_XLDS", 0);
    return (v > 0 && v <= 160 * 1024) ? v : 0;
  }();
  // SIFT_XXCD=0: plain round-robin block order (experiments)
  static const int xxcd = exp_knob("SIFT_XXCD", 1);
  L.xcd_band = xxcd != 0;
  const void* fn = L.lowbitmap ? (const void*)k_extrema<true> : (const void*)k_extrema<false>;
  if (xlds > 65536) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, xlds);
    if (e != hipSuccess) return e;
  }
  const int nu = (L.u_end - L.u_begin) * std::max(1, P.nimg);
  if (L.lowbitmap) hipLaunchKernelGGL(k_extrema<true>, dim3((nu + 3) / 4), dim3(256), xlds, st, P, L);
  else hipLaunchKernelGGL(k_extrema<false>, dim3((nu + 3) / 4), dim3(256), xlds, st, P, L);
  return hipGetLastError();
}

hipError_t launch_emit(const Pyramid& P, const EmitLaunch& E, hipStream_t st) {
  if (E.o_first < 0 || E.o_first >= E.n_oct) return hipErrorInvalidValue;
  const int rows = (E.row_off[E.n_oct] - E.row_off[E.o_first]) * std::max(1, P.nimg);
  hipLaunchKernelGGL(k_emit, dim3(std::max(1, (rows + 3) / 4)), dim3(256), 0, st, P, E);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_zero_words(unsigned* a, long long na, unsigned* b, long long nb,
                                                    unsigned* c, long long nc) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb + nc; i += stride) {
    if (i < na) a[i] = 0u;
    else if (i < na + nb) b[i - na] = 0u;
    else c[i - na - nb] = 0u;
  }
}

hipError_t launch_zero_words(unsigned* a, long long na, unsigned* b, long long nb, unsigned* c, long long nc,
                             hipStream_t st) {
  if (!a) na = 0;
  if (!b) nb = 0;
  if (!c) nc = 0;
  const long long n = na + nb + nc;
  if (n <= 0) return hipSuccess;
  const int grid = (int)std::min<long long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_zero_words, dim3(grid), dim3(256), 0, st, a, na, b, nb, c, nc);
  return hipGetLastError();
}

size_t exact_lds_bytes(const Pyramid& P) {
  // octaves with kept fp64 planes (l64) read their patches, no scratch
  int rmax = 0;
  for (int o = 0; o < P.O; ++o)
    if (P.oct[o].l64_off < 0) rmax = std::max(rmax, P.oct[o].rmax);
  return sizeof(double) * (size_t)(32 + 40 + exact_scratch_doubles(rmax));
}

hipError_t launch_exact_extrema(const Pyramid& P, const ExactLaunch& X, hipStream_t st) {
  const unsigned grid = std::max(1u, std::min(X.amb_cap, 4096u));
  const size_t lds = exact_lds_bytes(P);
  if (lds > 64 * 1024) {  // scratch of radii above ~335
    const hipError_t e = hipFuncSetAttribute((const void*)k_exact_extrema, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_exact_extrema, dim3(grid), dim3(64), lds, st, P, X);
  return hipGetLastError();
}

}  // namespace sift
