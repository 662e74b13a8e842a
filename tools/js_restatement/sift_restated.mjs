// Single-threaded JavaScript restatement of the reference's detector -- the
// CPU baseline `cpu_baseline_js` (kind "restatement") of bench.py, and a
// second, independent check of the reference's algorithm in its own
// language.  Clean-room: written from the algorithm (the steps below cite the
// reference lines each one follows), not from the reference's files; planes
// are flat Float64Arrays rather than the reference's nested Arrays and chunk
// objects, so it measures the algorithm on one core, not the reference's
// data-structure overheads.  Not part of the product path.
//
//   node sift_restated.mjs img.f32 W H octaves scales [out.json [--lists]
//        [minBlur assumedBlur minInterpixelDistance]]   (defaults 0.8 0.5 0.5)
//
// img.f32: W*H little-endian float32 gray values in [0, 1].  Prints (or
// writes) {seconds, candidates, lowContrast, keypoints[, lists]}.

import fs from 'fs';

// background.js:84 / :118 -- 2x nearest upsample, then halving: 2H, ceil(h/2)
export function octaveDims(W, H, O) {
  const dims = [];
  let h = 2 * H, w = 2 * W;
  for (let o = 0; o < O; o++) {
    if (o > 0) { h = Math.ceil(h / 2); w = Math.ceil(w / 2); }
    dims.push([h, w]);
  }
  return dims;
}

// background.js:89-177 -- blur targets and the incremental sigma of each plane
export function blurSchedule(O, S, minBlur, assumedBlur) {
  const k = Math.pow(2, 1 / S), NS = S + 3;
  const level = [], offset = [];
  let base = minBlur;
  for (let o = 0; o < O; o++) {
    level.push([]); offset.push([]);
    for (let s = 0; s < NS; s++) {
      if (o > 0 && s === 0) {
        base = level[o - 1][S];
        level[o].push(base); offset[o].push(0);
      } else {
        const t = base * Math.pow(k, s), from = o === 0 ? assumedBlur : base;
        level[o].push(t); offset[o].push(Math.sqrt(t * t - from * from));
      }
    }
  }
  return { level, offset };
}

// sift.js:31-67 -- normalised (2r+1)^2 Gaussian, r = round(3 sigma), row-major
function kernel2d(sigma) {
  const r = Math.round(3 * sigma), n = 2 * r + 1, K = new Float64Array(n * n);
  const s2 = sigma * sigma;
  let total = 0;
  for (let i = 0; i < n; i++) {
    for (let j = 0; j < n; j++) {
      const a = i - r, b = j - r;
      const g = Math.exp(((a * a + b * b) / s2) * -0.5) / (2 * Math.PI * s2);
      K[i * n + j] = g; total += g;
    }
  }
  for (let q = 0; q < n * n; q++) K[q] /= total;
  return { K, n, r };
}

// sift.js:72-149 -- 2D convolution, clamped edges; kernel row i walks x, its
// column j walks y, x-offset outer and y-offset inner (the summation order)
function blur2d(src, h, w, sigma) {
  const { K, n, r } = kernel2d(sigma);
  const out = new Float64Array(h * w);
  const xs = new Int32Array(n), ys = new Int32Array(n);
  for (let y = 0; y < h; y++) {
    for (let j = 0; j < n; j++) ys[j] = Math.min(h - 1, Math.max(0, y + j - r)) * w;
    for (let x = 0; x < w; x++) {
      for (let i = 0; i < n; i++) xs[i] = Math.min(w - 1, Math.max(0, x + i - r));
      let acc = 0;
      for (let i = 0; i < n; i++) {
        const xi = xs[i], kr = i * n;
        for (let j = 0; j < n; j++) acc += src[ys[j] + xi] * K[kr + j];
      }
      out[y * w + x] = acc;
    }
  }
  return out;
}

// background.js:71-237 -- Gaussian scale space, S+3 planes per octave; each
// octave's base is plane S of the previous one sampled at even (y, x)
export function scaleSpace(img, W, H, O, S, minBlur = 0.8, assumedBlur = 0.5) {
  const dims = octaveDims(W, H, O), { offset } = blurSchedule(O, S, minBlur, assumedBlur);
  const pyr = [];
  let [h, w] = dims[0];
  let base = new Float64Array(h * w);
  for (let y = 0; y < h; y++) for (let x = 0; x < w; x++) base[y * w + x] = img[(y >> 1) * W + (x >> 1)];
  for (let o = 0; o < O; o++) {
    [h, w] = dims[o];
    if (o > 0) {
      const pw = dims[o - 1][1], seed = pyr[o - 1][S];
      base = new Float64Array(h * w);
      for (let y = 0; y < h; y++) for (let x = 0; x < w; x++) base[y * w + x] = seed[2 * y * pw + 2 * x];
    }
    const planes = [];
    for (let s = 0; s < S + 3; s++) planes.push(o > 0 && s === 0 ? base : blur2d(base, h, w, offset[o][s]));
    pyr.push(planes);
  }
  return { dims, pyr };
}

// background.js:258-354, sift.js:154-188 -- D[s-1] = L[s-1] - L[s]
export function differenceOfGaussians(pyr) {
  return pyr.map(planes => {
    const d = [];
    for (let s = 1; s < planes.length; s++) {
      const a = planes[s - 1], b = planes[s], q = new Float64Array(a.length);
      for (let i = 0; i < a.length; i++) q[i] = a[i] - b[i];
      d.push(q);
    }
    return d;
  });
}

// sift.js:285, background.js:572
export const contrastThreshold = S => ((Math.pow(2, 1 / S) - 1) / (Math.pow(2, 1 / 3) - 1)) * 0.015;

// background.js:359-450 + sift.js:212-316 -- strict 26-neighbour extrema of
// DoG scales 1..S, raster order; |v| >= 0.8 thr -> candidates, else low contrast
export function findExtrema(dog, dims, S) {
  const cand = [], low = [], thr = 0.8 * contrastThreshold(S);
  for (let o = 0; o < dog.length; o++) {
    const [h, w] = dims[o];
    for (let s = 1; s <= S; s++) {
      const A = dog[o][s - 1], B = dog[o][s], C = dog[o][s + 1];
      for (let y = 1; y < h - 1; y++) {
        for (let x = 1; x < w - 1; x++) {
          const c = B[y * w + x];
          let mn = true, mx = true;
          for (let dy = -1; dy <= 1 && (mn || mx); dy++) {
            const row = (y + dy) * w + x;
            for (let dx = -1; dx <= 1; dx++) {
              const a = A[row + dx], cc = C[row + dx];
              if (!(a > c) || !(cc > c)) mn = false;
              if (!(a < c) || !(cc < c)) mx = false;
              if (dy !== 0 || dx !== 0) {
                const b = B[row + dx];
                if (!(b > c)) mn = false;
                if (!(b < c)) mx = false;
              }
            }
          }
          if (mn || mx) (Math.abs(c) >= thr ? cand : low).push([o, s, x, y, c]);
        }
      }
    }
  }
  return { cand, low };
}

// matrix2d.js:236-482 -- inverse through minors / cofactors / adjugate;
// null when |det| < eps (the reference's TypeError, background.js:531)
function negInverse3(M) {
  const mn = [[0, 0, 0], [0, 0, 0], [0, 0, 0]];
  for (let i = 0; i < 3; i++) {
    for (let j = 0; j < 3; j++) {
      const q = [];
      for (let a = 0; a < 3; a++) if (a !== i) for (let b = 0; b < 3; b++) if (b !== j) q.push(M[a][b]);
      mn[i][j] = q[0] * q[3] - q[1] * q[2];
    }
  }
  const det = M[0][0] * mn[0][0] - M[0][1] * mn[0][1] + M[0][2] * mn[0][2];
  if (Math.abs(det) < Number.EPSILON) return null;
  const inv = [[0, 0, 0], [0, 0, 0], [0, 0, 0]];
  for (let i = 0; i < 3; i++) {
    for (let j = 0; j < 3; j++) inv[i][j] = ((mn[j][i] * ((i + j) & 1 ? -1 : 1)) / det) * -1;
  }
  return inv;
}

// background.js:455-685 -- up to 5 quadratic interpolation steps around each
// candidate; offset < 0.6 in all of (scale, y, x) -> contrast and edge tests
// on the interpolated point; otherwise move to the rounded position
export function refine(dog, dims, cands, S, minBlur = 0.8, minDist = 0.5) {
  const thr = contrastThreshold(S), edge = (11 * 11) / 10;
  const out = [];
  let singular = 0;
  for (const [o, s0, x0, y0, v0] of cands) {
    const [h, w] = dims[o], D = dog[o];
    let s = s0, m = y0, n = x0;
    const at = (ss, yy, xx) => D[ss][yy * w + xx];
    for (let it = 0; it < 5; it++) {
      const c = at(s, m, n);
      const g = [(at(s + 1, m, n) - at(s - 1, m, n)) / 2, (at(s, m + 1, n) - at(s, m - 1, n)) / 2,
        (at(s, m, n + 1) - at(s, m, n - 1)) / 2];
      const h11 = at(s + 1, m, n) + at(s - 1, m, n) - 2 * c;
      const h22 = at(s, m + 1, n) + at(s, m - 1, n) - 2 * c;
      const h33 = at(s, m, n + 1) + at(s, m, n - 1) - 2 * c;
      const h12 = (at(s + 1, m + 1, n) - at(s + 1, m - 1, n) - at(s - 1, m + 1, n) + at(s - 1, m - 1, n)) / 4;
      const h13 = (at(s + 1, m, n + 1) - at(s + 1, m, n - 1) - at(s - 1, m, n + 1) + at(s - 1, m, n - 1)) / 4;
      const h23 = (at(s, m + 1, n + 1) - at(s, m + 1, n - 1) - at(s, m - 1, n + 1) + at(s, m - 1, n - 1)) / 4;
      const inv = negInverse3([[h11, h12, h13], [h12, h22, h23], [h13, h23, h33]]);
      if (inv === null) { singular++; break; }
      const a = inv.map(r => r[0] * g[0] + r[1] * g[1] + r[2] * g[2]);
      if (Math.abs(a[0]) < 0.6 && Math.abs(a[1]) < 0.6 && Math.abs(a[2]) < 0.6) {
        const omega = v0 + (0.5 * a[0] * g[0] + 0.5 * a[1] * g[1] + 0.5 * a[2] * g[2]);
        if (Math.abs(omega) < thr) break;
        const tr = h22 + h33, dt = h22 * h33 - h23 * h23;
        if ((tr * tr) / dt > edge) break;
        const delta = Math.pow(2, o - 1);
        out.push([o, s, n, m, (delta / minDist) * minBlur * Math.pow(2, (a[0] + s) / S),
          delta * (a[2] + n), delta * (a[1] + m), omega]);
        break;
      }
      s = Math.round(s + a[0]); m = Math.round(m + a[1]); n = Math.round(n + a[2]);
      if (s < 1 || s >= S + 1 || m < 1 || m >= h - 1 || n < 1 || n >= w - 1) break;
    }
  }
  return { keypoints: out, singular };
}

export function detect(img, W, H, O, S, minBlur = 0.8, assumedBlur = 0.5, minDist = 0.5) {
  const { dims, pyr } = scaleSpace(img, W, H, O, S, minBlur, assumedBlur);
  const dog = differenceOfGaussians(pyr);
  const { cand, low } = findExtrema(dog, dims, S);
  const { keypoints, singular } = refine(dog, dims, cand, S, minBlur, minDist);
  return { cand, low, keypoints, singular };
}

const isMain = process.argv[1] && import.meta.url.endsWith(process.argv[1].split('/').pop());
if (isMain) {
  const [file, W, H, O, S, outPath, flag, mb, ab, md] = process.argv.slice(2);
  const buf = fs.readFileSync(file);
  const img = new Float32Array(buf.buffer, buf.byteOffset, buf.byteLength / 4);
  const t0 = process.hrtime.bigint();
  const r = detect(img, +W, +H, +O, +S, mb === undefined ? 0.8 : +mb, ab === undefined ? 0.5 : +ab,
    md === undefined ? 0.5 : +md);
  const sec = Number(process.hrtime.bigint() - t0) / 1e9;
  const res = { seconds: sec, candidates: r.cand.length, lowContrast: r.low.length, keypoints: r.keypoints.length,
    singular: r.singular, node: process.version };
  if (flag === '--lists') Object.assign(res, { lists: { candidates: r.cand, low: r.low, keypoints: r.keypoints } });
  const text = JSON.stringify(res);
  if (outPath) fs.writeFileSync(outPath, text); else console.log(text);
}
