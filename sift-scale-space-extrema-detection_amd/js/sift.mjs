// sift.mjs -- the reference's call surface, backed by the MI355X HIP path.
//
// Drop-in for the hot path of bingjetli/sift-scale-space-extrema-detection:
//   computeGaussianScaleSpace   background.js:71   (worker.js:29 argument names/defaults)
//   computeDifferenceOfGaussians background.js:258 (worker.js:54)
//   findCandidateKeypoints      background.js:359  (worker.js:64)
//   refineCandidateKeypoints    background.js:455  (worker.js:81)
//   WorkerMessageTypes          src/worker.js:5-24
//   createWorkerHandler         background.js:14-50 (message dispatcher)
// plus the north-star aliases buildScaleSpace / findCandidateKeypoints and a
// one-call detect()/detectAsync().
//
// Images are ImageData-shaped gray Float32: {width, height, data: Float32Array}.
// A Matrix2D (nested arrays, matrix2d.js) is accepted and rounded to fp32; an
// RGBA ImageData (Uint8ClampedArray data) is converted to gray on the device
// with the reference's perceptual weights (image-utils.js:27-152).
// Planes come back ImageData-shaped, or as Matrix2D with {matrix2d: true}
// (what main.js-style callers index as image[y][x]).
//
// Results of one stage carry a hidden handle to the device-resident state, so
// chaining the stages on their own outputs never re-uploads a pyramid; any
// other input (edited or foreign arrays) is uploaded and processed as given.
import { createRequire } from 'module';

const require = createRequire(import.meta.url);
const native = require('../napi/sift_napi.node');

export const WorkerMessageTypes = {
  COMPUTE_GAUSSIAN_SCALE_SPACE: 'compute-gaussian-scale-space',
  RECEIVED_GAUSSIAN_SCALE_SPACE: 'received-gaussian-scale-space',
  RECEIVED_GAUSSIAN_BLURRED_CHUNK: 'received-gaussian-blurred-chunk',
  RECEIVED_GAUSSIAN_BLURRED_IMAGE: 'received-gaussian-blurred-image',

  COMPUTE_DIFFERENCE_OF_GAUSSIANS: 'compute-difference-of-gaussians',
  RECEIVED_DIFFERENCE_OF_GAUSSIANS: 'received-difference-of-gaussians',
  RECEIVED_DIFFERENCE_OF_GAUSSIAN_CHUNK: 'received-difference-of-gaussian-chunk',
  RECEIVED_DIFFERENCE_OF_GAUSSIAN_IMAGE: 'received-difference-of-gaussian-image',

  FIND_CANDIDATE_KEYPOINTS: 'find-candidate-keypoints',
  RECEIVED_CANDIDATE_KEYPOINT_IMAGE: 'received-candidate-keypoint-image',
  RECEIVED_CANDIDATE_KEYPOINT_BASE_IMAGE: 'received-candidate-keypoint-base-image',
  RECEIVED_CANDIDATE_KEYPOINT_MARKER: 'received-candidate-keypoint-marker',
  RECEIVED_CANDIDATE_KEYPOINTS: 'received-candidate-keypoints',

  REFINE_CANDIDATE_KEYPOINTS: 'refine-candidate-keypoints',
  RECEIVED_REFINED_KEYPOINTS: 'received-refined-keypoints',
};

const PLANE_GAUSS = 0;
const PLANE_DOG = 1;
const HANDLE = Symbol('sift-device-state');

// ---------------------------------------------------------------------------
// Device contexts (one per device, created lazily).
// ---------------------------------------------------------------------------
const contexts = new Map();

function deviceState(device = 0) {
  let st = contexts.get(device);
  if (!st) {
    // pool: detectAsync's contexts (asyncPool; a native context is not
    // re-entrant, the addon rejects any call on it while its job runs).
    st = { ctx: native.createContext(device), device, gen: 0, stage: null, W: 0, H: 0, params: null, pool: null };
    contexts.set(device, st);
  }
  return st;
}

function bump(st, stage, W, H, params) {
  st.lastCtx = st.ctx;  // lastTimings: the context of the latest call
  st.gen += 1;
  st.stage = stage;
  st.W = W;
  st.H = H;
  st.params = params;
  return st.gen;
}

function attach(obj, st, gen, extra) {
  // configurable: a stale object (its device pyramid replaced since) is
  // re-uploaded and re-attached when a later stage is given it again
  Object.defineProperty(obj, HANDLE, { value: Object.assign({ st, gen }, extra), enumerable: false,
    configurable: true });
  return obj;
}

function liveHandle(obj) {
  const h = obj && obj[HANDLE];
  return h && h.st.gen === h.gen ? h : null;
}

// ---------------------------------------------------------------------------
// Images.
// ---------------------------------------------------------------------------
function isMatrix2D(m) {
  return Array.isArray(m) && m.length > 0 && (Array.isArray(m[0]) || ArrayBuffer.isView(m[0]));
}

function isRgba(img) {
  return !!img && (img.data instanceof Uint8ClampedArray || img.data instanceof Uint8Array) && img.width > 0 &&
    img.height > 0 && img.data.length === img.width * img.height * 4;
}

function toGray(img) {
  if (isRgba(img)) return { width: img.width, height: img.height, data: img.data, rgba: true };
  if (img && ArrayBuffer.isView(img.data) && img.width > 0 && img.height > 0) {
    const n = img.width * img.height;
    if (img.data.length < n) throw new TypeError('image.data is shorter than width*height');
    const data = img.data instanceof Float32Array ? img.data : Float32Array.from(img.data.subarray(0, n));
    return { width: img.width, height: img.height, data };
  }
  if (isMatrix2D(img)) {
    const height = img.length, width = img[0].length;
    const data = new Float32Array(width * height);
    for (let y = 0; y < height; y++) {
      const row = img[y];
      for (let x = 0; x < width; x++) data[y * width + x] = row[x];
    }
    return { width, height, data };
  }
  throw new TypeError('expected an ImageData-shaped {width, height, data} gray image or a Matrix2D');
}

function planeImage(data, width, height, matrix2d) {
  if (!matrix2d) return { width, height, data };
  const out = new Array(height);
  for (let y = 0; y < height; y++) out[y] = Array.from(data.subarray(y * width, (y + 1) * width));
  return out;
}

function planeDims(image) {
  if (isMatrix2D(image)) return [image.length, image[0].length];
  return [image.height, image.width];
}

function planeData(image) {
  if (isMatrix2D(image)) return toGray(image).data;
  return image.data instanceof Float32Array ? image.data : Float32Array.from(image.data);
}

function flatten(pyramid) {
  let total = 0;
  for (const oct of pyramid) for (const e of oct) { const [h, w] = planeDims(e.image); total += h * w; }
  const flat = new Float32Array(total);
  let off = 0;
  for (const oct of pyramid) for (const e of oct) { const d = planeData(e.image); flat.set(d, off); off += d.length; }
  return flat;
}

// Input (W, H) of a pyramid: octave 0 is the 2x upsample (background.js:84).
function inputDimsOf(pyramid) {
  const [h0, w0] = planeDims(pyramid[0][0].image);
  if (h0 % 2 || w0 % 2 || h0 < 2 || w0 < 2) {
    throw new RangeError('octave 0 of a pyramid is the 2x upsample of the input (background.js:84): even dims expected');
  }
  return [w0 / 2, h0 / 2];
}

// ---------------------------------------------------------------------------
// Schedule in JS, exactly as background.js:89-177 computes it (Math.pow),
// handed to the native side so blur levels and sigmas are bit-identical.
// ---------------------------------------------------------------------------
export function scaleSchedule(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur) {
  const NS = scales_per_octave + 3;
  const blur = new Float64Array(number_of_octaves * NS);
  const sigma = new Float64Array(number_of_octaves * NS);
  const k = Math.pow(2, 1 / scales_per_octave);
  let base = min_blur_level;
  for (let o = 0; o < number_of_octaves; o++) {
    for (let s = 0; s < NS; s++) {
      if (o > 0 && s === 0) {
        base = blur[(o - 1) * NS + scales_per_octave];
        blur[o * NS] = base;
        sigma[o * NS] = 0;
      } else {
        const target = base * Math.pow(k, s);
        const from = o === 0 ? assumed_blur : base;
        blur[o * NS + s] = target;
        sigma[o * NS + s] = Math.sqrt((target * target) - (from * from));
      }
    }
  }
  return { blur, sigma };
}

function nativeParams(O, S, min_blur, assumed_blur, mid = 0.5) {
  return { num_octaves: O, scales_per_octave: S, min_blur, assumed_blur, min_interpixel_distance: mid };
}

// ---------------------------------------------------------------------------
// Stage 1: computeGaussianScaleSpace (background.js:71-237).  The DoG of
// background.js:258 is formed in the same device pass and kept resident.
// ---------------------------------------------------------------------------
export function computeGaussianScaleSpace(args, ...rest) {
  let a = args;
  if (!a || a.input_image === undefined) {
    // positional form of background.js:71
    a = { input_image: args, number_of_octaves: rest[0], scales_per_octave: rest[1],
      min_blur_level: rest[2], assumed_blur: rest[3], chunk_size: rest[4], ...(rest[5] || {}) };
  }
  const {
    input_image, number_of_octaves = 5, scales_per_octave = 3, min_blur_level = 0.8,
    assumed_blur = 0.5, device = 0, matrix2d = false,
  } = a;  // chunk_size only shaped the reference's progress messages; it never changes values
  const img = toGray(input_image);
  const st = deviceState(device);
  const { blur, sigma } = scaleSchedule(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur);
  const params = nativeParams(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur);
  if (img.rgba) native.buildScaleSpaceRgba(st.ctx, img.data, img.width, img.height, params, sigma);
  else native.buildScaleSpace(st.ctx, img.data, img.width, img.height, params, sigma);
  const gen = bump(st, 'built', img.width, img.height, params);
  const NS = scales_per_octave + 3;
  const scaleSpace = [];
  for (let o = 0; o < number_of_octaves; o++) {
    const [h, w] = native.getDims(st.ctx, o);
    const oct = [];
    for (let s = 0; s < NS; s++) {
      oct.push({ blurLevel: blur[o * NS + s], image: planeImage(native.getPlane(st.ctx, PLANE_GAUSS, o, s), w, h, matrix2d) });
    }
    scaleSpace.push(oct);
  }
  return attach(scaleSpace, st, gen, { blur, matrix2d, params, kind: PLANE_GAUSS });
}
export const buildScaleSpace = computeGaussianScaleSpace;

// ---------------------------------------------------------------------------
// Stage 2: computeDifferenceOfGaussians (background.js:258-354):
// D[s-1] = L[s-1] - L[s], blurLevel of L[s-1].
// ---------------------------------------------------------------------------
export function computeDifferenceOfGaussians(scale_space, chunk_size = 32, { device = 0, matrix2d } = {}) {
  void chunk_size;
  let h = liveHandle(scale_space);
  let st, gen, blur, asM;
  if (h) {
    ({ st, gen } = h);
    blur = h.blur;
    asM = matrix2d === undefined ? h.matrix2d : matrix2d;
  } else {
    st = deviceState(device);
    const O = scale_space.length, NS = scale_space[0].length;
    const [W, H] = inputDimsOf(scale_space);
    const params = nativeParams(O, NS - 3, 0.8, 0.5);
    native.loadScaleSpace(st.ctx, flatten(scale_space), W, H, params);
    gen = bump(st, 'foreign-gauss', W, H, params);
    blur = new Float64Array(O * NS);
    for (let o = 0; o < O; o++) for (let s = 0; s < NS; s++) blur[o * NS + s] = scale_space[o][s].blurLevel;
    asM = matrix2d === undefined ? isMatrix2D(scale_space[0][0].image) : matrix2d;
  }
  const O = scale_space.length, NS = scale_space[0].length;
  const dog = [];
  for (let o = 0; o < O; o++) {
    const [hh, ww] = native.getDims(st.ctx, o);
    const oct = [];
    for (let s = 1; s < NS; s++) {
      oct.push({ blurLevel: blur[o * NS + s - 1], image: planeImage(native.getPlane(st.ctx, PLANE_DOG, o, s - 1), ww, hh, asM) });
    }
    dog.push(oct);
  }
  return attach(dog, st, gen, { kind: PLANE_DOG });
}

function ensureDog(differenceOfGaussians, scalesPerOctave, device) {
  const h = liveHandle(differenceOfGaussians);
  if (h) return h.st;
  const st = deviceState(device);
  const O = differenceOfGaussians.length;
  const S = differenceOfGaussians[0].length - 2;
  if (scalesPerOctave !== undefined && scalesPerOctave !== S) {
    // the reference would index past the pyramid; keep its threshold argument but the data's shape
  }
  const [W, H] = inputDimsOf(differenceOfGaussians);
  const params = nativeParams(O, S, 0.8, 0.5);
  native.loadDog(st.ctx, flatten(differenceOfGaussians), W, H, params);
  const gen = bump(st, 'foreign-dog', W, H, params);
  attach(differenceOfGaussians, st, gen, { kind: PLANE_DOG });
  return st;
}

// ---------------------------------------------------------------------------
// Stage 3: findCandidateKeypoints (background.js:359-450).
// Output [octave][scale-1] = {scaleLevel, localExtremas: [{x, y, value}]}.
// ---------------------------------------------------------------------------
export function findCandidateKeypoints(args, octave_base_images, scales_per_octave) {
  let a = args;
  if (!a || a.differenceOfGaussians === undefined) {
    a = { differenceOfGaussians: args, octaveBaseImages: octave_base_images, scalesPerOctave: scales_per_octave };
  }
  // octaveBaseImages: unused (background.js:361).  withLowContrast: also
  // return SIFT_findExtremas' lowContrastKeypoints (an extra bitmap, scan and
  // host copy; the worker's preview stream asks for it, the keypoint path
  // does not).
  const { differenceOfGaussians, scalesPerOctave, device = 0, withLowContrast = false } = a;
  const st = ensureDog(differenceOfGaussians, scalesPerOctave, device);
  const r = native.findExtrema(st.ctx, !!withLowContrast);
  const O = differenceOfGaussians.length;
  const S = differenceOfGaussians[0].length - 2;
  const group = (ints, values) => {  // [octave][scale-1] = {scaleLevel, localExtremas: [{x, y, value}]}
    const out = [];
    for (let o = 0; o < O; o++) {
      const oct = [];
      for (let s = 1; s <= S; s++) oct.push({ scaleLevel: s, localExtremas: [] });
      out.push(oct);
    }
    for (let i = 0; i < values.length; i++) {
      const o = ints[4 * i], s = ints[4 * i + 1];
      out[o][s - 1].localExtremas.push({ x: ints[4 * i + 2], y: ints[4 * i + 3], value: values[i] });
    }
    return out;
  };
  const out = group(r.ints, r.values);
  Object.defineProperty(out, 'lowContrastCount', { value: r.lowContrast, enumerable: false });
  // SIFT_findExtremas' lowContrastKeypoints (sift.js:293-306), same shape; the
  // reference does not return them, it posts one marker each (background.js:408-413)
  if (withLowContrast) {
    Object.defineProperty(out, 'lowContrastKeypoints', { value: group(r.lowInts, r.lowValues), enumerable: false });
  }
  return attach(out, st, st.gen, { n: r.values.length });
}

// ---------------------------------------------------------------------------
// Stage 4: refineCandidateKeypoints (background.js:455-685).  Like the
// reference, a Hessian with |det| < Number.EPSILON raises a TypeError and no
// list is returned (matrix2d.js:482 -> :455).
// ---------------------------------------------------------------------------
export function refineCandidateKeypoints(args, candidate_keypoints, scales_per_octave, number_of_octaves,
  min_blur_level, min_interpixel_distance = 0.5) {
  let a = args;
  if (!a || a.differenceOfGaussians === undefined) {
    a = { differenceOfGaussians: args, candidateKeypoints: candidate_keypoints, scalesPerOctave: scales_per_octave,
      numberOfOctaves: number_of_octaves, minBlurLevel: min_blur_level, minInterpixelDistance: min_interpixel_distance };
  }
  const {
    differenceOfGaussians, scalesPerOctave, numberOfOctaves, candidateKeypoints, minBlurLevel,
    minInterpixelDistance = 0.5, device = 0, throwOnSingular = true,
  } = a;
  const st = ensureDog(differenceOfGaussians, scalesPerOctave, device);
  const hc = liveHandle(candidateKeypoints);
  if (!hc) {
    // upload the (possibly edited or foreign) candidate lists in reference order (background.js:468-471)
    let n = 0;
    for (let o = 0; o < numberOfOctaves; o++) for (let s = 0; s < scalesPerOctave; s++) n += candidateKeypoints[o][s].localExtremas.length;
    const ints = new Int32Array(4 * n), vals = new Float64Array(n);
    let i = 0;
    for (let o = 0; o < numberOfOctaves; o++) {
      for (let s = 0; s < scalesPerOctave; s++) {
        const sc = candidateKeypoints[o][s];
        for (const e of sc.localExtremas) {
          ints[4 * i] = o; ints[4 * i + 1] = sc.scaleLevel; ints[4 * i + 2] = e.x; ints[4 * i + 3] = e.y;
          vals[i] = e.value;
          i++;
        }
      }
    }
    native.setCandidates(st.ctx, ints, vals);
  }
  native.setRefineParams(st.ctx, minBlurLevel === undefined ? 0.8 : minBlurLevel, minInterpixelDistance);
  const r = native.refine(st.ctx);
  if (r.singular > 0 && throwOnSingular) {
    throw new TypeError("Cannot read property 'length' of null (singular Hessian in refinement, as in the reference)");
  }
  return keypointsFromNative(r);
}

// Keypoints as the caller asked for them: 'objects' (default: the
// reference's keypoint objects, background.js:660-671) or 'typed' (no
// per-keypoint objects: {count, ints, doubles}, ints = [octave, scaleLevel,
// localX, localY] and doubles = [absoluteSigma, absoluteX, absoluteY,
// interpolatedValue] per keypoint, in the reference's order).
function keypointsOut(r, format) {
  if (format === 'typed') return { count: r.ints.length / 4, ints: r.ints, doubles: r.doubles };
  if (format !== undefined && format !== 'objects') throw new TypeError(`unknown keypoint format '${format}'`);
  return keypointsFromNative(r);
}

function keypointsFromNative(r) {
  const n = r.ints.length / 4;
  const out = new Array(n);
  for (let i = 0; i < n; i++) {
    out[i] = {
      octave: r.ints[4 * i], scaleLevel: r.ints[4 * i + 1], localX: r.ints[4 * i + 2], localY: r.ints[4 * i + 3],
      absoluteSigma: r.doubles[4 * i], absoluteX: r.doubles[4 * i + 1], absoluteY: r.doubles[4 * i + 2],
      interpolatedValue: r.doubles[4 * i + 3],
    };
  }
  return out;
}

// ---------------------------------------------------------------------------
// One-call fast path: all four stages on device, keypoints out.
// ---------------------------------------------------------------------------
export function detect(input_image, { number_of_octaves = 5, scales_per_octave = 3, min_blur_level = 0.8,
  assumed_blur = 0.5, min_interpixel_distance = 0.5, device = 0, format } = {}) {
  const img = toGray(input_image);
  const st = deviceState(device);
  const params = nativeParams(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur, min_interpixel_distance);
  const r = img.rgba ? native.detectRgba(st.ctx, img.data, img.width, img.height, params)
    : native.detect(st.ctx, img.data, img.width, img.height, params);
  bump(st, 'detected', img.width, img.height, params);
  return keypointsOut(r, format);
}

// A batch of independent images of one size (BASELINE cfg 4's images per
// GPU) as ONE detection (sift_detect_batch: one launch per stage over the
// batch); returns one keypoint list per image, each exactly what detect()
// returns for that image.
export function detectBatch(images, { number_of_octaves = 5, scales_per_octave = 3, min_blur_level = 0.8,
  assumed_blur = 0.5, min_interpixel_distance = 0.5, device = 0, format } = {}) {
  if (!images.length) return [];
  const grays = images.map(toGray);
  const { width, height } = grays[0];
  if (grays.some((g) => g.width !== width || g.height !== height || g.rgba)) {
    throw new TypeError('detectBatch: gray images of one size');
  }
  const n = width * height;
  const data = new Float32Array(n * grays.length);
  grays.forEach((g, b) => data.set(g.data.subarray(0, n), b * n));
  const st = deviceState(device);
  const params = nativeParams(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur, min_interpixel_distance);
  const r = native.detectBatch(st.ctx, data, grays.length, width, height, params);
  bump(st, 'detected', width, height, params);
  const out = [];
  let at = 0;
  if (format === 'typed') {
    for (const c of r.counts) {
      out.push({ count: c, ints: r.ints.subarray(4 * at, 4 * (at + c)), doubles: r.doubles.subarray(4 * at, 4 * (at + c)) });
      at += c;
    }
    return out;
  }
  const all = keypointsOut(r, format);
  for (const c of r.counts) { out.push(all.slice(at, at + c)); at += c; }
  return out;
}

// Asynchronous detections run on a pool of `inflight` contexts per device
// (default 4 below 4 Mpix, 3 from there up -- the pool sizes measured best on
// MI355X with Node's 4 hardware queues, profiles/r5ah_js_inflight_probe.txt;
// each context has its own HIP stream and pyramid), so up to that many
// images are on the GPU at once and one image's host work (H2D of the
// input, keypoint copy, result conversion) overlaps the others' device
// work.  Jobs beyond the pool wait in FIFO order.  The pool's first context
// is the device's synchronous one: a synchronous call on the device while a
// job runs on it throws (SIFT_E_BUSY), as before.
function asyncPool(st, inflight) {
  if (!st.pool) st.pool = { ctxs: [{ ctx: st.ctx, busy: false }], waiters: [] };
  const want = Math.max(1, inflight | 0);
  while (st.pool.ctxs.length < want) st.pool.ctxs.push({ ctx: native.createContext(st.device), busy: false });
  return st.pool;
}

function releaseSlot(pool, slot) {
  const i = pool.waiters.findIndex((w) => pool.ctxs.indexOf(slot) < w.limit);
  if (i >= 0) {
    const [w] = pool.waiters.splice(i, 1);
    w.resolve(slot);  // handed over still busy
  } else {
    slot.busy = false;
  }
}

function defaultInflight(img) {
  const px = img && Number.isFinite(img.width) && Number.isFinite(img.height) ? img.width * img.height : 0;
  return px > 0 && px < 4e6 ? 4 : 3;
}

export function detectAsync(input_image, opts = {}) {
  const { number_of_octaves = 5, scales_per_octave = 3, min_blur_level = 0.8, assumed_blur = 0.5,
    min_interpixel_distance = 0.5, device = 0, format } = opts;
  const inflight = opts.inflight !== undefined ? opts.inflight : defaultInflight(input_image);
  const st = deviceState(device);
  const pool = asyncPool(st, inflight);
  const limit = Math.max(1, inflight | 0);
  const start = (slot) => {
    let job;
    try {
      let img = toGray(input_image);
      if (img.rgba) {
        img = { width: img.width, height: img.height,
          data: native.rgbaToGray(slot.ctx, img.data, img.width, img.height, false).gray };
      }
      const params = nativeParams(number_of_octaves, scales_per_octave, min_blur_level, assumed_blur, min_interpixel_distance);
      if (slot.ctx === st.ctx) bump(st, 'detecting', img.width, img.height, params);
      job = native.detectAsync(slot.ctx, img.data, img.width, img.height, params);
    } catch (e) {
      releaseSlot(pool, slot);
      return Promise.reject(e);
    }
    return job.then((r) => {
      releaseSlot(pool, slot);
      st.lastCtx = slot.ctx;
      return keypointsOut(r, format);
    }, (e) => {
      releaseSlot(pool, slot);
      throw e;
    });
  };
  // A free context starts the job before this returns; otherwise it waits.
  const free = pool.ctxs.slice(0, limit).find((c) => !c.busy);
  if (free) {
    free.busy = true;
    return start(free);
  }
  return new Promise((resolve) => pool.waiters.push({ resolve, limit })).then(start);
}

// Counts and timings of the device's latest call: a synchronous one, or the
// last detectAsync job to settle (whichever of the pool's contexts ran it).
export function lastCounts(device = 0) {
  const st = deviceState(device);
  return native.counts(st.lastCtx || st.ctx);
}

// Device stage times of the last call chain on a device (HIP events, ms:
// gaussDogMs, extremaMs, refineMs, h2dMs, gaussOct0Ms) and the host wall
// time of its last keypoint copy to the host (d2hMs).
export function lastTimings(device = 0) {
  const st = deviceState(device);
  return native.timings(st.lastCtx || st.ctx);
}

// ---------------------------------------------------------------------------
// Image products either side of the path (SURVEY.md §8f rows 2-3), on device.
// ---------------------------------------------------------------------------

// ImageUtils_convertImageDataToMatrix2D (image-utils.js:27-152), gray forms:
// gray = ((R*0.299) + (G*0.587) + (B*0.114)) / 255 (both grayscale flavours
// use the perceptual weights in the reference) and alpha = A / 255, returned
// as the reference returns them (gray, or [gray, alpha]) -- Matrix2D, or
// ImageData-shaped Float32 with {matrix2d: false}.  Values are the fp32
// rounding of the reference's fp64 ones (the path's Float32 image contract).
export function convertImageDataToMatrix2D({ imageData, convertToGrayscale = false, usePerceptualGrayscale = false,
  discardAlphaChannel = false, device = 0, matrix2d = true } = {}) {
  void usePerceptualGrayscale;  // image-utils.js:106-111: both branches use the perceptual weights
  if (convertToGrayscale !== true) {
    throw new RangeError('only the grayscale conversion feeds the SIFT path; split RGB channels on the host');
  }
  if (!isRgba(imageData)) throw new TypeError('expected an RGBA ImageData {width, height, data: Uint8ClampedArray}');
  const { width, height } = imageData;
  const r = native.rgbaToGray(deviceState(device).ctx, imageData.data, width, height, !discardAlphaChannel);
  const gray = planeImage(r.gray, width, height, matrix2d);
  return discardAlphaChannel ? gray : [gray, planeImage(r.alpha, width, height, matrix2d)];
}

const DISPLAY_MODES = { plain: 0, sigmoid: 1, sampled: 2 };

// Preview ImageData of plane (octave, scale) of a live stage result (the
// scale space or the DoG pyramid), as ImageUtils_convertMatrix2DToImageData
// (image-utils.js:171-217) makes them from the plain plane (Gaussian
// images, background.js:139/:218), Matrix2D_sigmoidNormalize(.., coefficient)
// (DoG chunks, background.js:303) or Matrix2D_sampledNormalize (DoG images,
// background.js:336/:387).  Chunk previews are crops of the whole-plane ones.
export function planeImageData(pyramid, octave, scale, { mode = 'plain', coefficient = 5 } = {}) {
  const h = liveHandle(pyramid);
  if (!h || h.kind === undefined) throw new TypeError('expected a live scale-space or difference-of-Gaussians result');
  const m = DISPLAY_MODES[mode];
  if (m === undefined) throw new RangeError('mode must be plain, sigmoid or sampled');
  const [rows, cols] = native.getDims(h.st.ctx, octave);
  return { width: cols, height: rows, data: native.planeImage(h.st.ctx, h.kind, octave, scale, m, coefficient) };
}

// Chunk previews (background.js:181-203, :294-321): crops of a plane preview
// over ImageUtils_generateChunkBoundaries' tiles (image-utils.js:295-332:
// x-major, the last tile of a row / column shortened to the image).
function postChunks(post, type, img, chunk) {
  const { width: W, height: H, data } = img;
  for (let x = 0; x < W; x += chunk) {
    const cw = x + chunk >= W ? W - x : chunk;
    for (let y = 0; y < H; y += chunk) {
      const ch = y + chunk >= H ? H - y : chunk;
      const out = new Uint8ClampedArray(cw * ch * 4);
      for (let r = 0; r < ch; r++) out.set(data.subarray(((y + r) * W + x) * 4, ((y + r) * W + x + cw) * 4), r * cw * 4);
      post({ type, imageData: { width: cw, height: ch, data: out }, dx: x, dy: y });
    }
  }
}

// ---------------------------------------------------------------------------
// background.js-compatible dispatcher (background.js:14-50): returns an
// onmessage(e) that answers each request with the reference's RECEIVED_*
// message.  Pyramids go out as Matrix2D by default, as the reference posts
// them (main.js indexes image[y][x]).  With {previews: true} every progress
// message of the reference is posted too, in its order, with device-made
// ImageData: per-chunk and per-plane Gaussian previews
// (RECEIVED_GAUSSIAN_BLURRED_CHUNK / _IMAGE), per-chunk sigmoid(5) and
// per-plane sampled DoG previews (RECEIVED_DIFFERENCE_OF_GAUSSIAN_CHUNK /
// _IMAGE), and per (octave, scale) the sampled base image, the low-contrast
// markers, the candidate markers and RECEIVED_CANDIDATE_KEYPOINT_IMAGE.
// {chunks: false} leaves out the per-chunk messages.
// ---------------------------------------------------------------------------
export function createWorkerHandler(post, { matrix2d = true, device = 0, previews = false, chunks = true } = {}) {
  return (e) => {
    const m = e && e.data !== undefined ? e.data : e;
    switch (m.type) {
      case WorkerMessageTypes.COMPUTE_GAUSSIAN_SCALE_SPACE: {
        const scaleSpace = computeGaussianScaleSpace({ input_image: m.inputImage, number_of_octaves: m.numberOfOctaves,
          scales_per_octave: m.scalesPerOctave, min_blur_level: m.minBlurLevel, assumed_blur: m.assumedBlur,
          chunk_size: m.chunkSize, matrix2d, device });
        if (previews) {  // background.js:136-143 (octave seeds), :194-202 (chunks), :215-222 (planes)
          const chunk = m.chunkSize || 32;
          scaleSpace.forEach((oct, o) => oct.forEach((_, s) => {
            const img = planeImageData(scaleSpace, o, s);
            if (chunks && !(o > 0 && s === 0)) postChunks(post, WorkerMessageTypes.RECEIVED_GAUSSIAN_BLURRED_CHUNK, img, chunk);
            post({ type: WorkerMessageTypes.RECEIVED_GAUSSIAN_BLURRED_IMAGE, imageData: img, octave: o });
          }));
        }
        post({ type: WorkerMessageTypes.RECEIVED_GAUSSIAN_SCALE_SPACE, scaleSpace });
        break;
      }
      case WorkerMessageTypes.COMPUTE_DIFFERENCE_OF_GAUSSIANS: {
        const dog = computeDifferenceOfGaussians(m.scaleSpace, 32, { device, matrix2d });
        if (previews) {  // background.js:303-320 (sigmoid chunks, chunk size 32), :333-339 (sampled planes)
          dog.forEach((oct, o) => oct.forEach((_, s) => {
            if (chunks) {
              postChunks(post, WorkerMessageTypes.RECEIVED_DIFFERENCE_OF_GAUSSIAN_CHUNK,
                planeImageData(dog, o, s, { mode: 'sigmoid', coefficient: 5 }), 32);
            }
            post({ type: WorkerMessageTypes.RECEIVED_DIFFERENCE_OF_GAUSSIAN_IMAGE,
              imageData: planeImageData(dog, o, s, { mode: 'sampled' }), octave: o });
          }));
        }
        post({ type: WorkerMessageTypes.RECEIVED_DIFFERENCE_OF_GAUSSIANS, differenceOfGaussians: dog });
        break;
      }
      case WorkerMessageTypes.FIND_CANDIDATE_KEYPOINTS: {
        const candidateKeypoints = findCandidateKeypoints({ ...m, device, withLowContrast: previews });
        if (previews) {  // background.js:380-429
          const dogs = m.differenceOfGaussians;
          const low = candidateKeypoints.lowContrastKeypoints;
          candidateKeypoints.forEach((oct, o) => oct.forEach((sc, j) => {
            post({ type: WorkerMessageTypes.RECEIVED_CANDIDATE_KEYPOINT_BASE_IMAGE,
              imageData: planeImageData(dogs, o, sc.scaleLevel, { mode: 'sampled' }) });
            for (const x of low[o][j].localExtremas) {
              post({ type: WorkerMessageTypes.RECEIVED_CANDIDATE_KEYPOINT_MARKER, x: x.x, y: x.y, isLowContrast: true });
            }
            for (const x of sc.localExtremas) {
              post({ type: WorkerMessageTypes.RECEIVED_CANDIDATE_KEYPOINT_MARKER, x: x.x, y: x.y, isLowContrast: false });
            }
            post({ type: WorkerMessageTypes.RECEIVED_CANDIDATE_KEYPOINT_IMAGE, octave: o });
          }));
        }
        post({ type: WorkerMessageTypes.RECEIVED_CANDIDATE_KEYPOINTS, candidateKeypoints });
        break;
      }
      case WorkerMessageTypes.REFINE_CANDIDATE_KEYPOINTS:
        post({ type: WorkerMessageTypes.RECEIVED_REFINED_KEYPOINTS,
          refinedKeypoints: refineCandidateKeypoints({ ...m, device }) });
        break;
      default:
        console.log('sift worker received an unknown message:', m);
    }
  };
}

// Hand results back early: every Gaussian / DoG plane of the given scale
// spaces (as computeGaussianScaleSpace / computeDifferenceOfGaussians return
// them) and every typed keypoint field (format 'typed') that lives in one of
// the addon's recycled buffers is detached and its memory returned at once, so
// the next call of the same geometry reads its planes into those (page-locked)
// buffers instead of fresh pages (planes of a 4K pyramid: 2.6 GB per chain).
// Opt-in, for callers that run the chain repeatedly (frames of a video):
// released arrays read as empty afterwards.  Returns the buffers released.
export function release(...results) {
  let n = 0;
  const seen = new Set();
  const visit = (v, depth) => {
    if (!v || typeof v !== 'object' || depth > 4) return;
    if (ArrayBuffer.isView(v)) {
      if (!seen.has(v.buffer)) {
        seen.add(v.buffer);
        if (native.releaseBuffer(v.buffer)) n++;
      }
      return;
    }
    if (Array.isArray(v)) {
      if (v.length && typeof v[0] !== 'object') return;  // a Matrix2D row or a number list
      for (const x of v) visit(x, depth + 1);
      return;
    }
    for (const k of ['image', 'data', 'ints', 'doubles']) if (k in v) visit(v[k], depth + 1);
  };
  for (const r of results) visit(r, 0);
  return n;
}

// The addon's recycled result buffers (>= 1 MiB planes and keypoint
// fields): buffers and bytes held for reuse, buffers and bytes page-locked.
export function poolStats() {
  const [buffers, bytes, pinned, pinnedBytes] = native.poolStats();
  return { buffers, bytes, pinned, pinnedBytes };
}

export const abiVersion = native.abiVersion();
