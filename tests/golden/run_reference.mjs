// Golden-vector generator: drives the UNMODIFIED reference worker
// (/root/reference/background.js) through its message protocol exactly as
// main.js:111-117 -> 239 -> 274 -> 325 chains it, with the browser globals
// it touches replaced by inert shims (postMessage capture, OffscreenCanvas
// stub, console.log muted).  Run only in the build container by
// make_golden.py; outputs raw binary + JSON under the directory given.
//
// usage: node --experimental-loader ./ref_loader.mjs run_reference.mjs \
//          <input.f32> <params.json> <outdir>
import fs from 'fs';
import path from 'path';

const [, , inPath, paramsPath, outDir] = process.argv;
const P = JSON.parse(fs.readFileSync(paramsPath, 'utf8'));
const W = P.width, H = P.height;
const raw = fs.readFileSync(inPath);
const f32 = new Float32Array(raw.buffer, raw.byteOffset, W * H);
const inputImage = [];
for (let y = 0; y < H; y++) {
  const row = [];
  for (let x = 0; x < W; x++) row.push(f32[y * W + x]);
  inputImage.push(row);
}

const captured = [];
globalThis.onmessage = null;
globalThis.postMessage = (m) => captured.push(m);
globalThis.OffscreenCanvas = class {
  constructor(w, h) { this.w = w; this.h = h; }
  getContext() {
    return { createImageData: (w, h) => ({ width: w, height: h, data: new Uint8ClampedArray(w * h * 4) }) };
  }
};
const realLog = console.log;
console.log = () => {};

function lastOf(type) {
  for (let i = captured.length - 1; i >= 0; i--) if (captured[i].type === type) return captured[i];
  return null;
}

function writePlanes(prefix, pyramid) {
  // Each plane as fp64 little-endian, concatenated octave-major.
  // Written plane by plane: a 4K pyramid (2.8 GB) exceeds Node 12's
  // largest Buffer.
  const meta = [];
  const fd = fs.openSync(path.join(outDir, prefix + '.f64'), 'w');
  for (let o = 0; o < pyramid.length; o++) {
    const om = [];
    for (let s = 0; s < pyramid[o].length; s++) {
      const img = pyramid[o][s].image;
      const h = img.length, w = img[0].length;
      const buf = new Float64Array(h * w);
      for (let y = 0; y < h; y++) for (let x = 0; x < w; x++) buf[y * w + x] = img[y][x];
      fs.writeSync(fd, Buffer.from(buf.buffer));
      om.push({ blurLevel: pyramid[o][s].blurLevel, h: h, w: w });
    }
    meta.push(om);
  }
  fs.closeSync(fd);
  return meta;
}

import('/root/reference/background.js').then(() => {
  const T = {};
  const t0 = Date.now();
  globalThis.onmessage({ data: {
    type: 'compute-gaussian-scale-space', inputImage: inputImage,
    numberOfOctaves: P.num_octaves, scalesPerOctave: P.scales_per_octave,
    minBlurLevel: P.min_blur, assumedBlur: P.assumed_blur, chunkSize: 32 } });
  const scaleSpace = lastOf('received-gaussian-scale-space').scaleSpace;
  const t1 = Date.now();
  globalThis.onmessage({ data: { type: 'compute-difference-of-gaussians', scaleSpace: scaleSpace } });
  const dog = lastOf('received-difference-of-gaussians').differenceOfGaussians;
  const t2 = Date.now();
  const nBefore = captured.length;
  globalThis.onmessage({ data: {
    type: 'find-candidate-keypoints', differenceOfGaussians: dog,
    octaveBaseImages: scaleSpace.map(o => o[0].image), scalesPerOctave: P.scales_per_octave } });
  const cands = lastOf('received-candidate-keypoints').candidateKeypoints;
  // low-contrast markers per (octave, scale): each scale starts with a
  // RECEIVED_CANDIDATE_KEYPOINT_BASE_IMAGE message (background.js:392).
  const low = [];
  let cur = -1;
  for (let i = nBefore; i < captured.length; i++) {
    const m = captured[i];
    if (m.type === 'received-candidate-keypoint-base-image') { low.push(0); cur++; }
    else if (m.type === 'received-candidate-keypoint-marker' && m.isLowContrast) low[cur]++;
  }
  const t3 = Date.now();
  let refined = null, refineError = null;
  try {
    globalThis.onmessage({ data: {
      type: 'refine-candidate-keypoints', differenceOfGaussians: dog,
      scalesPerOctave: P.scales_per_octave, numberOfOctaves: P.num_octaves,
      candidateKeypoints: cands, minBlurLevel: P.min_blur,
      minInterpixelDistance: P.min_interpixel_distance } });
    refined = lastOf('received-refined-keypoints').refinedKeypoints;
  } catch (e) {
    refineError = String(e);
  }
  const t4 = Date.now();

  const out = {
    params: P,
    timing_s: { gaussian: (t1 - t0) / 1e3, dog: (t2 - t1) / 1e3, extrema: (t3 - t2) / 1e3, refine: (t4 - t3) / 1e3 },
    gauss_meta: writePlanes('gauss', scaleSpace),
    dog_meta: writePlanes('dog', dog),
    candidates: cands.map(oct => oct.map(sc => ({ scaleLevel: sc.scaleLevel,
      xyv: sc.localExtremas.map(e => [e.x, e.y, e.value]) }))),
    low_contrast_counts: low,
    refined: refined === null ? null : refined.map(k => [k.octave, k.scaleLevel, k.localX, k.localY,
      k.absoluteSigma, k.absoluteX, k.absoluteY, k.interpolatedValue]),
    refine_error: refineError,
  };
  fs.writeFileSync(path.join(outDir, 'out.json'), JSON.stringify(out));
  realLog(JSON.stringify(out.timing_s));
});
