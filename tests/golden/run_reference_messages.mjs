// Message-stream fixture: drives the UNMODIFIED reference worker
// (/root/reference/background.js) through its four stages as main.js chains
// them (main.js:111-117 -> 239 -> 274 -> 325), with the browser globals it
// touches replaced by inert shims, and records EVERY message it posts: type,
// scalar fields (octave, dx, dy, x, y, isLowContrast) and the ImageData
// bytes.  Run only in the build container by make_messages_golden.py.
//
// usage: node --experimental-loader ./ref_loader.mjs run_reference_messages.mjs \
//          <input.f32> <params.json> <out.json> <out.u8>
import fs from 'fs';

const [, , inPath, paramsPath, outJson, outBytes] = process.argv;
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
console.log = () => {};

function lastOf(type) {
  for (let i = captured.length - 1; i >= 0; i--) if (captured[i].type === type) return captured[i];
  return null;
}

import('/root/reference/background.js').then(() => {
  globalThis.onmessage({ data: {
    type: 'compute-gaussian-scale-space', inputImage: inputImage,
    numberOfOctaves: P.num_octaves, scalesPerOctave: P.scales_per_octave,
    minBlurLevel: P.min_blur, assumedBlur: P.assumed_blur, chunkSize: P.chunk_size } });
  const scaleSpace = lastOf('received-gaussian-scale-space').scaleSpace;
  globalThis.onmessage({ data: { type: 'compute-difference-of-gaussians', scaleSpace: scaleSpace } });
  const dog = lastOf('received-difference-of-gaussians').differenceOfGaussians;
  globalThis.onmessage({ data: {
    type: 'find-candidate-keypoints', differenceOfGaussians: dog,
    octaveBaseImages: scaleSpace.map(o => o[0].image), scalesPerOctave: P.scales_per_octave } });
  const cands = lastOf('received-candidate-keypoints').candidateKeypoints;
  globalThis.onmessage({ data: {
    type: 'refine-candidate-keypoints', differenceOfGaussians: dog, scalesPerOctave: P.scales_per_octave,
    numberOfOctaves: P.num_octaves, candidateKeypoints: cands, minBlurLevel: P.min_blur,
    minInterpixelDistance: P.min_interpixel_distance } });
  const msgs = [];
  const bytes = [];
  let off = 0;
  for (const m of captured) {
    const r = { type: m.type };
    for (const k of ['octave', 'dx', 'dy', 'x', 'y', 'isLowContrast']) if (m[k] !== undefined) r[k] = m[k];
    if (m.imageData) {
      r.w = m.imageData.width;
      r.h = m.imageData.height;
      r.off = off;
      bytes.push(Buffer.from(m.imageData.data.buffer, m.imageData.data.byteOffset, m.imageData.data.length));
      off += m.imageData.data.length;
    }
    if (m.refinedKeypoints) r.n = m.refinedKeypoints.length;
    if (m.candidateKeypoints) r.n = m.candidateKeypoints.reduce((a, o) => a + o.reduce((b, s) => b + s.localExtremas.length, 0), 0);
    msgs.push(r);
  }
  fs.writeFileSync(outJson, JSON.stringify(msgs));
  fs.writeFileSync(outBytes, Buffer.concat(bytes));
});
