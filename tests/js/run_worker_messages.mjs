// The worker-protocol shim of the JS drop-in (createWorkerHandler with
// previews) driven the way main.js drives the reference worker; records every
// posted message in the format of tests/golden/run_reference_messages.mjs
// for tests/test_js.py to compare with the reference's own stream.
// usage: node run_worker_messages.mjs <input.f32> <params.json> <out.json> <out.u8>
import fs from 'fs';
import * as sift from '../../sift-scale-space-extrema-detection_amd/js/sift.mjs';

const [, , inPath, paramsPath, outJson, outBytes] = process.argv;
const P = JSON.parse(fs.readFileSync(paramsPath, 'utf8'));
const raw = fs.readFileSync(inPath);
const data = new Float32Array(raw.buffer, raw.byteOffset, P.width * P.height);
const image = { width: P.width, height: P.height, data };
const captured = [];
const onmessage = sift.createWorkerHandler(m => captured.push(m), { matrix2d: true, previews: true });
const last = (t) => { for (let i = captured.length - 1; i >= 0; i--) if (captured[i].type === t) return captured[i]; return null; };
onmessage({ data: { type: sift.WorkerMessageTypes.COMPUTE_GAUSSIAN_SCALE_SPACE, inputImage: image,
  numberOfOctaves: P.num_octaves, scalesPerOctave: P.scales_per_octave, minBlurLevel: P.min_blur,
  assumedBlur: P.assumed_blur, chunkSize: P.chunk_size } });
const ss = last('received-gaussian-scale-space').scaleSpace;
onmessage({ data: { type: sift.WorkerMessageTypes.COMPUTE_DIFFERENCE_OF_GAUSSIANS, scaleSpace: ss } });
const dd = last('received-difference-of-gaussians').differenceOfGaussians;
onmessage({ data: { type: sift.WorkerMessageTypes.FIND_CANDIDATE_KEYPOINTS, differenceOfGaussians: dd,
  octaveBaseImages: ss.map(o => o[0].image), scalesPerOctave: P.scales_per_octave } });
const cc = last('received-candidate-keypoints').candidateKeypoints;
onmessage({ data: { type: sift.WorkerMessageTypes.REFINE_CANDIDATE_KEYPOINTS, differenceOfGaussians: dd,
  scalesPerOctave: P.scales_per_octave, numberOfOctaves: P.num_octaves, candidateKeypoints: cc,
  minBlurLevel: P.min_blur, minInterpixelDistance: P.min_interpixel_distance } });
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
