// Times the JavaScript drop-in (js/sift.mjs over the N-API addon over
// libsift_hip.so) the way a Node caller of the reference's surface uses it:
// host Float32 ImageData in, keypoints out (src/worker.js:29-98 names).
//   1. detect(): one call, host image in -> keypoint objects out
//   2. detectAsync(): the same on the libuv pool (a Promise per image)
//   3. the four-stage chain of the reference: computeGaussianScaleSpace ->
//      computeDifferenceOfGaussians -> findCandidateKeypoints ->
//      refineCandidateKeypoints, every stage returning its host arrays
// usage: node bench_js.mjs <image.f32> <width> <height> <octaves> <scales> <reps> <out.json>
import fs from 'fs';
import { performance } from 'perf_hooks';
import * as sift from '../../sift-scale-space-extrema-detection_amd/js/sift.mjs';

const [, , inPath, Ws, Hs, Os, Ss, repsS, outPath] = process.argv;
const W = +Ws, H = +Hs, O = +Os, S = +Ss, reps = +repsS;
const raw = fs.readFileSync(inPath);
const data = new Float32Array(raw.buffer, raw.byteOffset, W * H);
const image = { width: W, height: H, data };
const opts = { number_of_octaves: O, scales_per_octave: S, min_blur_level: 0.8, assumed_blur: 0.5 };
const mpix = W * H / 1e6;
async function main() {
const med = (a) => { const b = [...a].sort((x, y) => x - y); return b[b.length >> 1]; };
const out = { width: W, height: H, octaves: O, scales: S, reps, node: process.version, node_flags: process.execArgv };
// Every timed section starts from a collected heap (node --expose-gc): a 4K
// result is 445 K keypoint objects (~40 MB of JS heap), and results a previous
// section still held would turn the next one's collections into full
// mark-sweeps near the heap limit.
const gc = () => { if (global.gc) { global.gc(); global.gc(); } };

// 1. detect (synchronous; the device work is serialised in the call)
gc();
let kp = sift.detect(image, opts);  // warm-up (allocations, code objects)
sift.detect(image, opts);
const wall = [], tm = [];
// (no collection between the warm-up and the timed calls: forced right after
// two calls, it left the keypoint-object loop unoptimised for the whole
// section on the box -- 334 instead of ~15 ms per 4K call)
const nsync = Math.max(3 * reps, 12);  // as many images as the queued rows below
const tsync = performance.now();
for (let i = 0; i < nsync; i++) {
  const t0 = performance.now();
  kp = sift.detect(image, opts);
  wall.push(performance.now() - t0);
  tm.push(sift.lastTimings());
}
const syncMean = (performance.now() - tsync) / nsync;
const pick = (k) => med(tm.map((t) => t[k]));
out.detect = {
  keypoints: kp.length, wall_ms: med(wall), mpix_per_s: mpix / (med(wall) / 1e3),
  // the queued / streamed rows below are totals over their images (collections included): compare them
  // with this mean, not with the median (which leaves out the calls a collection lands in)
  mean_ms: syncMean, mean_mpix_per_s: mpix / (syncMean / 1e3),
  h2d_ms: pick('h2dMs'), gauss_dog_ms: pick('gaussDogMs'), extrema_ms: pick('extremaMs'), refine_ms: pick('refineMs'),
  d2h_ms: pick('d2hMs'),
  what: 'sift.detect(ImageData-shaped Float32 host image) -> keypoint objects; wall = host clock around the call '
    + '(H2D of the image, G+DoG, extrema, refine, D2H of the 48-B records, JS objects); stage times = HIP events',
};
out.detect.host_other_ms = out.detect.wall_ms - (out.detect.h2d_ms + out.detect.gauss_dog_ms + out.detect.extrema_ms
  + out.detect.refine_ms + out.detect.d2h_ms);

// 2. detectAsync: one at a time, then `reps` images queued at once
kp = null;
gc();
const awall = [];
for (let i = 0; i < reps; i++) {
  const t0 = performance.now();
  kp = await sift.detectAsync(image, opts);
  awall.push(performance.now() - t0);
}
const nkA = kp.length;
kp = null;
gc();
const tq = performance.now();
let all = await Promise.all(Array.from({ length: reps }, () => sift.detectAsync(image, opts)));
const qms = performance.now() - tq;
all = null;
out.detectAsync = {
  keypoints: nkA, wall_ms: med(awall), mpix_per_s: mpix / (med(awall) / 1e3),
  queued_images: reps, queued_total_ms: qms, queued_mpix_per_s: reps * mpix / (qms / 1e3),
  d2h_ms: sift.lastTimings().d2hMs,
  what: 'await sift.detectAsync(image): the same call on the libuv pool (keypoint copy on the worker thread); '
    + 'queued: Promise.all over reps images (on the device\'s pool of 3 contexts)',
};

// 2b. the typed result format (no per-keypoint JS objects): synchronous,
// then queued asynchronously on the device's pool of 3 contexts
{
  const topts = { ...opts, format: 'typed' };
  sift.detect(image, topts);
  const tw = [];
  let tk;
  for (let i = 0; i < reps; i++) {
    const t0 = performance.now();
    tk = sift.detect(image, topts);
    tw.push(performance.now() - t0);
  }
  out.detect_typed = {
    keypoints: tk.count, wall_ms: med(tw), mpix_per_s: mpix / (med(tw) / 1e3),
    what: "sift.detect(image, {format: 'typed'}) -> {count, ints, doubles}: the same records without JS objects",
  };
  const nq = Math.max(3 * reps, 12);
  for (const [name, o] of [['detectAsync_typed_queued', { ...topts }],
    ['detectAsync_objects_queued', { ...opts }],
    ['detectAsync_typed_queued_inflight1', { ...topts, inflight: 1 }]]) {
    // warm-up: one untimed loop of the same shape (grows the context pool and
    // the result-buffer pool to their steady-state sizes)
    await Promise.all(Array.from({ length: nq }, () => sift.detectAsync(image, o)));
    gc();
    gc();
    const t0 = performance.now();
    let rs = await Promise.all(Array.from({ length: nq }, () => sift.detectAsync(image, o)));
    const ms = performance.now() - t0;
    const nk0 = rs[0].count !== undefined ? rs[0].count : rs[0].length;
    rs = null;
    out[name] = {
      keypoints: nk0, images: nq, total_ms: ms,
      ms_per_image: ms / nq, mpix_per_s: nq * mpix / (ms / 1e3),
      what: `Promise.all over ${nq} detectAsync(image, ${JSON.stringify({ format: o.format || 'objects', inflight: o.inflight === undefined ? 'default' : o.inflight })})`,
    };
  }
}

// 2c. detectAsync with keypoint objects as a server consumes them: up to 3
// images in flight, each result taken in order and dropped (Promise.all above
// keeps all of them alive at once: the GC then walks every image's 445 K
// objects at each collection)
{
  const nq = Math.max(3 * reps, 12), depth = 3;
  for (let i = 0; i < 3; i++) await sift.detectAsync(image, opts);
  gc();
  const t0 = performance.now();
  const q = [];
  let nkp = 0;
  for (let i = 0; i < nq; i++) {
    q.push(sift.detectAsync(image, opts));
    if (q.length === depth) nkp = (await q.shift()).length;
  }
  while (q.length) nkp = (await q.shift()).length;
  const ms = performance.now() - t0;
  out.detectAsync_objects_stream = {
    keypoints: nkp, images: nq, total_ms: ms, ms_per_image: ms / nq, mpix_per_s: nq * mpix / (ms / 1e3),
    what: `${nq} detectAsync(image) (keypoint objects), ${depth} in flight, each result awaited in order and dropped`,
  };
}

// 3. the reference's four stages on host arrays (ImageData-shaped planes)
const stages = { gauss: [], dog: [], find: [], refine: [] };
let nc = 0, nk = 0;
for (let i = 0; i < Math.max(2, Math.min(reps, 5)); i++) {
  let t0 = performance.now();
  const ss = sift.computeGaussianScaleSpace({ input_image: image, ...opts });
  stages.gauss.push(performance.now() - t0);
  t0 = performance.now();
  const dog = sift.computeDifferenceOfGaussians(ss);
  stages.dog.push(performance.now() - t0);
  t0 = performance.now();
  const cands = sift.findCandidateKeypoints({ differenceOfGaussians: dog, scalesPerOctave: S });
  stages.find.push(performance.now() - t0);
  const ext = sift.lastTimings().extremaMs;
  t0 = performance.now();
  const ref = sift.refineCandidateKeypoints({ differenceOfGaussians: dog, scalesPerOctave: S, numberOfOctaves: O,
    candidateKeypoints: cands, minBlurLevel: 0.8, minInterpixelDistance: 0.5 });
  stages.refine.push(performance.now() - t0);
  nc = 0;
  cands.forEach((oc) => oc.forEach((sc) => { nc += sc.localExtremas.length; }));
  nk = ref.length;
  stages.extrema_device_ms = ext;
}
let planeBytes = 0, dogBytes = 0;
{
  const dims = [];
  for (let o = 0, h = 2 * H, w = 2 * W; o < O; o++, h = Math.ceil(h / 2), w = Math.ceil(w / 2)) dims.push(h * w);
  planeBytes = dims.reduce((a, p) => a + 4 * p * (2 * S + 5), 0);
  dogBytes = dims.reduce((a, p) => a + 4 * p * (S + 2), 0);
}
const sum = med(stages.gauss) + med(stages.dog) + med(stages.find) + med(stages.refine);
out.stages = {
  candidates: nc, keypoints: nk,
  computeGaussianScaleSpace_ms: med(stages.gauss), computeDifferenceOfGaussians_ms: med(stages.dog),
  findCandidateKeypoints_ms: med(stages.find), refineCandidateKeypoints_ms: med(stages.refine),
  extrema_device_ms: stages.extrema_device_ms, total_ms: sum, mpix_per_s: mpix / (sum / 1e3),
  planes_to_host_bytes: planeBytes,
  // the DoG stage is pure plane reads (pyramid resident): sift_get_plane into fresh Float32Arrays
  dog_stage_read_gb_per_s: dogBytes / (med(stages.dog) / 1e3) / 1e9,
  what: 'the reference chain main.js -> worker stages: every Gaussian and DoG plane comes back to the host as an '
    + 'ImageData-shaped Float32Array (the reference returns them), candidates and keypoints as JS objects; '
    + 'the device pyramid stays resident between stages',
};
// 3b. the same chain, each iteration's planes handed back (sift.release)
// before the next: the planes are read into the recycled page-locked buffers
{
  const st2 = { gauss: [], dog: [] };
  const it = Math.max(3, Math.min(reps, 6));
  for (let i = 0; i < it; i++) {
    let t0 = performance.now();
    const ss = sift.computeGaussianScaleSpace({ input_image: image, ...opts });
    const tg = performance.now() - t0;
    t0 = performance.now();
    const dog = sift.computeDifferenceOfGaussians(ss);
    const td = performance.now() - t0;
    const cands = sift.findCandidateKeypoints({ differenceOfGaussians: dog, scalesPerOctave: S });
    sift.refineCandidateKeypoints({ differenceOfGaussians: dog, scalesPerOctave: S, numberOfOctaves: O,
      candidateKeypoints: cands, minBlurLevel: 0.8, minInterpixelDistance: 0.5 });
    if (i > 0) { st2.gauss.push(tg); st2.dog.push(td); }  // the first iteration fills the pool
    sift.release(ss, dog);
  }
  const gaussBytes = planeBytes - dogBytes;
  out.stages_released = {
    computeGaussianScaleSpace_ms: med(st2.gauss), computeDifferenceOfGaussians_ms: med(st2.dog),
    planes_to_host_bytes: planeBytes,
    planes_gb_per_s: planeBytes / ((med(st2.gauss) + med(st2.dog)) / 1e3) / 1e9,
    gauss_stage_gb_per_s: gaussBytes / (med(st2.gauss) / 1e3) / 1e9,
    dog_stage_read_gb_per_s: dogBytes / (med(st2.dog) / 1e3) / 1e9,
    pool: sift.poolStats(),
    what: 'the chain\'s first two stages with the previous iteration\'s planes handed back (sift.release(ss, dog)): '
      + 'every plane is one DMA into a recycled page-locked buffer; medians over the iterations after the first',
  };
}
fs.writeFileSync(outPath, JSON.stringify(out, null, 1));
process.stdout.write(JSON.stringify(out) + '\n');
}
main().catch((e) => { console.error(e); process.exitCode = 1; });
